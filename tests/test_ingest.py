"""the sustained-stream ingest (omega_ingest_*, csrc/ingest.hip) against the
oracle: the capture noise gate (golden: the reference's own _process_audio_frame), input gain, frames
of the gated stream every hop, meters carried across device batches, irregular byte pushes, s16le
input, the drop policy of unpolled results, and cfg5's 96 kHz 8-channel stream past the 3600-frame
integrated window."""
import numpy as np
import pytest

from conftest import load_golden, normwise
from oracle import omega_ref as R
from oracle import signals as S

pytestmark = pytest.mark.gpu
SPEC_TOL, LU_TOL, TP_TOL_DB = 1e-4, 0.1, 0.01


def _pieces(b: bytes, sizes=(1000, 7, 12293, 4096, 3, 65536)):
    i, k = 0, 0
    while i < len(b):
        n = sizes[k % len(sizes)]
        yield b[i:i + n]
        i += n
        k += 1


def _check_frames(out, streams, fs, W, H, frames, C, check_meters=True):
    """Per-frame outputs against the oracle on each channel's analysed stream y_c; meters against the
    oracle's calculate_lufs sequence fed the device's instantaneous values."""
    for c in range(C):
        st = R.MeterState(fs)
        for f in range(len(out["lufs_inst"]) // C):
            cf = f * C + c
            li, tp = float(out["lufs_inst"][cf]), float(out["true_peak_db"][cf])
            if f in frames:
                fr = streams[c][f * H:f * H + W]
                _, comb, rli, rtp = R.full_frame(fr, configs=R.NORTHSTAR_CONFIGS if W == 16384 else
                                                 (R.FFTConfig((20, 20000), W, H, 1.0),), fs=fs,
                                                 target_bins=out["combined"].shape[1])
                if np.max(comb) > 0:
                    assert normwise(out["combined"][cf], comb) < SPEC_TOL, (c, f)
                else:
                    assert not out["combined"][cf].any(), (c, f)
                assert abs(li - rli) < LU_TOL, (c, f, li, rli)
                assert abs(tp - rtp) < TP_TOL_DB, (c, f, tp, rtp)
            if check_meters:
                ref = np.array(list(st.update(np.ones(1), li, tp).values()))
                np.testing.assert_allclose(out["meters"][cf], ref, rtol=0, atol=1e-9)


def test_ingest_golden_capture_gate_mono():
    """The reference-recorded capture signal (fades into gated silence, a noise floor moving the
    background level) pushed as float32le bytes in irregular pieces: every frame of the gated,
    gain-scaled stream against the oracle, meters carried across the 16 device batches."""
    from omega_gpu import Engine, Resolution
    from omega_gpu.ingest import StreamIngest
    g = load_golden("capture")
    x = g["x"]
    W, H = 4096, 512
    eng = Engine([Resolution((20, 20000), W, H, 1.0)], 48000, 20000, target_bins=256, frame_size=W)
    ing = StreamIngest(eng, hop=H, batch_hops=16, ring_slots=3, gain=4.0)
    got = []
    for p in _pieces(x.tobytes()):
        ing.push(p)
        got.append(ing.poll())
    ing.flush()
    got.append(ing.poll(wait=True))
    out = {k: np.concatenate([d[k] for d in got]) for k in got[0]}
    y = R.capture_stream(x, gain=4.0)
    np.testing.assert_array_equal(y, g["out"] * np.float32(4.0))  # (the oracle's gate is the golden one)
    F = (len(y) - W) // H + 1
    assert len(out["lufs_inst"]) == F
    st = ing.stats()
    assert st["frames"] == F and st["dropped_frames"] == 0 and st["bytes_in"] == x.nbytes
    _check_frames(out, [y], 48000, W, H, set(range(F)), 1)
    # gated stretches come out silent: LUFS -100 for frames wholly inside them
    silent = [f for f in range(F) if not y[f * H:f * H + W].any()]
    assert silent and all(out["lufs_inst"][f] == -100.0 for f in silent)


def test_ingest_golden_capture_gate_stereo():
    """The reference-recorded interleaved stereo capture (gen_golden.gen_capture_stereo: the gate reads
    512 interleaved samples at a time, one RMS and one state for both channels) pushed as float32le
    bytes in irregular pieces: the gated stream is the golden one (silent frames exactly where the
    joint gate closed), every frame of both channels against the oracle."""
    from omega_gpu import Engine, Resolution
    from omega_gpu.ingest import StreamIngest
    g = load_golden("capture_stereo")
    x = g["x"]
    W, H = 2048, 512
    eng = Engine([Resolution((20, 20000), W, H, 1.0)], 48000, 20000, target_bins=128, frame_size=W, n_channels=2)
    ing = StreamIngest(eng, hop=H, batch_hops=16, ring_slots=3, gain=4.0)
    got = []
    for p in _pieces(x.tobytes()):
        ing.push(p)
        got.append(ing.poll())
    ing.flush()
    got.append(ing.poll(wait=True))
    out = {k: np.concatenate([d[k] for d in got]) for k in got[0]}
    y = R.capture_stream_interleaved(x, gain=4.0)
    np.testing.assert_array_equal(y.T.reshape(-1), g["out"][:y.size] * np.float32(4.0))
    F = (y.shape[1] - W) // H + 1
    assert len(out["lufs_inst"]) == 2 * F and ing.stats()["dropped_frames"] == 0
    _check_frames(out, [y[0], y[1]], 48000, W, H, set(range(0, F, 3)) | {F - 1}, 2)
    silent = [f for f in range(F) if not y[:, f * H:f * H + W].any()]
    assert silent and all(out["lufs_inst"][2 * f + c] == -100.0 for f in silent for c in range(2))


def test_ingest_s16le_stereo_and_drop_policy():
    """Interleaved s16le stereo (int16 / 32768, one gate over the interleaved chunks), never polled while 8 batches go
    through with room for 3 pending result blocks: the oldest results are dropped and counted, the
    last ones still match the oracle."""
    from omega_gpu import Engine, Resolution
    from omega_gpu.ingest import StreamIngest
    rng = np.random.default_rng(4)
    n, W, H = 8 * 4096, 2048, 512
    planar = np.stack([S.sine(300, 0.3, n) + S.noise(1, n, 0.01), S.sine(1234, 0.2, n) + S.noise(2, n, 0.01)])
    pcm = np.clip(np.round(planar * 32767), -32768, 32767).astype(np.int16)
    pcm[1, 2048:12288] = rng.integers(-20, 20, 10240)  # a near-silent stretch on the right channel
    inter = pcm.T.ravel()
    eng = Engine([Resolution((20, 20000), W, H, 1.0)], 48000, 20000, target_bins=128, frame_size=W, n_channels=2)
    ing = StreamIngest(eng, hop=H, batch_hops=8, ring_slots=2, max_pending_batches=3, gain=2.0,
                       audio_format="s16le")
    for p in _pieces(inter.tobytes()):
        ing.push(p)
    st = ing.stats()
    assert st["batches"] == 8 and st["dropped_frames"] > 0
    out = ing.poll(wait=True)
    dropped = ing.stats()["dropped_frames"]
    streams = R.capture_stream_interleaved(R.s16le_samples(inter.tobytes()).reshape(-1, 2), gain=2.0)
    F = (n - W) // H + 1
    assert dropped + len(out["lufs_inst"]) // 2 == F
    # the surviving frames are the last ones of the stream
    f0 = dropped
    for c in range(2):
        for j in range(0, len(out["lufs_inst"]) // 2, 3):
            f = f0 + j
            _, comb, li, tp = R.full_frame(streams[c][f * H:f * H + W], configs=(R.FFTConfig((20, 20000), W, H, 1.0),),
                                           target_bins=128)
            assert normwise(out["combined"][j * 2 + c], comb) < SPEC_TOL
            assert abs(out["lufs_inst"][j * 2 + c] - li) < LU_TOL
            assert abs(out["true_peak_db"][j * 2 + c] - tp) < TP_TOL_DB


def test_ingest_cfg5_past_integrated_window():
    """BASELINE cfg5: a 96 kHz 8-channel float32le stream pushed in 512-sample interleaved chunks,
    16384-point frames every 1024 samples (north-star resolutions, 4x true peak, K-LUFS at 96 kHz)
    past frame 3600 of every channel: sampled frames against the oracle, the integrated meter and the
    range over the full 3600-frame window against the oracle's calculate_lufs on channels 0 and 7."""
    from omega_gpu import Engine, NORTHSTAR_RESOLUTIONS
    from omega_gpu.ingest import StreamIngest
    fs, C, W, H = 96000, 8, 16384, 1024
    F = 3700
    n = W + H * (F - 1)
    x = S.cfg5_stream(n, C, fs)
    inter = np.ascontiguousarray(x.T)  # [n, C]
    eng = Engine(NORTHSTAR_RESOLUTIONS, fs, 20000, target_bins=512, n_channels=C)
    ing = StreamIngest(eng, hop=H, batch_hops=64, ring_slots=4, gain=1.0)
    got = []
    for i in range(0, n, 512):
        ing.push(inter[i:i + 512])
        if i % (64 * 1024) == 0:
            got.append(ing.poll())
    ing.flush()
    got.append(ing.poll(wait=True))
    out = {k: np.concatenate([d[k] for d in got]) for k in got[0]}
    assert len(out["lufs_inst"]) == F * C and ing.stats()["dropped_frames"] == 0
    streams = R.capture_stream_interleaved(inter, fs=fs, gain=1.0)
    assert all(np.array_equal(streams[c], x[c][:len(streams[c])]) for c in range(C))  # the gate stays open
    sample = {0, 1, 63, 64, 2047, 3599, 3600, F - 1}
    for c in (0, 7):
        sub = {k: v.reshape(F, C, *v.shape[1:])[:, c] for k, v in out.items()}
        _check_frames(sub, [streams[c]], fs, W, H, sample, 1)
    assert np.isfinite(out["meters"]).all()
    m = out["meters"].reshape(F, C, 5)
    assert (m[3600:, :, 2] > -100).all()
