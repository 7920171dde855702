"""Pin the oracle: the numpy restatement must reproduce the reference's own outputs (golden vectors
made by oracle/gen_golden.py from /root/reference) before it is trusted as the GPU checker."""
import numpy as np
import pytest

from conftest import load_golden, normwise
from oracle import omega_ref as R
from oracle import signals as S

FS = 48000


@pytest.fixture(scope="module")
def mr():
    return load_golden("mrfft")


@pytest.fixture(scope="module")
def me():
    return load_golden("meters")


def test_fixture_versions(mr):
    assert list(mr["versions"]) == ["2.2.6", "1.15.3"]


@pytest.mark.parametrize("name", ["sine1k_2048", "noise_2048", "triad_4096", "comp_4096",
                                  "silence_4096", "sine50_8192"])
def test_mrfft_default(mr, name):
    x = mr[f"{name}/x"]
    res = R.mrfft_frame(x, R.DEFAULT_CONFIGS, FS)
    assert sorted(res) == list(mr[f"{name}/res"])
    for i in res:
        np.testing.assert_allclose(res[i], mr[f"{name}/mag{i}"], rtol=0, atol=0)
        assert res[i].dtype == np.float32
    raw = R.mrfft_frame(x, R.DEFAULT_CONFIGS, FS, apply_weighting=False)
    for i in raw:
        np.testing.assert_array_equal(raw[i], mr[f"{name}/raw{i}"])
    for T in (512, 1024):
        c, t = R.combine(res, R.DEFAULT_CONFIGS, FS, 20000, T)
        np.testing.assert_allclose(c, mr[f"{name}/comb{T}"], rtol=1e-6, atol=1e-7)
        np.testing.assert_array_equal(t, mr[f"{name}/tgt{T}"])


@pytest.mark.parametrize("k", [0, 1, 2])
def test_mrfft_northstar(mr, k):
    x = mr[f"ns{k}/x"]
    res = R.mrfft_frame(x, R.NORTHSTAR_CONFIGS, FS)
    for i in range(4):
        np.testing.assert_array_equal(res[i], mr[f"ns{k}/mag{i}"])
    c, _ = R.combine(res, R.NORTHSTAR_CONFIGS, FS, 20000, 512)
    np.testing.assert_allclose(c, mr[f"ns{k}/comb512"], rtol=1e-6, atol=1e-7)


def test_mrfft_stream(mr):
    x = mr["stream/x"]
    st = R.MRFFTStream(R.DEFAULT_CONFIGS, FS)
    for c in range(24):
        r = st.process(x[c * 512:(c + 1) * 512])
        assert sum(1 << i for i in r) == mr["stream/resmask"][c]
        comb = R.combine(r, R.DEFAULT_CONFIGS, FS, 20000, 512)[0] if r else np.zeros(512)
        np.testing.assert_allclose(comb, mr["stream/comb512"][c], rtol=1e-6, atol=1e-7)
    for i in r:
        np.testing.assert_array_equal(r[i], mr[f"stream/mag{i}"])


def test_mrfft_small_sizes_oracle():
    """FFTConfig sizes below 512 (256 / 128 / 64 with 512): the oracle against the reference."""
    g = load_golden("mrfft_small")
    cfgs = [R.FFTConfig(*c) for c in ((((20, 2000), 256, 128, 1.5)), (((200, 6000), 128, 64, 1.2)),
                                      (((1000, 12000), 64, 32, 1.0)), (((5000, 20000), 512, 256, 1.5)))]
    for name in ("sine", "noise", "triad"):
        res = R.mrfft_frame(g[f"{name}/x"], cfgs, FS)
        assert sorted(res) == list(g[f"{name}/res"])
        for i in res:
            np.testing.assert_array_equal(res[i], g[f"{name}/mag{i}"])
        c, _ = R.combine(res, cfgs, FS, 20000, 512)
        np.testing.assert_allclose(c, g[f"{name}/comb512"], rtol=1e-6, atol=1e-7)


def test_combine_plan_matches_combine(mr):
    """The host-side interpolation plan the HIP epilogue uses reproduces combine()."""
    x = mr["ns0/x"]
    res = R.mrfft_frame(x, R.NORTHSTAR_CONFIGS, FS)
    plan = R.combine_table(R.NORTHSTAR_CONFIGS, FS, 20000, 512)
    out = np.zeros(512)
    for t, entries in enumerate(plan):
        acc = ws = 0.0
        for (i, j, fr) in entries:
            m = res[i].astype(np.float64)
            v = m[j] if fr == 0.0 else m[j] + fr * (m[j + 1] - m[j])
            w = R.NORTHSTAR_CONFIGS[i].weight
            acc += v * w
            ws += w
        out[t] = acc / ws if ws > 0 else 0.0
    assert normwise(out, mr["ns0/comb512"]) < 1e-6


def test_k_weighting_coeffs(me):
    hp_b, hp_a, sh_b, sh_a = R.k_weighting_coeffs(FS)
    np.testing.assert_array_equal(hp_b, me["coef/hp_b"])
    np.testing.assert_array_equal(hp_a, me["coef/hp_a"])
    np.testing.assert_array_equal(sh_b, me["coef/sh_b"])
    np.testing.assert_array_equal(sh_a, me["coef/sh_a"])


@pytest.mark.parametrize("name", ["comp4800", "square480", "sine2048", "hann2048_f64"])
def test_k_weighting_signal(me, name):
    y = R.apply_k_weighting(me[f"kw/{name}/x"], FS)
    np.testing.assert_allclose(y, me[f"kw/{name}/y"], rtol=1e-12, atol=1e-14)
    assert abs(R.true_peak(me[f"kw/{name}/x"]) - me[f"kw/{name}/tp"]) < 1e-5


@pytest.mark.parametrize("fs", [48000, 44100])
def test_ac_weighting_oracle(fs):
    """A / C weighting (professional_meters.py:74-218): the oracle's cascade against the reference's
    outputs, and the facade's closed-form Butterworth sections against scipy's coefficients."""
    g = load_golden("weighting_ac")
    for name in ("sine2048", "comp4800", "hann2048_f64", "low50_4096", "noise16384", "quiet1024"):
        x = g[f"{fs}/{name}/x"]
        for mode in ("A", "C"):
            np.testing.assert_allclose(R.apply_ac_weighting(x, fs, mode), g[f"{fs}/{name}/{mode}"], rtol=1e-12, atol=1e-14)
    assert not g[f"{fs}/quiet1024/A"].any()  # the RMS gate
    from omega_gpu import professional_meters as P
    nyq = fs / 2
    closed = {"coefA/hp1": P._butter2_highpass(20.598997, fs), "coefA/hp2": P._butter1(107.65265, fs, True),
              "coefA/lp1": P._butter1(737.86223, fs, False),
              "coefA/lp2": P._butter2_lowpass(min(12194.217 / nyq, 0.99) * nyq, fs),
              "coefC/hp": P._butter2_highpass(20.598997, fs), "coefC/lp": P._butter2_lowpass(min(12194.217 / nyq, 0.99) * nyq, fs)}
    for k, (b, a) in closed.items():
        np.testing.assert_allclose(b, g[f"{fs}/{k}/b"], rtol=1e-9, atol=1e-15)
        np.testing.assert_allclose(a, g[f"{fs}/{k}/a"], rtol=1e-9, atol=1e-15)
    for (b, a), k in zip(R.ac_weighting_coeffs(fs, "A"), ("hp1", "hp2", "lp1", "lp2")):
        np.testing.assert_array_equal(b, g[f"{fs}/coefA/{k}/b"])


def test_ac_weighting_lufs_sequence():
    """calculate_lufs with weighting_mode A / C: the oracle's meter state over the reference's frames."""
    g = load_golden("weighting_ac")
    for mode in ("A", "C"):
        st = R.MeterState(FS)
        for f, x in enumerate(g["seq/x"]):
            r = st.update(x, R.lufs_instant(x, FS, mode), R.true_peak(x))
            got = np.array(list(r.values()), np.float64)
            np.testing.assert_allclose(got[:4], g[f"seq/{mode}/agg"][f, :4], rtol=1e-9, atol=1e-9)
            assert abs(got[4] - g[f"seq/{mode}/agg"][f, 4]) < 1e-5  # float32 true peak (scipy's resample), 1 ulp


@pytest.mark.parametrize("name", ["hist4800", "peaks4800", "square480", "noise1000", "prime1021", "smooth4410",
                                  "long9600", "tiny10"])
def test_meters_any_length_oracle(name):
    """Frames of non-power-of-two lengths (the reference meters any chunk, test_enhanced_meters.py:82-135):
    the oracle's LUFS_inst / true peak / aggregates against the reference's outputs."""
    g = load_golden("meters_any")
    fr = g[f"{name}/x"]
    li, tp, agg = R.meter_sequence(fr, FS)
    np.testing.assert_allclose(li, g[f"{name}/lufs_inst"], rtol=0, atol=1e-9)
    np.testing.assert_allclose(tp, g[f"{name}/tp"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(agg[:, :4], g[f"{name}/agg"][:, :4], rtol=0, atol=1e-9)
    np.testing.assert_allclose(R.apply_k_weighting(fr[0], FS), g[f"{name}/kw0"], rtol=1e-12, atol=1e-14)
    for o in (2, 1):
        np.testing.assert_allclose([R.true_peak(x, o) for x in fr], g[f"{name}/tp{o}"], rtol=0, atol=1e-5)


def test_filtfilt_restatement_matches_scipy():
    import scipy.signal as ss
    x = S.noise(3, 3000, 0.3).astype(np.float64)
    for b, a in (R.k_weighting_coeffs(FS)[:2], R.k_weighting_coeffs(FS)[2:]):
        np.testing.assert_allclose(R.filtfilt(b, a, x), ss.filtfilt(b, a, x), rtol=1e-13, atol=1e-15)
        np.testing.assert_allclose(R.lfilter_zi2(b, a), ss.lfilter_zi(b, a), rtol=1e-10)  # 1+a1+a2 ~ 2.5e-5: ill-conditioned


def test_resample_restatement_matches_scipy():
    import scipy.signal as ss
    for n in (480, 1024, 4800):
        x = S.noise(n, n, 0.5)
        np.testing.assert_allclose(R.resample_fft(x, 4 * n), ss.resample(x, 4 * n), rtol=0, atol=2e-6)


@pytest.mark.parametrize("name", ["cfg2L", "sine2048", "low50_4096", "silence", "steps1024", "square1024"])
def test_meter_sequences(me, name):
    li, tp, agg = R.meter_sequence(me[f"{name}/x"], FS)
    np.testing.assert_allclose(li, me[f"{name}/lufs_inst"], rtol=0, atol=1e-9)
    np.testing.assert_allclose(tp, me[f"{name}/tp"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(agg, me[f"{name}/agg"], rtol=0, atol=1e-5)


@pytest.mark.parametrize("name", ["dc09_n1e4", "dc05_n1e3", "dcm07_n3e4", "dc03_sine", "dc09_sine1e3", "dc_step",
                                  "hann_dc05"])
def test_meter_dc_offset_oracle(name):
    """DC-biased frames (tests/golden/meters_dc.npz, the reference's calculate_lufs): the oracle, and
    the identity the batch kernel's float32 scan relies on -- K(x) = K(x - c) for any constant c
    (filtfilt is linear; both sections are high-passes, b sums to 0, and the odd extension and the
    lfilter_zi initial states keep a constant at its steady state, whose response is 0)."""
    g = load_golden("meters_dc")
    fr = S.dc_meter_frames()[name]
    li, tp, agg = R.meter_sequence(fr, FS)
    np.testing.assert_allclose(li, g[f"{name}/lufs_inst"], rtol=0, atol=1e-9)
    np.testing.assert_allclose(tp, g[f"{name}/tp"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(agg[:, :4], g[f"{name}/agg"][:, :4], rtol=0, atol=1e-9)
    for x in fr[:3].astype(np.float64):
        y0 = R.apply_k_weighting(x, FS)
        for c in (np.mean(x), np.float32(np.mean(x)), x[0], 0.37):
            y1 = R.apply_k_weighting(x - c, FS)
            assert np.max(np.abs(y1 - y0)) < 1e-9 * max(1.0, np.max(np.abs(x))), (c, np.max(np.abs(y1 - y0)))


def test_meter_dc_offset_float64_app_form():
    g = load_golden("meters_dc")
    fr64 = S.dc_meter_frames()["dc05_n1e3"].astype(np.float64) * np.hanning(16384)
    li, tp, agg = R.meter_sequence(fr64, FS)
    np.testing.assert_allclose(li, g["hann64_dc05/lufs_inst"], rtol=0, atol=1e-9)
    np.testing.assert_allclose(agg[:, :4], g["hann64_dc05/agg"][:, :4], rtol=0, atol=1e-9)


def test_meter_long_window(me):
    """3700 frames: the 3600-deep integrated deque evicts (professional_meters.py:22)."""
    li, tp, agg = R.meter_sequence(S.level_steps(3700, 512, seed=9), FS)
    np.testing.assert_allclose(li, me["long/lufs_inst"], rtol=0, atol=1e-9)
    np.testing.assert_allclose(agg, me["long/agg"], rtol=0, atol=1e-5)


def test_known_answers(me):
    li, tp, agg = R.meter_sequence(np.zeros((3, 2048), np.float32), FS)
    assert (li == -100).all() and (tp == -100).all()
    assert agg[-1].tolist() == [-100.0, -100.0, -100.0, 0.0, -100.0]


def test_bands(golden):
    g = golden("bands")
    mags = g["mags8192"]
    for nb, fft in ((512, 8192), (768, 4096)):
        s, e, c = R.pipeline_band_table(FS, nb, fft)
        np.testing.assert_array_equal(s, g[f"pipe{nb}_{fft}/starts"])
        np.testing.assert_array_equal(e, g[f"pipe{nb}_{fft}/ends"])
        np.testing.assert_array_equal(c, g[f"pipe{nb}_{fft}/comp"])
        src = mags if fft == 8192 else mags[:, : fft // 2 + 1]
        out = np.stack([R.map_to_bands(m, s, e, c, nb) for m in src])
        np.testing.assert_array_equal(out, g[f"pipe{nb}_{fft}/out"])
        st = np.zeros(nb, np.float32)
        sm = np.stack([R.map_to_bands(m, s, e, c, nb, st) for m in src])
        np.testing.assert_allclose(sm, g[f"pipe{nb}_{fft}/smooth"], rtol=1e-6)
        assert out[:, -1].max() == 0  # only B-1 bands are produced
    for fft, nb in ((2048, 512), (8192, 512)):
        bands = R.mel_band_table(FS, fft, nb)
        np.testing.assert_array_equal(np.array(bands), g[f"mel{fft}_{nb}/bands"])
        comp = R.mel_compensation(FS, fft)
        np.testing.assert_array_equal(comp, g[f"mel{fft}_{nb}/comp"])
        spec = g[f"mel{fft}_{nb}/spec"]
        for key, fn in (("out_comp", lambda s: R.map_spectrum_to_bars(s, bands, comp, nb, True)),
                        ("out_raw", lambda s: R.map_spectrum_to_bars(s, bands, comp, nb, False)),
                        ("out_512in", lambda s: R.map_spectrum_to_bars(s[:512], bands, comp, nb, False))):
            np.testing.assert_allclose(np.stack([fn(s) for s in spec]), g[f"mel{fft}_{nb}/{key}"], rtol=1e-6)


def test_chroma(golden):
    g = golden("chroma")
    st = R.ChromaState()
    out = np.stack([st.compute(m, g["freqs"]) for m in g["mags"]])
    np.testing.assert_allclose(out, g["out"], rtol=1e-10, atol=1e-14)
    a = R.ChromaState().compute(g["a440_mag"], g["freqs"])
    np.testing.assert_allclose(a, g["a440_out"], rtol=1e-10)
    assert int(np.argmax(a)) == 9  # A


@pytest.mark.parametrize("genre", ["metal", "rock", "jazz"])
def test_chroma_genre(golden, genre):
    """compute_chromagram with current_genre metal / rock (per-frame tuning offset: drop D, E, Eb and
    the 30-deep mode with its first-inserted tie break) and jazz (blend 0.5), 16384-point spectra."""
    g = golden("chroma_genre")
    st = R.ChromaState(genre)
    out, offs = [], []
    for m in g["mags"]:
        out.append(st.compute(m, g["freqs"]))
        offs.append(st.offset)
    np.testing.assert_array_equal(offs, g[f"{genre}/offset"])
    np.testing.assert_allclose(np.stack(out), g[f"{genre}/out"], rtol=1e-10, atol=1e-14)
    if genre != "jazz":
        assert set(offs) == {-2, -1}


def test_gpu_accelerated_fft(golden):
    """GPUAcceleratedFFT.compute_fft / compute_multi_resolution_fft (reference CPU branch) against the
    restatement; the reference's first-100-bytes cache returns the first signal's spectrum."""
    g = golden("gpufft")
    for name, w in (("noise_4096_hann", "hann"), ("comp_f64_2048_hamming", "hamming"),
                    ("triad_8192_blackman", "blackman"), ("sine_16384_hann", "hann")):
        mag, cp = R.gpu_fft(g[f"fft/{name}/x"], w)
        np.testing.assert_array_equal(mag, g[f"fft/{name}/mag"])
        np.testing.assert_array_equal(cp, g[f"fft/{name}/complex"])
    np.testing.assert_array_equal(g["cache/mag_b"], g["cache/mag_a"])
    assert not np.array_equal(R.gpu_fft(g["cache/b"])[0], g["cache/mag_b"])
    x = g["multi/x"]
    for k, n in (("bass", 8192), ("mid", 4096), ("high", 1024)):
        chunk = x[-n:] if len(x) >= n else np.pad(x, (0, n - len(x)))
        np.testing.assert_array_equal(R.gpu_fft(chunk)[0], g[f"multi/{k}/magnitude"])
        np.testing.assert_array_equal(np.fft.rfftfreq(n, 1 / 48000), g[f"multi/{k}/freqs"])


def test_batched(golden):
    g = golden("batched")
    for name, n, w in (("app_f64_2048_hann", 2048, "hann"), ("f32_4096_blackman", 4096, "blackman"),
                       ("pad_1000_1024_hamming", 1024, "hamming"), ("trim_20000_16384_hann", 16384, "hann")):
        r = R.batched_fft(g[f"{name}/x"], n, w)
        np.testing.assert_array_equal(r["magnitude"], g[f"{name}/mag"])
        np.testing.assert_array_equal(r["complex"], g[f"{name}/complex"])


# ---- drum-detection features (golden: the reference's detectors themselves) ----

@pytest.mark.parametrize("name", ["drums_1025", "drums_2049"])
def test_drum_features(name):
    g = load_golden("drums")
    mags, ref = g[f"{name}/mags"], g[f"{name}/out"]
    o = R.drum_sequence(mags)
    # golden columns: kick sub/body/click flux, sub/body/click threshold, snare fund/body/snap/rattle flux,
    # spectral centroid (the snare thresholds are not in the reference's return dict)
    np.testing.assert_array_equal(o[:, [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 13]], ref)
    # the kick sub band skips the stream's first frame, so its threshold starts one frame after the click band's
    assert o[9, 5] > 0 and o[9, 3] == 0 and o[10, 3] > 0


POST_CFG = {"default": {}, "vocal_supp_norm": dict(vocal_suppression=0.4, normalization=True),
            "flat": dict(psycho=False, freq_comp=False, smoothing=False)}


@pytest.mark.parametrize("name", sorted(POST_CFG))
def test_app_post(name):
    """The app's own process_audio_spectrum (run on the reference's methods, gen_golden.gen_post) over
    24 frames of one stream: the restatement is bit-exact on spectrum, band values and content type."""
    g = load_golden("app_post")
    s, b, c = R.app_post_sequence(g[f"{name}/combined"], g[f"{name}/freqs"], **POST_CFG[name])
    np.testing.assert_array_equal(s, g[f"{name}/spectrum"])
    np.testing.assert_array_equal(b, g[f"{name}/bands"])
    np.testing.assert_array_equal(c, g[f"{name}/content"])
    assert set(c.tolist()) >= {1, 2}


def test_capture_gate_stereo_interleaved():
    """The reference's gate on an interleaved stereo capture (gen_golden.gen_capture_stereo: chunks of
    512 interleaved samples, one RMS and one state for both channels): the restatement's
    capture_stream_interleaved gives the golden chunks bit for bit, and differs from gating each
    channel on its own."""
    g = load_golden("capture_stereo")
    y = R.capture_stream_interleaved(g["x"], gain=1.0)
    np.testing.assert_array_equal(y.T.reshape(-1), g["out"][:y.size])
    per_channel = np.stack([R.capture_stream(g["x"][:, c], gain=1.0) for c in range(2)])
    assert not np.array_equal(per_channel[:, :y.shape[1]], y)


def post_ema_input(g):
    """post_ema.npz's combined spectra, padded with the zero spectra of the silent tail."""
    c = np.zeros((int(g["n_frames"]), g["combined"].shape[1]), np.float32)
    c[:len(g["combined"])] = g["combined"]
    return c


def test_app_post_ema_through_silence():
    """The reference's own loop (gen_golden.gen_post_ema) over 1000 note frames and 500 silent ones:
    the restatement's band EMA is bit-exact, float64 band arrays on the clamping frames and the decay
    into float32 denormals included."""
    g = load_golden("post_ema")
    s, b, c = R.app_post_sequence(post_ema_input(g), g["freqs"])
    np.testing.assert_array_equal(b, g["bands"])
    np.testing.assert_array_equal(c, g["content"])
    tail = b[-1]
    assert g["band_f64"][:1000].any() and not g["band_f64"][-100:].any()
    assert (tail < 1e-30).all() and (tail > 0).sum() > 400  # still decaying, not 0


def test_app_post_threshold_labels_are_the_references():
    """post_threshold.npz's labels come from the reference's update_content_type
    (gen_golden.gen_post_threshold), and the restatement agrees with them."""
    g = load_golden("post_threshold")
    assert "reference" in str(g["labels_source"])
    np.testing.assert_array_equal([R.app_content_type(x) for x in g["combined"]], g["content"])


def test_capture_gate(golden):
    """The capture noise gate (golden: the reference's own _process_audio_frame, chunk by chunk): the
    gated chunks, the background level (float32 after its first update) and the silence counter."""
    g = golden("capture")
    gate = R.CaptureGate()
    x = g["x"]
    outs, bg, sil = [], [], []
    for k in range(len(x) // 512):
        outs.append(gate.process(x[k * 512:(k + 1) * 512]))
        bg.append(float(gate.background_level))
        sil.append(gate.silence_samples)
    np.testing.assert_array_equal(np.concatenate(outs), g["out"])
    np.testing.assert_array_equal(bg, g["bg"])
    np.testing.assert_array_equal(sil, g["silence"])
    assert type(gate.background_level).__name__ == str(g["bg_type"][0])
    gated = (g["out"].reshape(-1, 512) == 0).all(axis=1) & (x.reshape(-1, 512) != 0).any(axis=1)
    assert gated.sum() >= 15  # chunks the gate zeroed (besides the exact-zero stretch)
    np.testing.assert_array_equal(R.capture_stream(x, gain=4.0), g["out"] * np.float32(4.0))


def test_spectra_batch_matches_per_frame_chain():
    """The whole-batch cfg3 oracle (omega_ref.spectra_batch, used by the GPU full-batch test) equals
    the per-frame chain batched_fft -> map_to_bands / ChromaState().compute frame by frame."""
    x = S.cfg3_batch(24)
    st, en, comp = R.pipeline_band_table(FS, 512, 8192)
    mag, bands, chroma = R.spectra_batch(x, st, en, comp, 512)
    freqs = np.fft.rfftfreq(8192, 1 / FS)
    for f in range(len(x)):
        m = R.batched_fft(x[f], 8192, "hann")["magnitude"].astype(np.float32)
        np.testing.assert_array_equal(mag[f], m)
        np.testing.assert_array_equal(bands[f], R.map_to_bands(m, st, en, comp, 512))
        np.testing.assert_allclose(chroma[f], R.ChromaState().compute(m, freqs), rtol=1e-12, atol=1e-15)
