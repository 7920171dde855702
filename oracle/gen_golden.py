"""Generate golden vectors by importing the reference itself (build container only).

TEST INFRASTRUCTURE ONLY. Run from the repo root:

    PYTHONDONTWRITEBYTECODE=1 python oracle/gen_golden.py

It imports the reference modules from ``/root/reference`` (read-only; hence no bytecode) with a
``pygame`` stub for the two panel modules that import pygame at the top
(professional_meters.py:6, chromagram.py:8) -- no drawing code runs. Nothing of the reference is
copied: only inputs and the reference's outputs are written, as small ``.npz`` files under
``tests/golden/`` together with the numpy/scipy versions used (SURVEY.md §8(c) recipe).
"""
from __future__ import annotations

import os
import sys
import types
from types import SimpleNamespace

import numpy as np
import scipy

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
from oracle import signals as S  # noqa: E402

REF = "/root/reference"
OUT = os.path.join(REPO, "tests", "golden")
FS = 48000
VERSIONS = np.array([np.__version__, scipy.__version__])


def _import_reference():
    sys.dont_write_bytecode = True
    pg = types.ModuleType("pygame")
    pg.font = SimpleNamespace(Font=object)
    pg.Surface = object
    sys.modules.setdefault("pygame", pg)
    sys.path.insert(0, REF)
    from omega4.audio.multi_resolution_fft import MultiResolutionFFT, FFTConfig
    from omega4.panels.professional_meters import ProfessionalMetering
    from omega4.audio.pipeline import AudioProcessingPipeline
    from omega4.audio.audio_config import PipelineConfig
    from omega4.optimization.freq_mapper import PrecomputedFrequencyMapper
    from omega4.panels.chromagram import ChromagramAnalyzer
    from omega4.optimization.batched_fft_processor import BatchedFFTProcessor
    from omega4.analyzers.drum_detection import EnhancedKickDetector, EnhancedSnareDetector
    from omega4.optimization.gpu_accelerated_fft import GPUAcceleratedFFT
    from omega4.audio.capture import AudioCaptureConfig, PipeWireMonitorCapture
    from omega4.panels.vu_meters import VUMetersPanel
    from omega4.analyzers.transient import TransientAnalyzer
    return SimpleNamespace(**locals())


def _mrfft(R, configs=None):
    m = R.MultiResolutionFFT(FS)
    if configs is not None:
        m.configs = [R.FFTConfig(*c) for c in configs]
        m._setup_windows(); m._setup_buffers(); m._setup_frequency_arrays(); m._setup_working_arrays()
    return m


NS = [((20, 200), 16384, 1024, 1.5), ((200, 1000), 8192, 512, 1.2),
      ((1000, 5000), 4096, 256, 1.0), ((5000, 20000), 1024, 256, 1.5)]


def gen_mrfft(R):
    d = {"versions": VERSIONS}
    # default configs, fresh instance per frame, 2048- and 4096-sample chunks
    cases = {"sine1k_2048": S.sine(1000, 0.5, 2048), "noise_2048": S.noise(0, 2048, 0.3),
             "triad_4096": S.triad(4096, 0.3), "comp_4096": S.composite(4096),
             "silence_4096": np.zeros(4096, np.float32), "sine50_8192": S.sine(50, 0.8, 8192)}
    for name, x in cases.items():
        m = _mrfft(R)
        r = m.process_audio_chunk(x)
        d[f"{name}/x"] = x
        d[f"{name}/res"] = np.array(sorted(r.keys()))
        for i, fr in r.items():
            d[f"{name}/mag{i}"] = fr.magnitude
        for T in (512, 1024):
            c, t = m.combine_results_optimized(r, target_bins=T)
            d[f"{name}/comb{T}"] = c
            d[f"{name}/tgt{T}"] = t
        r2 = _mrfft(R).process_audio_chunk(x, apply_weighting=False)
        for i, fr in r2.items():
            d[f"{name}/raw{i}"] = fr.magnitude
    # north-star sizes on cfg2-style frames
    xb = S.cfg2_batch(2)
    for k, x in enumerate([xb[0, 0], xb[1, 1], S.triad(16384, 0.5)]):
        m = _mrfft(R, NS)
        r = m.process_audio_chunk(x)
        d[f"ns{k}/x"] = x
        for i, fr in r.items():
            d[f"ns{k}/mag{i}"] = fr.magnitude
        d[f"ns{k}/comb512"] = m.combine_results_optimized(r, target_bins=512)[0]
    # stream layout: one instance fed 512-sample chunks (CircularBuffer semantics)
    st = np.concatenate([S.sine(440, 0.25, 512 * 24) + S.noise(5, 512 * 24, 0.05)])
    m = _mrfft(R)
    res_sets, combs = [], []
    for c in range(24):
        r = m.process_audio_chunk(st[c * 512:(c + 1) * 512])
        res_sets.append(sum(1 << i for i in r))
        combs.append(m.combine_results_optimized(r, target_bins=512)[0] if r else np.zeros(512, np.float32))
        if c == 23:
            for i, fr in r.items():
                d[f"stream/mag{i}"] = fr.magnitude
    d["stream/x"] = st
    d["stream/resmask"] = np.array(res_sets)
    d["stream/comb512"] = np.array(combs, np.float32)
    np.savez_compressed(os.path.join(OUT, "mrfft.npz"), **d)


def _meter_run(R, frames):
    pm = R.ProfessionalMetering(FS)
    li, tp, agg = [], [], []
    for x in frames:
        w = pm.apply_weighting(x)
        ms = np.mean(w ** 2)
        li.append(-0.691 + 10 * np.log10(ms) if ms > 1e-10 else -100.0)
        tp.append(pm.calculate_true_peak(x))
        r = pm.calculate_lufs(x)
        agg.append([r[k] for k in ("momentary", "short_term", "integrated", "range", "true_peak")])
    return np.array(li), np.array(tp, np.float64), np.array(agg, np.float64)


def gen_meters(R):
    d = {"versions": VERSIONS}
    seqs = {
        "cfg2L": S.cfg2_batch(8)[:, 0],                                  # M = 16384
        "sine2048": (S.sine(997, 0.25, 40 * 2048) + S.noise(11, 40 * 2048, 0.02)).reshape(40, 2048),
        "low50_4096": S.sine(50, 0.5, 6 * 4096).reshape(6, 4096),
        "silence": np.zeros((5, 2048), np.float32),
        "steps1024": S.level_steps(300, 1024),
        "square1024": np.stack([S.square(1024)] * 3),
    }
    for name, fr in seqs.items():
        li, tp, agg = _meter_run(R, fr)
        d[f"{name}/x"] = fr
        d[f"{name}/lufs_inst"], d[f"{name}/tp"], d[f"{name}/agg"] = li, tp, agg
    # long stream past the 3600-frame integrated window: inputs regenerated from signals.level_steps
    li, tp, agg = _meter_run(R, S.level_steps(3700, 512, seed=9))
    d["long/lufs_inst"], d["long/tp"], d["long/agg"] = li, tp, agg
    # the weighting filter output itself and the reference test signals of odd lengths
    pm = R.ProfessionalMetering(FS)
    for name, x in {"comp4800": S.composite(4800), "square480": S.square(480),
                    "sine2048": S.sine(1000, 0.1, 2048), "hann2048_f64": (S.composite(2048) * np.hanning(2048))}.items():
        d[f"kw/{name}/x"] = x
        d[f"kw/{name}/y"] = pm.apply_k_weighting(x)
        d[f"kw/{name}/tp"] = np.float64(pm.calculate_true_peak(x))
    kf = pm.k_weighting_filter
    d["coef/hp_b"], d["coef/hp_a"], d["coef/sh_b"], d["coef/sh_a"] = kf["hp_b"], kf["hp_a"], kf["shelf_b"], kf["shelf_a"]
    np.savez_compressed(os.path.join(OUT, "meters.npz"), **d)


def gen_bands(R):
    d = {"versions": VERSIONS}
    xb = S.cfg3_batch(4)
    mags = np.stack([np.abs(np.fft.rfft(x * np.blackman(8192).astype(np.float32))) for x in xb]).astype(np.float32)
    d["mags8192"] = mags
    for nb, fft in ((512, 8192), (768, 4096)):
        cfg = R.PipelineConfig(num_bands=nb, fft_size=fft, ring_buffer_size=fft * 4)
        p = R.AudioProcessingPipeline(cfg)
        d[f"pipe{nb}_{fft}/starts"] = np.array(p.band_indices["starts"])
        d[f"pipe{nb}_{fft}/ends"] = np.array(p.band_indices["ends"])
        d[f"pipe{nb}_{fft}/comp"] = p.freq_compensation
        src = mags if fft == 8192 else mags[:, : fft // 2 + 1]
        d[f"pipe{nb}_{fft}/out"] = np.stack([p.map_to_bands(m, apply_smoothing=False) for m in src])
        d[f"pipe{nb}_{fft}/smooth"] = np.stack([p.map_to_bands(m, apply_smoothing=True) for m in src])
    for fft, nb in ((2048, 512), (8192, 512)):
        fm = R.PrecomputedFrequencyMapper(FS, fft, nb)
        d[f"mel{fft}_{nb}/bands"] = np.array(fm.mapping.band_indices)
        d[f"mel{fft}_{nb}/comp"] = fm.mapping.compensation_curve
        spec = mags[:, : fft // 2 + 1]
        d[f"mel{fft}_{nb}/spec"] = spec
        d[f"mel{fft}_{nb}/out_comp"] = np.stack([fm.map_spectrum_to_bars(s, True) for s in spec])
        d[f"mel{fft}_{nb}/out_raw"] = np.stack([fm.map_spectrum_to_bars(s, False) for s in spec])
        d[f"mel{fft}_{nb}/out_512in"] = np.stack([fm.map_spectrum_to_bars(s[:512], False) for s in spec])
    np.savez_compressed(os.path.join(OUT, "bands.npz"), **d)


def gen_chroma(R):
    d = {"versions": VERSIONS}
    xb = S.cfg3_batch(6)
    mags = np.stack([np.abs(np.fft.rfft(x * np.blackman(8192).astype(np.float32))) for x in xb]).astype(np.float32)
    freqs = np.fft.rfftfreq(8192, 1 / FS)
    ca = R.ChromagramAnalyzer(FS)
    d["mags"], d["freqs"] = mags, freqs
    d["out"] = np.stack([ca.compute_chromagram(m, freqs) for m in mags])
    # known answer: a 440 Hz sine gives chroma argmax 9 (A)
    s = np.abs(np.fft.rfft(S.sine(440, 0.5, 8192) * np.blackman(8192).astype(np.float32))).astype(np.float32)
    d["a440_mag"] = s
    d["a440_out"] = R.ChromagramAnalyzer(FS).compute_chromagram(s, freqs)
    np.savez_compressed(os.path.join(OUT, "chroma.npz"), **d)


def metal_frames(n=16384):
    """Blackman-windowed 16384-point magnitude frames of power chords on E2 (standard), Eb2 (half
    step down) and D2 (drop D) bass notes with octave and fifth, a noise frame and a silent frame: the
    tuning detection of chromagram.py:581-639 sees 0 / -1 / -2 and keeps its offset on frames without
    a bass peak."""
    rng = np.random.default_rng(21)
    t = np.arange(n) / FS
    w = np.blackman(n).astype(np.float32)

    def chord(f0):
        x = sum(a * np.sin(2 * np.pi * f0 * m * t) for m, a in ((1, 0.5), (1.5, 0.3), (2, 0.3), (3, 0.15)))
        return (x + 0.01 * rng.standard_normal(n)).astype(np.float32)

    seq = [73.42] * 6 + [82.41] * 3 + [77.78] * 7 + ["noise", "silence"] + [73.42] * 2
    out = []
    for f in seq:
        if f == "noise":
            x = (0.2 * rng.standard_normal(n)).astype(np.float32)
        elif f == "silence":
            x = np.zeros(n, np.float32)
        else:
            x = chord(f)
        out.append(np.abs(np.fft.rfft(x * w)).astype(np.float32))
    return np.stack(out)


def gen_chroma_genre(R):
    """compute_chromagram sequences with current_genre metal / rock (tuning offset per frame) and jazz
    (blend 0.5), 16384-point spectra."""
    d = {"versions": VERSIONS}
    mags = metal_frames()
    freqs = np.fft.rfftfreq(16384, 1 / FS)
    d["mags"], d["freqs"] = mags, freqs
    for genre in ("metal", "rock", "jazz"):
        ca = R.ChromagramAnalyzer(FS)
        ca.current_genre = genre
        outs, offs = [], []
        for m in mags:
            outs.append(ca.compute_chromagram(m, freqs))
            offs.append(ca.transposition_offset)
        d[f"{genre}/out"] = np.stack(outs)
        d[f"{genre}/offset"] = np.array(offs, np.int32)
    np.savez_compressed(os.path.join(OUT, "chroma_genre.npz"), **d)


def gen_gpufft(R):
    """GPUAcceleratedFFT (gpu_accelerated_fft.py, CPU branch: CuPy is absent) -- compute_fft per
    window and input dtype, its first-100-bytes cache, compute_multi_resolution_fft with a zero-padded
    resolution."""
    d = {"versions": VERSIONS}
    g = R.GPUAcceleratedFFT()
    cases = (("noise_4096_hann", S.noise(11, 4096, 0.2), "hann"),
             ("comp_f64_2048_hamming", S.composite(2048).astype(np.float64), "hamming"),
             ("triad_8192_blackman", S.triad(8192, 0.3), "blackman"),
             ("sine_16384_hann", S.sine(997, 0.4, 16384), "hann"))
    for name, x, w in cases:
        mag, cp = g.compute_fft(x, w, return_complex=True)
        d[f"fft/{name}/x"], d[f"fft/{name}/mag"], d[f"fft/{name}/complex"] = x, mag, cp
    # the cache: a second signal with the same first 25 float32 samples returns the first's result
    a = S.noise(12, 4096, 0.2)
    b = a.copy()
    b[100:] = S.noise(13, 4096 - 100, 0.2)
    g2 = R.GPUAcceleratedFFT()
    d["cache/a"], d["cache/b"] = a, b
    d["cache/mag_a"] = g2.compute_fft(a, "hann")[0]
    d["cache/mag_b"] = g2.compute_fft(b, "hann")[0]
    x = S.noise(14, 6000, 0.2)
    res = R.GPUAcceleratedFFT().compute_multi_resolution_fft(x, {"bass": 8192, "mid": 4096, "high": 1024}, "hann")
    d["multi/x"] = x
    for k, v in res.items():
        for f in ("magnitude", "complex", "freqs"):
            d[f"multi/{k}/{f}"] = v[f]
    np.savez_compressed(os.path.join(OUT, "gpufft.npz"), **d)


def capture_signal(n_chunks=240, chunk=512, seed=31):
    """float32 capture chunks: music-level tone + noise, a fade into near-silence held past the 0.25 s
    silence threshold, a noise floor between the gate floor and twice it (the background EMA
    updates), a loud burst, and an exact-zero stretch."""
    rng = np.random.default_rng(seed)
    n = n_chunks * chunk
    t = np.arange(n) / FS
    x = 0.3 * np.sin(2 * np.pi * 220 * t) + 0.02 * rng.standard_normal(n)
    env = np.ones(n)
    env[40 * chunk:50 * chunk] = np.linspace(1, 1e-4, 10 * chunk)
    env[50 * chunk:90 * chunk] = 1e-4
    x[90 * chunk:130 * chunk] = 0.0015 * rng.standard_normal(40 * chunk)
    env[90 * chunk:130 * chunk] = 1
    x[130 * chunk:150 * chunk] *= 3
    x[200 * chunk:220 * chunk] = 0
    return (x * env).astype(np.float32)


def gen_capture(R):
    """PipeWireMonitorCapture._process_audio_frame (capture.py:620-641) chunk by chunk on one capture
    object with the default config (no process is started): outputs, background level and silence
    counter after each chunk."""
    d = {"versions": VERSIONS}
    cap = R.PipeWireMonitorCapture("golden", R.AudioCaptureConfig())
    x = capture_signal()
    outs, bg, sil = [], [], []
    for k in range(len(x) // 512):
        outs.append(np.array(cap._process_audio_frame(x[k * 512:(k + 1) * 512])))
        bg.append(float(cap.background_level))
        sil.append(cap.silence_samples)
    d["x"], d["out"] = x, np.concatenate(outs).astype(np.float32)
    d["bg"], d["silence"] = np.array(bg), np.array(sil, np.int64)
    d["bg_type"] = np.array([type(cap.background_level).__name__])
    np.savez_compressed(os.path.join(OUT, "capture.npz"), **d)


def gen_capture_stereo(R):
    """The same gate with an interleaved stereo capture (AudioCaptureConfig(channels=2)): the capture
    loop reads chunk_size samples of the interleaved stream (capture.py:549-550) -- 256 frames of two
    channels per chunk -- and _process_audio_frame gates each chunk as a whole. The left channel is
    the mono golden's signal, the right one quieter (its own gaps keep the joint RMS up or let it fall).
    Outputs, background level and silence counter after each chunk."""
    d = {"versions": VERSIONS}
    cap = R.PipeWireMonitorCapture("golden", R.AudioCaptureConfig(channels=2))
    left = capture_signal()
    n = len(left) // 2
    rng = np.random.default_rng(23)
    right = (0.3 * left[:n][::-1] + 0.0005 * rng.standard_normal(n)).astype(np.float32)
    right[n // 3: n // 2] = 0.0
    x = np.ascontiguousarray(np.stack([left[:n], right], axis=1))  # [n, 2] interleaved
    flat = x.reshape(-1)
    outs, bg, sil = [], [], []
    for k in range(len(flat) // 512):
        outs.append(np.array(cap._process_audio_frame(flat[k * 512:(k + 1) * 512])))
        bg.append(float(cap.background_level))
        sil.append(cap.silence_samples)
    d["x"], d["out"] = x, np.concatenate(outs).astype(np.float32)
    d["bg"], d["silence"] = np.array(bg), np.array(sil, np.int64)
    np.savez_compressed(os.path.join(OUT, "capture_stereo.npz"), **d)


def vu_frames(n=240, m=2048, seed=41):
    """The app's VU input: Hann-windowed float64 frames (omega4_main.py:1077-1082) of a tone whose level
    steps down (the display falls, the peak holds 2 s and then decays), then a silent stretch."""
    rng = np.random.default_rng(seed)
    t = np.arange(m) / FS
    lv = np.concatenate([np.full(60, 0.5), np.full(60, 0.05), np.full(90, 0.01), np.zeros(30)])[:n]
    return np.stack([(a * np.sin(2 * np.pi * 440 * t + 0.1 * k) + a * 0.1 * rng.standard_normal(m)) * np.hanning(m)
                     for k, a in enumerate(lv)])


def gen_vu(R):
    """VUMetersPanel.update over 240 display frames (float64 windowed input, dt = 1/60) and then 40 float32
    512-sample chunks with varying dt: the level, display and peak after every call."""
    d = {"versions": VERSIONS}
    vp = R.VUMetersPanel(FS)
    x64 = vu_frames()
    x32 = (0.3 * np.random.default_rng(42).standard_normal((40, 512))).astype(np.float32)
    dt32 = np.random.default_rng(43).uniform(0.005, 0.05, 40)
    rec = []
    for fr in x64:
        vp.update(fr, 1 / 60)
        rec.append((vp.vu_left_db, vp.vu_left_display, vp.vu_left_peak_db, vp.vu_right_db))
    for fr, dt in zip(x32, dt32):
        vp.update(fr, float(dt))
        rec.append((vp.vu_left_db, vp.vu_left_display, vp.vu_left_peak_db, vp.vu_right_db))
    d["x64"], d["x32"], d["dt32"] = x64, x32, dt32
    d["out"] = np.array(rec, np.float64)
    np.savez_compressed(os.path.join(OUT, "vu.npz"), **d)


def transient_frames(seed=51):
    """Drum-like frames: decaying clicks and tone bursts at varying positions and sharpness over a noise
    floor -- float64 Hann-windowed 2048-sample frames (the app's input, omega4_main.py:1241) and raw
    float32 1024-sample frames."""
    rng = np.random.default_rng(seed)
    out64, out32 = [], []
    for k in range(24):
        m = 2048
        t = np.arange(m) / FS
        x = 0.01 * rng.standard_normal(m)
        for _ in range(1 + k % 4):
            p0 = int(rng.integers(50, m - 200))
            tau = rng.uniform(0.0005, 0.01)
            f0 = rng.uniform(50, 3000)
            env = np.where(t >= t[p0], np.exp(-(t - t[p0]) / tau), 0.0)
            x += rng.uniform(0.2, 0.9) * env * np.sin(2 * np.pi * f0 * (t - t[p0]))
        out64.append(x * np.hanning(m))
    for k in range(12):
        m = 1024
        x = (0.02 * rng.standard_normal(m)).astype(np.float32)
        p0 = int(rng.integers(30, m - 100))
        x[p0:p0 + 60] += (np.linspace(0.8, 0.0, 60) * rng.choice([-1, 1], 60)).astype(np.float32)
        out32.append(x)
    return np.stack(out64), np.stack(out32)


def gen_transients(R):
    """TransientAnalyzer.analyze_transients over one analyzer (its envelope history carries over): the
    returned dicts for float64 2048-sample and float32 1024-sample frames and a 40-sample frame."""
    d = {"versions": VERSIONS}
    ta = R.TransientAnalyzer(FS)
    x64, x32 = transient_frames()
    keys = ("transients_detected", "attack_time", "punch_factor", "envelope_peak", "envelope_rms")
    rec = []
    for fr in list(x64) + list(x32):
        r = ta.analyze_transients(fr)
        rec.append([float(r.get(k, np.nan)) for k in keys])
    short = ta.analyze_transients(np.ones(40))
    d["x64"], d["x32"], d["out"] = x64, x32, np.array(rec)
    d["history"] = np.array(ta.get_envelope_history())
    d["short"] = np.array([short["transients_detected"], short["attack_time"], short["punch_factor"]])
    np.savez_compressed(os.path.join(OUT, "transients.npz"), **d)


def gen_weighting_ac(R):
    """apply_a_weighting / apply_c_weighting outputs and calculate_lufs sequences with
    weighting_mode 'A' and 'C' (professional_meters.py:155-229), at 48 kHz and 44.1 kHz."""
    d = {"versions": VERSIONS}
    sigs = {"sine2048": S.sine(1000, 0.1, 2048), "comp4800": S.composite(4800),
            "hann2048_f64": S.composite(2048) * np.hanning(2048), "low50_4096": S.sine(50, 0.5, 4096),
            "noise16384": S.noise(12, 16384, 0.2), "quiet1024": S.sine(440, 5e-7, 1024)}
    for fs in (48000, 44100):
        pm = R.ProfessionalMetering(fs)
        for name, x in sigs.items():
            d[f"{fs}/{name}/x"] = x
            d[f"{fs}/{name}/A"] = pm.apply_a_weighting(x)
            d[f"{fs}/{name}/C"] = pm.apply_c_weighting(x)
        for k in ("hp1", "hp2", "lp1", "lp2"):
            d[f"{fs}/coefA/{k}/b"], d[f"{fs}/coefA/{k}/a"] = pm.a_weighting_filter[k]
        for k in ("hp", "lp"):
            d[f"{fs}/coefC/{k}/b"], d[f"{fs}/coefC/{k}/a"] = pm.c_weighting_filter[k]
    frames = (S.sine(997, 0.25, 30 * 2048) + S.noise(13, 30 * 2048, 0.02)).reshape(30, 2048)
    d["seq/x"] = frames
    for mode in ("A", "C"):
        pm = R.ProfessionalMetering(FS)
        pm.weighting_mode = mode
        agg = []
        for x in frames:
            r = pm.calculate_lufs(x)
            agg.append([r[k] for k in ("momentary", "short_term", "integrated", "range", "true_peak")])
        d[f"seq/{mode}/agg"] = np.array(agg, np.float64)
    np.savez_compressed(os.path.join(OUT, "weighting_ac.npz"), **d)


SMALL = [((20, 2000), 256, 128, 1.5), ((200, 6000), 128, 64, 1.2), ((1000, 12000), 64, 32, 1.0),
         ((5000, 20000), 512, 256, 1.5)]


def gen_mrfft_small(R):
    """FFTConfig sizes below 512 (any power of two is valid, multi_resolution_fft.py:39): a fresh
    MultiResolutionFFT per 512-sample frame, magnitudes and combine(512)."""
    d = {"versions": VERSIONS}
    frames = {"sine": S.sine(1000, 0.3, 512) + S.noise(31, 512, 0.01), "noise": S.noise(32, 512, 0.2),
              "triad": S.triad(512)}
    for name, x in frames.items():
        m = _mrfft(R, SMALL)
        res = m.process_audio_chunk(x)
        d[f"{name}/x"] = x
        d[f"{name}/res"] = np.array(sorted(res))
        for i, fr in res.items():
            d[f"{name}/mag{i}"] = fr.magnitude
        d[f"{name}/comb512"] = m.combine_results_optimized(res, target_bins=512)[0]
    np.savez_compressed(os.path.join(OUT, "mrfft_small.npz"), **d)


def meters_any_seqs():
    """Frames of lengths the power-of-two kernels do not take: the reference's own level-histogram and
    peak-hold signals (test_enhanced_meters.py:82-135: 100 ms = 4800-sample float64 chunks), odd, prime
    and 7-smooth lengths, and 200 ms frames (9600: above the LDS-resident transform size)."""
    hist = []
    for db in [-40, -30, -23, -20, -14, -10, -23, -23, -23]:
        sig = 10 ** (db / 20) * np.sin(2 * np.pi * 1000 * np.linspace(0, 0.1, 4800))
        hist += [sig] * 10
    peaks = []
    for db in [-6, -3, -1, -10]:
        sig = np.zeros(4800)
        sig[2400:2500] = 10 ** (db / 20)
        peaks.append(sig)
    rng = np.random.default_rng(17)
    peaks += [0.001 * rng.standard_normal(4800) for _ in range(6)]
    return {
        "hist4800": np.stack(hist),
        "peaks4800": np.stack(peaks),
        "square480": np.stack([S.square(480)] * 3),
        "noise1000": S.noise(21, 12 * 1000, 0.1).reshape(12, 1000),
        "prime1021": (S.sine(440, 0.3, 6 * 1021) + S.noise(22, 6 * 1021, 0.02)).reshape(6, 1021),
        "smooth4410": (S.sine(3000, 0.2, 5 * 4410) + S.noise(23, 5 * 4410, 0.05)).reshape(5, 4410),
        "long9600": (S.sine(60, 0.5, 4 * 9600) + S.noise(24, 4 * 9600, 0.05)).reshape(4, 9600),
        "tiny10": S.noise(25, 4 * 10, 0.3).reshape(4, 10),
    }


def gen_meters_any(R):
    d = {"versions": VERSIONS}
    for name, fr in meters_any_seqs().items():
        li, tp, agg = _meter_run(R, fr)
        d[f"{name}/x"] = fr
        d[f"{name}/lufs_inst"], d[f"{name}/tp"], d[f"{name}/agg"] = li, tp, agg
        pm = R.ProfessionalMetering(FS)
        d[f"{name}/kw0"] = pm.apply_k_weighting(fr[0])
        d[f"{name}/tp2"] = np.array([pm.calculate_true_peak(x, 2) for x in fr], np.float64)
        d[f"{name}/tp1"] = np.array([pm.calculate_true_peak(x, 1) for x in fr], np.float64)
    np.savez_compressed(os.path.join(OUT, "meters_any.npz"), **d)


def gen_transients_any(R):
    """analyze_transients on frames of lengths that are not powers of two (the reference takes any
    length >= 64): 100 ms float64 chunks (4800), float32 1000 / 100, a prime (1021) and 9600 samples,
    one analyzer per length group (its envelope history carries over)."""
    d = {"versions": VERSIONS}
    x64, x32 = transient_frames(seed=77)
    rng = np.random.default_rng(78)
    groups = {
        "f64_4800": np.stack([np.resize(x64[k], 4800) * np.hanning(4800) for k in range(6)]),
        "f32_1000": np.stack([x32[k][:1000] for k in range(5)]),
        "f64_1021": np.stack([np.resize(x64[k], 1021) for k in range(4)]),
        "f64_9600": np.stack([np.resize(x64[k], 9600) + 0.001 * rng.standard_normal(9600) for k in range(3)]),
        "f32_100": np.stack([x32[k][:100] for k in range(4)]),
        "zeros_3000": np.zeros((1, 3000)),
    }
    keys = ("transients_detected", "attack_time", "punch_factor", "envelope_peak", "envelope_rms")
    for name, fr in groups.items():
        ta = R.TransientAnalyzer(FS)
        rec = []
        for x in fr:
            r = ta.analyze_transients(x)
            rec.append([float(r.get(k, np.nan)) for k in keys])
        d[f"{name}/x"] = fr
        d[f"{name}/out"] = np.array(rec)
        d[f"{name}/history"] = np.array(ta.get_envelope_history())
    np.savez_compressed(os.path.join(OUT, "transients_any.npz"), **d)


def gen_batched(R):
    d = {"versions": VERSIONS}
    bp = R.BatchedFFTProcessor()
    reqs = []
    x64 = S.composite(2048).astype(np.float64) * np.hanning(2048)  # app path: double Hann
    for name, x, n, w in (("app_f64_2048_hann", x64, 2048, "hann"), ("f32_4096_blackman", S.noise(2, 4096, 0.1), 4096, "blackman"),
                          ("pad_1000_1024_hamming", S.sine(440, 0.3, 1000), 1024, "hamming"),
                          ("trim_20000_16384_hann", S.noise(4, 20000, 0.1), 16384, "hann")):
        rid = bp.prepare_batch(name, x, n, w)
        reqs.append((name, rid, x, n, w))
    bp.process_batch()
    res = bp.distribute_results()
    for name, rid, x, n, w in reqs:
        d[f"{name}/x"] = x
        d[f"{name}/mag"] = res[rid]["magnitude"]
        d[f"{name}/complex"] = res[rid]["complex"]
    np.savez_compressed(os.path.join(OUT, "batched.npz"), **d)


def drum_signal(n_frames, n_fft=2048, hop=512, seed=7):
    """Hann-windowed magnitude frames of a synthetic drum track: a decaying 55 Hz kick every 8 frames,
    a noise snare (with a 200 Hz body) every 8 frames offset by 4, a quiet noise floor."""
    rng = np.random.default_rng(seed)
    n = n_fft + hop * (n_frames - 1)
    t = np.arange(n) / FS
    x = 0.01 * rng.standard_normal(n)
    for k in range(0, n_frames, 8):
        t0 = k * hop
        d = np.exp(-np.arange(n - t0) / (0.05 * FS))
        x[t0:] += 0.8 * np.sin(2 * np.pi * 55 * t[: n - t0]) * d
        s0 = t0 + 4 * hop
        if s0 < n:
            d2 = np.exp(-np.arange(n - s0) / (0.02 * FS))
            x[s0:] += (0.3 * rng.standard_normal(n - s0) + 0.3 * np.sin(2 * np.pi * 200 * t[: n - s0])) * d2
    w = np.hanning(n_fft)
    return np.stack([np.abs(np.fft.rfft(x[i * hop:i * hop + n_fft] * w)) for i in range(n_frames)]).astype(np.float32)


def gen_drums(R):
    """EnhancedKickDetector / EnhancedSnareDetector run frame by frame on the same magnitudes: the
    fluxes, kick thresholds (the click threshold through the detector's own calculate_adaptive_threshold)
    and the snare spectral centroid. The onset flags read the wall clock and are not recorded."""
    d = {"versions": VERSIONS}
    for name, nf, nfft in (("drums_1025", 40, 2048), ("drums_2049", 24, 4096)):
        mags = drum_signal(nf, nfft)
        kd, sd = R.EnhancedKickDetector(FS), R.EnhancedSnareDetector(FS)
        rows = []
        for m in mags:
            k = kd.detect_kick_onset(m)
            s = sd.detect_snare_onset(m)
            rows.append([k["sub_flux"], k["body_flux"], k["click_flux"], k["sub_threshold"], k["body_threshold"],
                         kd.calculate_adaptive_threshold(kd.click_flux_history),
                         s["fundamental_flux"], s["body_flux"], s["snap_flux"], s["rattle_flux"],
                         s["spectral_centroid"]])
        d[f"{name}/mags"] = mags
        d[f"{name}/out"] = np.array(rows, dtype=np.float64)
    np.savez_compressed(os.path.join(OUT, "drums.npz"), **d)


def _import_app():
    """omega4_main (the app module): it needs a more permissive pygame stub than the panel modules --
    module attributes that are classes whose attributes are classes (type annotations, pygame.Rect)."""
    class _Meta(type):
        def __getattr__(cls, n):
            return _Any

    class _Any(metaclass=_Meta):
        def __init__(self, *a, **k):
            pass

        def __call__(self, *a, **k):
            return _Any()

        def __getattr__(self, n):
            return _Any()

    for n in ("pygame", "pygame.gfxdraw", "pygame.font", "pygame.mixer", "pygame.locals", "pygame.surfarray",
              "pygame.draw"):
        m = types.ModuleType(n)
        m.__getattr__ = lambda name: _Any
        m.__path__ = []
        sys.modules[n] = m
    import omega4_main
    return omega4_main


class _Stop(Exception):
    pass


def _post_app(R, M, A, kw):
    """A stand-in analyzer object with the reference's own post-processing methods bound to it, the
    real MultiResolutionFFT behind a recorder of each frame's combined spectrum and a drum detector
    that stops process_audio_spectrum once spectrum and band values are final (:1069). run(x) feeds
    one FFT_SIZE_BASE frame and returns (combined, spectrum, bands float64, content index)."""
    app = SimpleNamespace()
    for m in ("process_multi_resolution_fft", "update_content_type", "apply_frequency_compensation",
              "auto_adjust_gain", "_create_equal_loudness_curve"):
        setattr(app, m, types.MethodType(getattr(A, m), app))
    mf = R.MultiResolutionFFT(FS)
    rec = []

    class Rec:
        def process_audio_chunk(self, x, apply_weighting=True):
            return mf.process_audio_chunk(x, apply_weighting)

        def combine_results_optimized(self, res, target_bins=1024):
            s, f = mf.combine_results_optimized(res, target_bins)
            rec.append((s.copy(), f.copy()))
            return s, f

    class Drums:
        def process_audio(self, spectrum, bands):
            raise _Stop(spectrum.copy(), np.array(bands, dtype=np.float64))

    prof = SimpleNamespace(profiler=SimpleNamespace(update_audio_latency=lambda *a: None))
    bf = SimpleNamespace(prepare_batch=lambda *a, **k: 0, process_batch=lambda: 0, distribute_results=lambda: {})
    app.__dict__.update(dict(
        bars=512, freqs=np.fft.rfftfreq(M.FFT_SIZE_BASE, 1 / M.SAMPLE_RATE), multi_fft=Rec(),
        psychoacoustic_enabled=True, freq_compensation_enabled=True, normalization_enabled=False,
        smoothing_enabled=True, vocal_suppression=0.0, psycho_bass_boost=1.5, auto_gain_enabled=False,
        voice_active=False, voice_confidence=0, adaptive_allocation_enabled=False,
        current_content_type="instrumental", current_allocation=0.7, performance_profiler=prof,
        batched_fft=bf, transient_events=[], last_transient_time=0.0, drum_detector=Drums(),
        buffer_pos=M.FFT_SIZE_BASE, ring_buffer=np.zeros(M.FFT_SIZE_BASE * 4, np.float32)))
    app.band_indices = R.PrecomputedFrequencyMapper(M.SAMPLE_RATE, M.FFT_SIZE_BASE, 512).mapping.band_indices
    app.equal_loudness_curve = app._create_equal_loudness_curve()
    app.__dict__.update(kw)

    def run(x):
        app.ring_buffer[:M.FFT_SIZE_BASE] = x
        try:
            A.process_audio_spectrum(app)
            raise RuntimeError("process_audio_spectrum returned before drum detection")
        except _Stop as e:
            spec, bands = e.args
        return (rec[-1][0], spec, bands, ("instrumental", "vocal", "bass_heavy").index(app.current_content_type))

    return app, rec, run


def gen_post(R):
    """The app's own per-frame post-processing, run through the reference's methods on a stand-in
    analyzer object: process_audio_spectrum (omega4_main.py:928-1056) calling the real
    process_multi_resolution_fft / update_content_type / apply_frequency_compensation, with the real
    MultiResolutionFFT behind a recorder of its combined spectrum (the input of the GPU path) and a drum
    detector that stops the frame once spectrum and band values are final (:1069)."""
    M = _import_app()
    A = M.ProfessionalLiveAudioAnalyzer
    d = {"versions": VERSIONS}
    rng = np.random.default_rng(11)
    for name, kw in (("default", {}), ("vocal_supp_norm", {"vocal_suppression": 0.4, "normalization_enabled": True}),
                     ("flat", {"psychoacoustic_enabled": False, "freq_compensation_enabled": False,
                               "smoothing_enabled": False})):
        app, rec, run = _post_app(R, M, A, kw)
        t = np.arange(M.FFT_SIZE_BASE) / FS
        comb, spec, bands, content = [], [], [], []
        for i in range(24):
            # alternate bass-heavy, vocal-range and broadband frames so every content branch is taken
            f0 = (55.0, 700.0, 2500.0)[i % 3] * (1 + 0.05 * i)
            x = (0.4 * np.sin(2 * np.pi * f0 * t) + 0.2 * np.sin(2 * np.pi * 3.1 * f0 * t)
                 + 0.02 * (i % 4) * rng.standard_normal(len(t))).astype(np.float32)
            c, s_, b, k = run(x)
            comb.append(c), spec.append(s_), bands.append(b), content.append(k)
        d[f"{name}/combined"] = np.stack(comb).astype(np.float32)
        d[f"{name}/freqs"] = rec[-1][1]
        d[f"{name}/spectrum"] = np.stack(spec)
        d[f"{name}/bands"] = np.stack(bands)
        d[f"{name}/content"] = np.array(content, np.int32)
    np.savez_compressed(os.path.join(OUT, "app_post.npz"), **d)


def gen_post_ema(R):
    """The band EMA through a silence (omega4_main.py:1041-1056), from the reference's own loop: 1000
    frames of a note whose pitch and level drift, every fifth frame broadband noise (the note frames'
    bands clamp to the int 1, so their band arrays are float64; the noise frames' are float32), then 500 silent frames over which every band decays
    towards the smallest float32 denormal. Stores the combined spectra up to the last non-zero one (the
    later ones are zero), the band values of every frame and the content types."""
    M = _import_app()
    A = M.ProfessionalLiveAudioAnalyzer
    app, rec, run = _post_app(R, M, A, {})
    t = np.arange(M.FFT_SIZE_BASE) / FS
    rng = np.random.default_rng(21)
    comb, bands, content, f64 = [], [], [], []
    n_note, n_sil = 1000, 500
    for i in range(n_note + n_sil):
        if i < n_note and i % 5 == 4:  # broadband frames: no band clamps, a float32 band array
            x = (0.2 * rng.standard_normal(M.FFT_SIZE_BASE)).astype(np.float32)
        elif i < n_note:
            f0 = 330.0 * (1 + 0.25 * np.sin(i / 37.0))
            a = 0.3 * (1 + 0.8 * np.sin(i / 11.0) ** 2)
            x = (a * np.sin(2 * np.pi * f0 * t) + 0.3 * a * np.sin(2 * np.pi * 2.02 * f0 * t)).astype(np.float32)
        else:
            x = np.zeros(M.FFT_SIZE_BASE, np.float32)
        c, _, b, k = run(x)
        comb.append(c)
        bands.append(b)
        content.append(k)
        f64.append(app.prev_band_values.dtype == np.float64)
    # the resolutions' ring buffers still hold note samples for a few silent frames: keep the combined
    # spectra up to the last non-zero one (the rest are zero)
    comb = np.stack(comb).astype(np.float32)
    nz = int(np.flatnonzero(comb.any(axis=1))[-1]) + 1
    np.savez_compressed(os.path.join(OUT, "post_ema.npz"), versions=VERSIONS, freqs=rec[-1][1],
                        combined=comb[:nz], n_frames=np.int64(n_note + n_sil), n_silent=np.int64(n_sil),
                        bands=np.stack(bands), content=np.array(content, np.int32),
                        band_f64=np.array(f64, bool))


def gen_post_threshold(R):
    """Content-type labels of tests/golden/post_threshold.npz's frames (combined spectra whose bass
    ratio sits within a few float32 ulps of 0.6; tests/golden/gen_post_threshold.py chose them) from the
    reference's own update_content_type (omega4_main.py:805-840) on the app's float32 spectrum, with
    the psychoacoustic curve off as in the test -- the labels are the reference's, not the oracle's."""
    M = _import_app()
    A = M.ProfessionalLiveAudioAnalyzer
    path = os.path.join(OUT, "post_threshold.npz")
    g = dict(np.load(path))
    app = SimpleNamespace(voice_active=False, voice_confidence=0, adaptive_allocation_enabled=False,
                          current_content_type="instrumental")
    labels = []
    for s in g["combined"]:
        A.update_content_type(app, np.array(s, np.float32), None)
        labels.append(("instrumental", "vocal", "bass_heavy").index(app.current_content_type))
    g["content"] = np.array(labels, np.int32)
    g["versions"] = VERSIONS
    g["labels_source"] = np.array("reference omega4_main.ProfessionalLiveAudioAnalyzer.update_content_type")
    np.savez_compressed(path, **g)


def gen_meters_dc(R):
    """The reference's own calculate_lufs / apply_weighting / calculate_true_peak on DC-offset frames
    (SURVEY §8(a) A6-A9); also the float64 Hann-windowed form the app feeds the panel."""
    d = {"versions": VERSIONS}
    for name, fr in S.dc_meter_frames().items():
        li, tp, agg = _meter_run(R, fr)
        d[f"{name}/lufs_inst"], d[f"{name}/tp"], d[f"{name}/agg"] = li, tp, agg
    h = np.hanning(16384)
    fr64 = S.dc_meter_frames()["dc05_n1e3"].astype(np.float64) * h
    li, tp, agg = _meter_run(R, fr64)
    d["hann64_dc05/lufs_inst"], d["hann64_dc05/tp"], d["hann64_dc05/agg"] = li, tp, agg
    d["hann64_dc05/tp_dtype"] = np.array(str(np.asarray(R.ProfessionalMetering(FS).calculate_true_peak(fr64[0])).dtype))
    d["dc09_n1e4/tp_dtype"] = np.array(str(np.asarray(R.ProfessionalMetering(FS).calculate_true_peak(
        S.dc_meter_frames()["dc09_n1e4"][0])).dtype))
    np.savez_compressed(os.path.join(OUT, "meters_dc.npz"), **d)


if __name__ == "__main__":
    if not os.path.isdir(REF):
        sys.exit("reference not present: golden vectors can only be generated in the build container")
    os.makedirs(OUT, exist_ok=True)
    R = _import_reference()
    for g in [globals()[f"gen_{n}"] for n in (sys.argv[1:] or ("mrfft", "meters", "bands", "chroma", "batched", "drums", "post", "chroma_genre", "gpufft", "capture", "vu", "transients", "weighting_ac", "meters_any", "mrfft_small", "transients_any", "post_ema", "post_threshold", "capture_stereo", "meters_dc"))]:
        g(R)
        print("wrote", g.__name__)
