"""numpy/scipy restatement of the reference hot path (the parity oracle).

TEST INFRASTRUCTURE ONLY -- see ``oracle/__init__.py``. The product path (``omega_gpu`` over
``libomega.so``) never imports this module.

Every function restates one reference function in a *stateless frame form*  and
cites the reference ``file:line`` it follows (paths relative to the reference repo root). The
arithmetic lives in numpy.fft (pocketfft) and scipy.signal, exactly as in the reference; both are
third-party dependencies pinned here at numpy 2.2.6 / scipy 1.15.3 (``requirements.txt:3-4`` only
says ``numpy>=1.21``, ``scipy>=1.7``). numpy >= 2 computes a float32 rfft in single precision;
numpy < 2 would promote to float64 -- the golden fixtures record the versions they were made with.
"""
from __future__ import annotations

from collections import deque
from dataclasses import dataclass
from functools import lru_cache
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import scipy.signal as _sig

# ----------------------------------------------------------------------------------------------
# A1: FFTConfig + windows + frequency arrays   (omega4/audio/multi_resolution_fft.py:26-44,
#     :149-154, :171-193, :210-215)
# ----------------------------------------------------------------------------------------------


@dataclass(frozen=True)
class FFTConfig:
    """One resolution: (freq_range, fft_size, hop_size, weight); window is Blackman
    (multi_resolution_fft.py:26-33; validation :35-44 is mirrored by the facade)."""

    freq_range: Tuple[float, float]
    fft_size: int
    hop_size: int
    weight: float
    window: str = "blackman"


# multi_resolution_fft.py:149-154
DEFAULT_CONFIGS: Tuple[FFTConfig, ...] = (
    FFTConfig((20, 200), 4096, 1024, 1.5),
    FFTConfig((200, 1000), 2048, 512, 1.2),
    FFTConfig((1000, 5000), 1024, 256, 1.0),
    FFTConfig((5000, 20000), 1024, 256, 1.5),
)

# BASELINE.json north-star sizes over the same ranges and weights.
NORTHSTAR_CONFIGS: Tuple[FFTConfig, ...] = (
    FFTConfig((20, 200), 16384, 1024, 1.5),
    FFTConfig((200, 1000), 8192, 512, 1.2),
    FFTConfig((1000, 5000), 4096, 256, 1.0),
    FFTConfig((5000, 20000), 1024, 256, 1.5),
)


def _frozen(a):
    a = np.asarray(a)
    a.flags.writeable = False
    return a


# The setup-time constants below are computed once per argument set, as the reference computes them
# once per instance (windows and frequency arrays in MultiResolutionFFT._setup_windows /
# _setup_frequency_arrays, multi_resolution_fft.py:171-215; the filter coefficients in
# ProfessionalMetering.__init__, professional_meters.py:27-33): the per-frame CPU loop then costs what
# the reference's steady state costs (bench.py cpu_baseline). Returned arrays are read-only.
@lru_cache(maxsize=None)
def window_f32(n: int, kind: str = "blackman") -> np.ndarray:
    """np.<window>(n) cast to float32 (multi_resolution_fft.py:177-188; batched_fft_processor.py:91-101)."""
    if kind == "blackman":
        w = np.blackman(n)
    elif kind == "hann":
        w = np.hanning(n)
    elif kind == "hamming":
        w = np.hamming(n)
    else:  # 'rect' / unknown -> ones (batched_fft_processor.py:99-100)
        w = np.ones(n)
    return _frozen(w.astype(np.float32))


@lru_cache(maxsize=None)
def rfft_freqs(n: int, fs: float) -> np.ndarray:
    """np.fft.rfftfreq(n, 1/fs) (multi_resolution_fft.py:215)."""
    return _frozen(np.fft.rfftfreq(n, 1 / fs))


# ----------------------------------------------------------------------------------------------
# A4: psychoacoustic weights   (multi_resolution_fft.py:304-333)
# ----------------------------------------------------------------------------------------------


@lru_cache(maxsize=None)
def psycho_weights(cfg: FFTConfig, fs: float) -> np.ndarray:
    """Per-bin float32 weight table: fill(weight) then compounding products on inclusive masks,
    only inside the inclusive [lo, hi] range (multi_resolution_fft.py:310-326)."""
    freqs = rfft_freqs(cfg.fft_size, fs)
    w = np.ones(cfg.fft_size // 2 + 1, dtype=np.float32)
    w.fill(cfg.weight)
    lo, hi = cfg.freq_range
    rng = (freqs >= lo) & (freqs <= hi)
    w[rng & (freqs >= 60) & (freqs <= 120)] *= 1.8
    w[rng & (freqs >= 200) & (freqs <= 400)] *= 1.4
    w[rng & (freqs >= 2000) & (freqs <= 5000)] *= 1.2
    w[rng & (freqs >= 20) & (freqs <= 80)] *= 1.6
    return _frozen(w)


# ----------------------------------------------------------------------------------------------
# A2 + A3: stateless multi-resolution FFT of one frame   (multi_resolution_fft.py:228-302)
# ----------------------------------------------------------------------------------------------


def mrfft_frame(x: np.ndarray, configs: Sequence[FFTConfig] = DEFAULT_CONFIGS, fs: float = 48000,
                apply_weighting: bool = True) -> Dict[int, np.ndarray]:
    """Magnitudes of a *fresh* MultiResolutionFFT fed one chunk ``x``.

    A fresh CircularBuffer of size >= 2N holds the last min(len, size) samples; ``read_latest(N)``
    returns None until N samples were written (:99-126), so resolution i exists iff len(x) >= N_i
    and then sees the last N_i samples. Per resolution: float32 window
    multiply (:268-269), np.fft.rfft (complex64 for float32 input on numpy >= 2, :272), np.abs
    (:273), weighting (:276-279), fresh copy (:283).
    """
    x = np.asarray(x, dtype=np.float32)  # CircularBuffer is float32 (:55, :60)
    out: Dict[int, np.ndarray] = {}
    for i, cfg in enumerate(configs):
        n = cfg.fft_size
        if len(x) < n:
            continue
        windowed = np.multiply(x[-n:], window_f32(n, cfg.window))
        mag = np.abs(np.fft.rfft(windowed))
        if apply_weighting:
            mag = mag * psycho_weights(cfg, fs)[: len(mag)]
        out[i] = mag.copy()
    return out


class MRFFTStream:
    """Stateful restatement of MultiResolutionFFT's per-resolution CircularBuffers
    (multi_resolution_fft.py:52-133, :195-208) for the stream layout."""

    def __init__(self, configs: Sequence[FFTConfig] = DEFAULT_CONFIGS, fs: float = 48000):
        self.configs = list(configs)
        self.fs = fs
        self.bufs = [np.zeros(0, np.float32) for _ in configs]
        self.sizes = [max(c.fft_size * 2, c.fft_size + c.hop_size) for c in configs]  # :202

    def process(self, chunk: np.ndarray, apply_weighting: bool = True) -> Dict[int, np.ndarray]:
        chunk = np.asarray(chunk, dtype=np.float32)
        if len(chunk) == 0:  # :240-242
            return {}
        out = {}
        for i, cfg in enumerate(self.configs):
            self.bufs[i] = np.concatenate([self.bufs[i], chunk])[-self.sizes[i]:]
            if len(self.bufs[i]) < cfg.fft_size:
                continue
            out.update({i: mrfft_frame(self.bufs[i], [cfg], self.fs, apply_weighting)[0]})
        return out


# ----------------------------------------------------------------------------------------------
# A5: combine onto a linear target grid   (multi_resolution_fft.py:335-408)
# ----------------------------------------------------------------------------------------------


def combine(results: Dict[int, np.ndarray], configs: Sequence[FFTConfig] = DEFAULT_CONFIGS,
            fs: float = 48000, max_freq: float = 20000, target_bins: int = 1024
            ) -> Tuple[np.ndarray, np.ndarray]:
    """Edge-clamped np.interp of each resolution's in-range bins onto linspace(0, max_freq, T),
    weight-summed into float32 accumulators (zeroed pool arrays, array_pool.py:53) and divided
    by the weight sum where it is > 0 (:393-395)."""
    max_freq = min(max_freq, fs / 2)  # :146
    target = np.linspace(0, max_freq, target_bins)
    if not results:  # :347-349
        return np.zeros(target_bins), target
    acc = np.zeros(target_bins, np.float32)
    wsum = np.zeros(target_bins, np.float32)
    for i, mag in results.items():
        cfg = configs[i]
        freqs = rfft_freqs(cfg.fft_size, fs)
        lo, hi = cfg.freq_range
        valid = (freqs >= lo) & (freqs <= hi)
        if not np.any(valid) or valid.sum() < 2:
            continue
        tmask = (target >= lo) & (target <= hi)
        if not np.any(tmask):
            continue
        idx = np.where(tmask)[0]
        interp = np.interp(target[tmask], freqs[valid], mag[valid])
        acc[idx] += interp * cfg.weight
        wsum[idx] += cfg.weight
    ok = wsum > 0
    acc[ok] /= wsum[ok]
    return acc.copy(), target


def combine_table(configs: Sequence[FFTConfig], fs: float, max_freq: float, target_bins: int):
    """The per-target interpolation plan implied by :func:`combine` (host-side precompute the HIP
    epilogue also uses): for each target bin, (resolution, lower bin, fraction) per owner."""
    max_freq = min(max_freq, fs / 2)
    target = np.linspace(0, max_freq, target_bins)
    plan: List[List[Tuple[int, int, float]]] = [[] for _ in range(target_bins)]
    for i, cfg in enumerate(configs):
        freqs = rfft_freqs(cfg.fft_size, fs)
        lo, hi = cfg.freq_range
        vidx = np.where((freqs >= lo) & (freqs <= hi))[0]
        if len(vidx) < 2:
            continue
        vf = freqs[vidx]
        for t in np.where((target >= lo) & (target <= hi))[0]:
            x = target[t]
            if x <= vf[0]:
                plan[t].append((i, int(vidx[0]), 0.0))
            elif x >= vf[-1]:
                plan[t].append((i, int(vidx[-1]), 0.0))
            else:
                j = int(np.searchsorted(vf, x, side="right") - 1)
                plan[t].append((i, int(vidx[j]), float((x - vf[j]) / (vf[j + 1] - vf[j]))))
    return plan


# ----------------------------------------------------------------------------------------------
# A6: K-weighting = 2 x filtfilt + blend   (omega4/panels/professional_meters.py:48-72, :129-153)
# ----------------------------------------------------------------------------------------------


@lru_cache(maxsize=None)
def k_weighting_coeffs(fs: float = 48000):
    """scipy butter(2, 38/nyq, 'high') and iirfilter(2, 1500/nyq, 'high', 'butter')
    (professional_meters.py:50-64). ``shelf_gain`` (:59) is computed but never used."""
    nyq = fs / 2
    hp_b, hp_a = _sig.butter(2, 38 / nyq, btype="high")
    sh_b, sh_a = _sig.iirfilter(2, 1500 / nyq, btype="high", ftype="butter", output="ba")
    return _frozen(hp_b), _frozen(hp_a), _frozen(sh_b), _frozen(sh_a)


def lfilter_zi2(b, a) -> np.ndarray:
    """Closed form of scipy.signal.lfilter_zi for a biquad (solve (I - companion(a).T) zi = B)."""
    b0 = b[0]
    B0 = b[1] - a[1] * b0
    B1 = b[2] - a[2] * b0
    z0 = (B0 + B1) / (1 + a[1] + a[2])
    return np.array([z0, B1 - a[2] * z0])


def odd_ext(x: np.ndarray, n: int) -> np.ndarray:
    """scipy.signal._arraytools.odd_ext along the last axis."""
    left = 2 * x[..., :1] - x[..., n:0:-1]
    right = 2 * x[..., -1:] - x[..., -2:-(n + 2):-1]
    return np.concatenate([left, x, right], axis=-1)


def filtfilt(b, a, x: np.ndarray) -> np.ndarray:
    """scipy.signal.filtfilt(b, a, x) with its defaults (padtype='odd', padlen=3*max(len(a),len(b))
    = 9, method='pad'): DF2T lfilter forward from zi*ext[0], backward from zi*y[-1], then crop."""
    edge = 3 * max(len(a), len(b))
    x = np.asarray(x)
    if x.shape[-1] <= edge:
        raise ValueError("The length of the input vector x must be greater than padlen, which is %d." % edge)
    ext = odd_ext(x, edge).astype(np.float64)  # the extension is formed in the input dtype
    zi = _sig.lfilter_zi(b, a)
    y, _ = _sig.lfilter(b, a, ext, zi=zi * ext[..., :1])
    y, _ = _sig.lfilter(b, a, y[..., ::-1], zi=zi * y[..., -1:])
    return y[..., ::-1][..., edge:-edge]


def apply_k_weighting(x: np.ndarray, fs: float = 48000) -> np.ndarray:
    """professional_meters.py:129-153: RMS gate (< 1e-6 -> zeros), HP38 filtfilt, shelf filtfilt,
    y = f + 0.3 (s - f)."""
    x = np.asarray(x)
    if np.sqrt(np.mean(x ** 2)) < 1e-6:
        return np.zeros_like(x)
    hp_b, hp_a, sh_b, sh_a = k_weighting_coeffs(fs)
    f = filtfilt(hp_b, hp_a, x)
    s = filtfilt(sh_b, sh_a, f)
    return f + (s - f) * 0.3


def ac_weighting_coeffs(fs: float = 48000, mode: str = "A"):
    """professional_meters.py:74-127: A = butter(2, 20.598997, 'high'), butter(1, 107.65265, 'high'),
    butter(1, 737.86223, 'low'), butter(2, min(12194.217 / nyq, 0.99), 'low'); C = the first and last."""
    nyq = fs / 2
    hp1 = _sig.butter(2, 20.598997 / nyq, btype="high")
    lp2 = _sig.butter(2, min(12194.217 / nyq, 0.99), btype="low")
    if mode == "C":
        return [hp1, lp2]
    return [hp1, _sig.butter(1, 107.65265 / nyq, btype="high"), _sig.butter(1, 737.86223 / nyq, btype="low"), lp2]


def apply_ac_weighting(x: np.ndarray, fs: float = 48000, mode: str = "A") -> np.ndarray:
    """professional_meters.py:155-192 (A: cascaded filtfilt, then *= 2.5) and :194-218 (C)."""
    x = np.asarray(x)
    if np.sqrt(np.mean(x ** 2)) < 1e-6:
        return np.zeros_like(x)
    y = x.copy()
    for b, a in ac_weighting_coeffs(fs, mode):
        y = filtfilt(b, a, y)
    if mode == "A":
        y *= 2.5
    return y


def apply_weighting(x: np.ndarray, fs: float = 48000, mode: str = "K") -> np.ndarray:
    """professional_meters.py:220-229."""
    if mode == "K":
        return apply_k_weighting(x, fs)
    if mode in ("A", "C"):
        return apply_ac_weighting(x, fs, mode)
    return np.asarray(x)


def lufs_instant(x: np.ndarray, fs: float = 48000, weighting: str = "K") -> float:
    """professional_meters.py:236-246 (instantaneous part of calculate_lufs)."""
    y = apply_weighting(x, fs, weighting)
    ms = np.mean(y ** 2)
    return float(-0.691 + 10 * np.log10(ms)) if ms > 1e-10 else -100.0


# ----------------------------------------------------------------------------------------------
# A8: true peak by 4x FFT resampling   (professional_meters.py:283-299; scipy.signal.resample)
# ----------------------------------------------------------------------------------------------


def resample_fft(x: np.ndarray, num: int) -> np.ndarray:
    """scipy.signal.resample(x, num) for real 1-D x, no window: rfft, copy bins 0..N//2, halve an
    even-length Nyquist bin when upsampling, irfft(num), scale num/len (dtype follows input)."""
    x = np.asarray(x)
    nx = len(x)
    X = np.fft.rfft(x)
    Y = np.zeros(num // 2 + 1, X.dtype)
    n = min(num, nx)
    Y[: n // 2 + 1] = X[: n // 2 + 1]
    if n % 2 == 0:
        if num < nx:
            Y[n // 2] *= 2.0
        elif nx < num:
            Y[n // 2] *= 0.5
    y = np.fft.irfft(Y, num)
    y *= float(num) / float(nx)
    return y


def true_peak(x: np.ndarray, oversampling: int = 4) -> float:
    """professional_meters.py:283-299: 20*log10(max|resample(x, 4M)|), -100 if peak < 1e-10 or empty."""
    if len(x) == 0:
        return -100.0
    peak = np.max(np.abs(resample_fft(x, len(x) * oversampling)))
    if peak < 1e-10:
        return -100.0
    return 20 * np.log10(peak)


# ----------------------------------------------------------------------------------------------
# A7 + A9: calculate_lufs with its frame-count deques   (professional_meters.py:16-46, :231-281)
# ----------------------------------------------------------------------------------------------


class MeterState:
    """Per-stream state of ProfessionalMetering: 24/180/3600-deep LUFS deques and a 60-deep TP
    deque (professional_meters.py:20-25), gate -70 (:36), current values (:39-45)."""

    def __init__(self, fs: float = 48000):
        self.fs = fs
        self.mom = deque(maxlen=int(0.4 * 60))
        self.short = deque(maxlen=int(3.0 * 60))
        self.integ = deque(maxlen=int(60 * 60))
        self.peaks = deque(maxlen=int(1.0 * 60))
        self.gate = -70.0
        self.current = {"momentary": -100.0, "short_term": -100.0, "integrated": -100.0,
                        "range": 0.0, "true_peak": -100.0}

    def update(self, x: np.ndarray, lufs_inst: Optional[float] = None,
               tp: Optional[float] = None) -> Dict[str, float]:
        """One calculate_lufs call. ``lufs_inst``/``tp`` may be injected (to score aggregates
        against device-computed instantaneous values); otherwise computed from ``x``."""
        if len(x) == 0:  # :233-234
            return self.current
        li = lufs_instant(x, self.fs) if lufs_inst is None else lufs_inst
        self.mom.append(li)
        self.short.append(li)
        self.integ.append(li)
        self.current["momentary"] = np.mean(self.mom)
        self.current["short_term"] = np.mean(self.short)
        gated = [v for v in self.integ if v > self.gate]
        if gated:
            self.current["integrated"] = np.mean(gated)
            self.current["range"] = np.percentile(gated, 95) - np.percentile(gated, 10)
        else:
            self.current["integrated"] = -100.0
            self.current["range"] = 0.0
        self.peaks.append(true_peak(x) if tp is None else tp)
        self.current["true_peak"] = max(self.peaks)
        return self.current


AGG_KEYS = ("momentary", "short_term", "integrated", "range", "true_peak")


def meter_sequence(frames: np.ndarray, fs: float = 48000) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """Run one stream of frames [F, M] through a fresh MeterState; returns (lufs_inst[F], tp[F],
    aggregates[F, 5] in AGG_KEYS order)."""
    st = MeterState(fs)
    li = np.zeros(len(frames))
    tp = np.zeros(len(frames))
    agg = np.zeros((len(frames), 5))
    for f, x in enumerate(frames):
        li[f] = lufs_instant(x, fs)
        tp[f] = true_peak(x)
        d = st.update(x, li[f], tp[f])
        agg[f] = [d[k] for k in AGG_KEYS]
    return li, tp, agg


# ----------------------------------------------------------------------------------------------
# A10: perceptual log/linear bands, max-reduce   (omega4/audio/pipeline.py:145-230, :295-335)
# ----------------------------------------------------------------------------------------------


def pipeline_band_table(fs: float = 48000, num_bands: int = 768, fft_size: int = 4096,
                        min_freq: float = 20.0, max_freq: float = 20000.0,
                        transition: float = 1000.0, low_ratio: float = 0.5):
    """(starts, ends, compensation) of AudioProcessingPipeline (pipeline.py:165-230, :145-163).
    Only num_bands-1 bands exist (len(all_freqs) - 1)."""
    nyq = fs / 2
    width = nyq / (fft_size // 2)
    max_f = min(max_freq, nyq)
    tb = int(num_bands * low_ratio)
    lows = np.logspace(np.log10(min_freq), np.log10(transition), tb)
    highs = np.linspace(transition, max_f, num_bands - tb + 1)[1:]
    allf = np.concatenate([lows, highs])
    starts, ends, fs_, fe_ = [], [], [], []
    for i in range(min(len(allf) - 1, num_bands)):
        a, b = allf[i], allf[i + 1]
        s, e = int(a / width), int(b / width)
        if e <= s:
            e = s + 1
        s = max(0, min(s, fft_size // 2 - 1))
        e = max(s + 1, min(e, fft_size // 2))
        starts.append(s), ends.append(e), fs_.append(a), fe_.append(b)
    centers = (np.array(fs_) + np.array(fe_)) / 2
    comp = np.ones_like(centers)
    comp[centers < 100] = 2.0
    comp[(centers >= 100) & (centers < 250)] = 1.5
    comp[(centers >= 250) & (centers < 1000)] = 1.2
    comp[centers >= 10000] = 1.3
    return np.array(starts), np.array(ends), comp


def map_to_bands(mag: np.ndarray, starts, ends, comp, num_bands: int,
                 smooth_state: Optional[np.ndarray] = None, smoothing: float = 0.7) -> np.ndarray:
    """pipeline.py:295-335: v[i] = max(mag[s:e]) when the band fits, v[:len(comp)] *= comp, then
    optionally s = 0.7 s + 0.3 v (in place on ``smooth_state``)."""
    v = np.zeros(num_bands, np.float32)
    if mag is None or len(mag) == 0:
        return v
    nvalid = min(num_bands, len(starts), len(ends))
    for i in range(nvalid):
        s, e = starts[i], ends[i]
        if s < len(mag) and e <= len(mag):
            v[i] = np.max(mag[s:e])
    v[: len(comp)] *= comp
    if smooth_state is not None:
        smooth_state *= smoothing
        smooth_state += (1 - smoothing) * v
        return smooth_state.copy()
    return v.copy()


# ----------------------------------------------------------------------------------------------
# A11: mel bands, mean-reduce   (omega4/optimization/freq_mapper.py:83-196)
# ----------------------------------------------------------------------------------------------


def mel_band_table(fs: float, fft_size: int, num_bars: int) -> List[Tuple[int, int]]:
    """freq_mapper.py:83-124."""
    width = fs / fft_size
    hz_to_mel = lambda hz: 2595 * np.log10(1 + hz / 700)
    mel_to_hz = lambda mel: 700 * (10 ** (mel / 2595) - 1)
    mel = np.linspace(hz_to_mel(20), hz_to_mel(20000), num_bars + 1)
    fp = [mel_to_hz(m) for m in mel]
    fp[0] = max(20, fp[0])
    fp[-1] = min(20000, fp[-1])
    bands = []
    for i in range(num_bars):
        if i >= len(fp) - 1:
            break
        s, e = int(fp[i] / width), int(fp[i + 1] / width)
        if e <= s:
            e = s + 1
        s = max(0, min(s, fft_size // 2))
        e = max(s + 1, min(e, fft_size // 2 + 1))
        bands.append((s, e))
    return bands


def mel_compensation(fs: float, fft_size: int) -> np.ndarray:
    """freq_mapper.py:146-163 over np.arange(N/2+1) * fs/N (:57-58)."""
    f = np.arange(fft_size // 2 + 1) * (fs / fft_size)
    c = np.ones_like(f)
    for i, fr in enumerate(f):
        if fr > 0:
            if fr < 100:
                c[i] = 1.0 + (100 - fr) / 100 * 0.5
            elif fr < 1000:
                c[i] = 1.0
            elif fr < 4000:
                c[i] = 1.0 + (fr - 1000) / 3000 * 0.3
            else:
                c[i] = 1.3 - (fr - 4000) / 16000 * 0.5
    return c


def map_spectrum_to_bars(spec: np.ndarray, bands, comp: np.ndarray, num_bars: int,
                         apply_compensation: bool = True) -> np.ndarray:
    """freq_mapper.py:165-196: optional per-bin compensation when lengths match, then the band
    mean; stops at the first band whose end runs past the spectrum."""
    out = np.zeros(num_bars, np.float32)
    if apply_compensation and len(spec) == len(comp):
        spec = spec * comp
    for i, (s, e) in enumerate(bands):
        if i >= num_bars or e > len(spec):
            break
        out[i] = np.mean(spec[s:e]) if e > s else (spec[s] if s < len(spec) else 0)
    return out


# ----------------------------------------------------------------------------------------------
# A12: chromagram binning   (omega4/panels/chromagram.py:109-237; genre 'pop', offset 0)
# ----------------------------------------------------------------------------------------------

_GENRE_BLEND = {"metal": 0.7, "rock": 0.7, "jazz": 0.5}


def suppress_harmonics(fft: np.ndarray, freqs: np.ndarray) -> np.ndarray:
    """chromagram.py:161-189: strict local maxima above 0.1*max; for h = 2..5 scale the bin closest
    to h*f (first on ties) by 1/h when it is within 10 Hz."""
    enh = fft.copy()
    thr = np.max(fft) * 0.1
    peaks = [i for i in range(1, len(fft) - 1)
             if fft[i] > fft[i - 1] and fft[i] > fft[i + 1] and fft[i] > thr]
    for p in peaks:
        if p < len(freqs):
            f0 = freqs[p]
            for h in range(2, 6):
                hf = f0 * h
                c = int(np.argmin(np.abs(freqs - hf)))
                if c < len(enh) and abs(freqs[c] - hf) < 10:
                    enh[c] *= 1.0 / h
    return enh


def spectral_weight(f):
    """chromagram.py:191-201."""
    return np.where(f < 100, 0.5, np.where(f < 1000, 1.0, np.where(f < 4000, 0.8, 0.6)))


def chroma_matrix(freqs: np.ndarray, offset: float = 0.0) -> np.ndarray:
    """The constant 12 x K projection of chromagram.py:122-146 (Gaussian over 5 neighbours times the
    spectral weight) for bins with 20 < f < 8000."""
    M = np.zeros((12, len(freqs)))
    sel = np.where((freqs > 20) & (freqs < 8000))[0]
    f = freqs[sel]
    c = (69 + 12 * np.log2(f / 440.0) + offset) % 12
    base = np.floor(c).astype(int)  # int() of a non-negative float
    sw = spectral_weight(f)
    for o in range(-2, 3):
        tgt = (base + o) % 12
        d = np.abs(c - (base + o))
        w = np.exp(-0.5 * (d / 0.5) ** 2) * sw
        np.add.at(M, (tgt, sel), w)
    return M


_TUNING_REFS = ((0, 82.41), (-1, 82.41 * 0.944), (-2, 82.41 * 0.891), (-3, 82.41 * 0.841), (-4, 82.41 * 0.794))


def find_peaks_simple(data: np.ndarray, prominence: float = 0.3) -> List[int]:
    """chromagram.py:641-654: strict interior local maxima above prominence * max."""
    if len(data) < 3:
        return []
    thr = np.max(data) * prominence
    return [i for i in range(1, len(data) - 1) if data[i] > data[i - 1] and data[i] > data[i + 1] and data[i] > thr]


def detect_tuning_offset(fft: np.ndarray, freqs: np.ndarray, history: List[int], current: int) -> int:
    """chromagram.py:581-639: the first peak of the 70-100 Hz bins against the E2 references within
    50 cents (closest wins, 0 if none); the mode of the last 30 detections once there are 5
    (Counter.most_common: first-inserted among equal counts). history is mutated."""
    m = (freqs > 70) & (freqs < 100)
    bass, bf = fft[m], freqs[m]
    if len(bass) == 0:
        return current
    pk = find_peaks_simple(bass, 0.3)
    if not pk:
        return current
    pf = bf[pk[0]]
    best, dmin = 0, float("inf")
    for off, rf in _TUNING_REFS:
        if pf > 0 and rf > 0:
            d = abs(1200 * np.log2(pf / rf))
            if d < dmin and d < 50:
                dmin, best = d, off
    history.append(best)
    if len(history) > 30:
        history.pop(0)
    if len(history) >= 5:
        from collections import Counter
        return Counter(history).most_common(1)[0][0]
    return best


class ChromaState:
    """Per-stream chroma_history (chromagram.py:96) with the genre blend (:215-237) and, for metal /
    rock, the per-frame tuning offset (:111-113, :128-129) -- an integer semitone shift of the pitch
    map."""

    def __init__(self, genre: str = "pop"):
        self.hist = deque(maxlen=8)
        self.genre = genre
        self.offset = 0
        self.tuning_history: List[int] = []

    def compute(self, fft: np.ndarray, freqs: np.ndarray) -> np.ndarray:
        if self.genre.lower() in ("metal", "rock"):
            self.offset = detect_tuning_offset(fft, freqs, self.tuning_history, self.offset)
        enh = suppress_harmonics(np.asarray(fft).copy(), freqs)
        chroma = chroma_matrix(freqs, self.offset) @ enh.astype(np.float64)
        sm = np.array([0.25 * chroma[(i - 1) % 12] + 0.5 * chroma[i] + 0.25 * chroma[(i + 1) % 12]
                       for i in range(12)])
        if np.sum(sm) > 0:
            sm = sm / np.sum(sm)
        self.hist.append(sm.copy())
        if len(self.hist) == 1:
            return self.hist[-1]
        a = _GENRE_BLEND.get(self.genre.lower(), 0.3)
        return self.hist[-2] * (1 - a) + self.hist[-1] * a


def spectra_batch(x: np.ndarray, starts, ends, comp, num_bands: int, fs: float = 48000,
                  window: str = "hann"):
    """cfg3 over a whole batch f32[F, N] at once (test infrastructure: the full-batch parity check),
    the same arithmetic as the per-frame chain batched_fft -> map_to_bands / ChromaState().compute
    (a fresh state per frame, no blend): |rfft(x * window_f32)| (A13, batched_fft_processor.py:269-285),
    the band maxima times the compensation (A10, pipeline.py:295-335), and the chromagram
    (A12, chromagram.py:109-213) with the harmonic suppression applied in the reference's order (peak
    by peak, h = 2..5; on a uniform rfftfreq grid the bin closest to h*f_p is min(h*p, K-1)).
    tests/test_oracle_golden.py pins it against the per-frame oracle. Returns (mag, bands, chroma)."""
    n = x.shape[1]
    mag = np.abs(np.fft.rfft(x * window_f32(n, window), axis=1)).astype(np.float32)
    F, K = mag.shape
    bands = np.zeros((F, num_bands), np.float32)
    for i in range(min(num_bands, len(starts), len(ends))):
        s, e = starts[i], ends[i]
        if s < K and e <= K:
            bands[:, i] = mag[:, s:e].max(axis=1)
    bands[:, :len(comp)] *= comp
    freqs = np.fft.rfftfreq(n, 1 / fs)
    thr = mag.max(axis=1) * np.float32(0.1)
    mid = mag[:, 1:-1]
    pk = (mid > mag[:, :-2]) & (mid > mag[:, 2:]) & (mid > thr[:, None])
    fi, pi = np.nonzero(pk)  # row-major: frame, then peak bin ascending (the reference's loop order)
    pi = pi + 1
    enh = mag.copy()
    hs = np.arange(2, 6)
    hf = freqs[pi][:, None] * hs[None, :]
    c = np.minimum(pi[:, None] * hs[None, :], K - 1)
    ok = np.abs(freqs[c] - hf) < 10
    fac = np.broadcast_to((1.0 / hs).astype(np.float32), c.shape)
    fr = np.broadcast_to(fi[:, None], c.shape)
    np.multiply.at(enh, (fr[ok], c[ok]), fac[ok])  # (ravelled in (peak, h) order; applied in order)
    ch = enh.astype(np.float64) @ chroma_matrix(freqs).T
    sm = 0.25 * np.roll(ch, 1, axis=1) + 0.5 * ch + 0.25 * np.roll(ch, -1, axis=1)
    tot = sm.sum(axis=1, keepdims=True)
    sm = np.where(tot > 0, sm / np.where(tot > 0, tot, 1), sm)
    return mag, bands, sm


# ----------------------------------------------------------------------------------------------
# A13: BatchedFFTProcessor CPU branch   (omega4/optimization/batched_fft_processor.py:119-146,
#      :269-285)
# ----------------------------------------------------------------------------------------------


def gpu_fft(audio: np.ndarray, window_type: str = "hann"):
    """GPUAcceleratedFFT.compute_fft (gpu_accelerated_fft.py:92-177) without its prefix cache:
    audio * window(n).astype(float32) (np.hanning / np.hamming / else np.blackman), rfft, |.|; the
    arithmetic follows the input dtype (the CPU branch; the CuPy branch casts to float32)."""
    n = len(audio)
    w = {"hann": np.hanning, "hamming": np.hamming}.get(window_type, np.blackman)(n).astype(np.float32)
    c = np.fft.rfft(audio * w)
    return np.abs(c), c


def batched_fft(audio: np.ndarray, fft_size: int, window_type: str = "hann", fs: float = 48000):
    """prepare_batch pads/trims to fft_size (:136-139), then window * data, np.fft.rfft, abs;
    frequencies are hard-coded for 48 kHz in the reference (:257)."""
    a = np.asarray(audio)
    if len(a) > fft_size:
        a = a[-fft_size:]
    elif len(a) < fft_size:
        a = np.pad(a, (0, fft_size - len(a)))
    c = np.fft.rfft(a * window_f32(fft_size, window_type))
    return {"magnitude": np.abs(c), "complex": c, "frequencies": np.fft.rfftfreq(fft_size, 1 / 48000)}


# ----------------------------------------------------------------------------------------------
# One BASELINE cfg2 channel-frame, chained as SURVEY.md §8(c)
# ----------------------------------------------------------------------------------------------


def full_frame(x: np.ndarray, configs=NORTHSTAR_CONFIGS, fs=48000, target_bins=512):
    """MRFFT + combine(T) + LUFS_inst + TP for one channel-frame (the per-frame part of cfg2)."""
    res = mrfft_frame(x, configs, fs)
    comb, _ = combine(res, configs, fs, 20000, target_bins)
    return res, comb, lufs_instant(x, fs), true_peak(x)


# ----------------------------------------------------------------------------------------------
# drum-detection spectral features -- band flux, adaptive thresholds and the
# snare spectral centroid (omega4/analyzers/drum_detection.py: EnhancedKickDetector :19-28, :47-103;
# EnhancedSnareDetector :183-194, :212-266, :279-305). The onset decisions themselves read the wall
# clock (time.time(), :82, :270) and are not part of the data-parallel path.
# ----------------------------------------------------------------------------------------------

KICK_BANDS = ((20, 60), (60, 120), (2000, 5000))                       # drum_detection.py:20-22
SNARE_BANDS = ((150, 400), (400, 1000), (2000, 8000), (8000, 15000))   # :183-186
SNARE_MULT = (2.5, 2.3, 2.0)                                           # :295, :300, :305
DRUM_COLUMNS = ("kick_sub_flux", "kick_body_flux", "kick_click_flux",
                "kick_sub_threshold", "kick_body_threshold", "kick_click_threshold",
                "snare_fundamental_flux", "snare_body_flux", "snare_snap_flux", "snare_rattle_flux",
                "snare_fundamental_threshold", "snare_body_threshold", "snare_snap_threshold",
                "snare_centroid")


def drum_band_bins(band, n_bins: int, fs: float = 48000):
    """int(f * len(magnitude) / nyquist) for both edges (:86-96, :240-259)."""
    ny = fs / 2
    return int(band[0] * n_bins / ny), int(band[1] * n_bins / ny)


def adaptive_threshold(hist, mult: float, sensitivity: float = 1.0):
    """median + sensitivity * mult * MAD over the history, 0 below 10 values (:69-78, :290-305)."""
    if len(hist) < 10:
        return 0.0
    a = np.array(list(hist))
    med = np.median(a)
    mad = np.median(np.abs(a - med))
    return med + sensitivity * mult * mad


class DrumFluxState:
    """One stream's kick + snare feature state: previous magnitude frame and the 21-deep flux
    histories, updated per frame exactly as detect_kick_onset / detect_snare_onset do."""

    def __init__(self, fs: float = 48000, sensitivity: float = 1.0):
        self.fs, self.sens = fs, sensitivity
        self.prev_k = None  # EnhancedKickDetector.prev_magnitude
        self.prev_s = None  # EnhancedSnareDetector.prev_magnitude
        self.hk = [deque(maxlen=21) for _ in KICK_BANDS]
        self.hs = [deque(maxlen=21) for _ in SNARE_BANDS]

    def update(self, mag: np.ndarray) -> np.ndarray:
        n = len(mag)
        # kick (:85-103): on the first frame the sub band sets prev and returns 0 WITHOUT appending
        # (:51-53); body and click then see prev == mag and append 0
        kf = []
        for b, band in enumerate(KICK_BANDS):
            s, e = drum_band_bins(band, n, self.fs)
            if self.prev_k is None:
                self.prev_k = mag.copy()
                kf.append(0.0)
                continue
            f = np.sum(np.maximum(mag[s:e] - self.prev_k[s:e], 0))
            self.hk[b].append(f)
            kf.append(f)
        self.prev_k = mag.copy()
        kt = [adaptive_threshold(h, 2.8, self.sens) for h in self.hk]
        # snare (:231-266): zeros on the first frame (prev set), appended by detect_snare_onset
        if self.prev_s is None:
            self.prev_s = mag.copy()
            sf = [0.0] * 4
        else:
            sf = []
            for band in SNARE_BANDS:
                s, e = drum_band_bins(band, n, self.fs)
                sf.append(np.sum(np.maximum(mag[s:e] - self.prev_s[s:e], 0)))
            self.prev_s = mag.copy()
        # spectral centroid (:212-229): frequencies of rfftfreq(2 len - 1), 150 Hz .. 15 kHz
        freqs = np.fft.rfftfreq(n * 2 - 1, 1 / self.fs)
        s, e = int(SNARE_BANDS[0][0] * n / (self.fs / 2)), int(SNARE_BANDS[3][1] * n / (self.fs / 2))
        rel = mag[s:e]
        cen = np.sum(freqs[s:e] * rel) / np.sum(rel) if np.sum(rel) > 0 else 0
        for h, v in zip(self.hs, sf):
            h.append(v)
        st = [0.0] * 3
        if len(self.hs[0]) >= 10:
            st = [adaptive_threshold(self.hs[i], SNARE_MULT[i], self.sens) for i in range(3)]
        return np.array([*kf, *kt, *sf, *st, cen], dtype=np.float64)


def drum_sequence(mags: np.ndarray, fs: float = 48000, sensitivity: float = 1.0) -> np.ndarray:
    """Features of consecutive magnitude frames of one stream: [F, 14] (DRUM_COLUMNS)."""
    st = DrumFluxState(fs, sensitivity)
    return np.stack([st.update(m) for m in mags])


# ---- App spectrum post-processing: omega4_main.ProfessionalLiveAudioAnalyzer,
# FFT_SIZE_BASE = 2048 and bars = 512 there. float32 arrays throughout, in-place multiplies by Python
# scalars (NEP 50 weak scalars -> float32), as the reference runs them.

def app_equal_loudness(fs: float = 48000, fft_base: int = 2048) -> np.ndarray:
    """_create_equal_loudness_curve omega4_main.py:617-644 (float64, indexed by position)."""
    f = np.fft.rfftfreq(fft_base, 1 / fs)[:fft_base // 2 + 1]
    c = np.ones_like(f)
    c[f < 200] = 1 + (200 - f[f < 200]) / 50
    for lo, hi, g in ((500, 2000, 0.85), (2000, 5000, 1.05)):
        c[(f > lo) & (f < hi)] *= g
    c[f > 6000] *= 0.5
    c[f > 10000] *= 0.2
    return c


def app_content_type(s: np.ndarray, fs: float = 48000) -> int:
    """update_content_type :805-840 without voice detection: 0 instrumental, 1 vocal, 2 bass-heavy."""
    n = len(s)
    w = fs / (2 * n)
    be, vs, ve, hs = int(250 / w), int(200 / w), int(4000 / w), int(6000 / w)
    eb = np.mean(s[:be]) if be < n else 0
    ev = np.mean(s[vs:ve]) if ve < n else 0
    eh = np.mean(s[hs:]) if hs < n else 0
    et = np.mean(s)
    if not et > 0:
        return 0
    br, vr = eb / et, ev / et
    if br > 0.6:
        return 2
    if (vr > 0.4 and br < 0.4) or (vr > 0.3 and eh < ev * 0.5):
        return 1
    return 0


def app_compensation(s: np.ndarray, f: np.ndarray, content: int, vocal_suppression: float = 0.0) -> np.ndarray:
    """apply_frequency_compensation :855-926 (freqs = the base FFT's, by position)."""
    out = s.copy()
    first = ((0.15, 0.2, 0.6, 1.5) if content == 1 else (0.8, 1.0, 1.1, 0.85))
    edges = (-np.inf, 60, 250, 500, 2000, 6000, 10000, np.inf)
    for (lo, hi), g in zip(zip(edges[:-1], edges[1:]), first + (1.2, 0.8, 0.3)):
        m = (f < hi) if lo == -np.inf else ((f >= lo) & (f < hi))
        out[m] *= g
    if vocal_suppression > 0:
        out[(f >= 800) & (f < 4000)] *= (1.0 - vocal_suppression * 0.5)
    return out


def app_band_table(fs: float = 48000, fft_base: int = 2048, bars: int = 512, n_bins: int = 512):
    """PrecomputedFrequencyMapper band_indices (freq_mapper.py:83-124) as the spectrum loop uses them
    (:1011-1036: stop at the first band ending past the spectrum, then [:bars]) and the EMA factor by the
    band's start frequency (:1044-1052)."""
    width = fs / fft_base
    mel = np.linspace(2595 * np.log10(1 + 20 / 700), 2595 * np.log10(1 + 20000 / 700), bars + 1)
    fp = [700 * (10 ** (m / 2595) - 1) for m in mel]
    fp[0], fp[-1] = max(20, fp[0]), min(20000, fp[-1])
    bands = []
    for i in range(min(bars, len(fp) - 1)):
        s, e = int(fp[i] / width), int(fp[i + 1] / width)
        e = s + 1 if e <= s else e
        s = max(0, min(s, fft_base // 2))
        bands.append((s, max(s + 1, min(e, fft_base // 2 + 1))))
    keep = []
    for s, e in bands:
        if e > n_bins:
            break
        keep.append((s, e))
    keep = keep[:bars]
    sf = [0.6 if s * fs / fft_base < 250 else (0.75 if s * fs / fft_base < 2000 else 0.85) for s, _ in keep]
    return keep, sf


class AppPostState:
    """process_multi_resolution_fft :748-752 + process_audio_spectrum :991-1056 for one stream."""

    def __init__(self, comb_freqs, fs=48000, fft_base=2048, bars=512, psycho=True, bass_boost=1.5,
                 freq_comp=True, normalization=False, smoothing=True, vocal_suppression=0.0):
        self.cf, self.fs, self.fft_base, self.bars = np.asarray(comb_freqs), fs, fft_base, bars
        self.psycho, self.boost, self.freq_comp = psycho, bass_boost, freq_comp
        self.norm, self.smooth, self.vs = normalization, smoothing, vocal_suppression
        self.curve = app_equal_loudness(fs, fft_base)
        self.freqs = np.fft.rfftfreq(fft_base, 1 / fs)
        self.prev = None

    def update(self, comb: np.ndarray):
        s = np.array(comb, dtype=np.float32)
        n = len(s)
        if self.psycho:
            s *= self.curve[:n]
            s[self.cf < 250] *= self.boost
        content = app_content_type(s, self.fs)
        if np.max(s) > 0:
            ref = np.percentile(s, 98)
            if ref > 0:
                s = s / ref * 0.8
        if self.freq_comp:
            s = app_compensation(s, self.freqs[:n], content, self.vs)
        if self.norm and np.max(s) > 0:
            s = s / np.max(s)
        bands, sf = app_band_table(self.fs, self.fft_base, self.bars, n)
        vals = []
        for a, b in bands:
            v = np.mean(s[a:b]) if b > a else s[a]
            if v > 0:
                v = max(0, min(1, np.sqrt(v)))
            vals.append(v)
        vals = np.array(vals)
        if self.smooth and self.prev is not None:
            for i, f in enumerate(sf):
                vals[i] = self.prev[i] * f + vals[i] * (1 - f)
        self.prev = vals.copy()
        return s, vals, content


def app_post_sequence(combined: np.ndarray, comb_freqs, **kw):
    """[F, T] combined spectra of one stream -> (spectrum [F, T], bands [F, nb], content [F])."""
    st = AppPostState(comb_freqs, **kw)
    out = [st.update(c) for c in combined]
    return (np.stack([o[0] for o in out]), np.stack([o[1] for o in out]).astype(np.float64),
            np.array([o[2] for o in out], np.int32))


# ----------------------------------------------------------------------------------------------
# the capture stream before the path -- parec chunks, the per-chunk noise
# gate (omega4/audio/capture.py:546-600, :620-641) and the app's input gain (omega4_main.py:648-688)
# ----------------------------------------------------------------------------------------------


class CaptureGate:
    """PipeWireMonitorCapture._process_audio_frame (capture.py:620-641) with AudioCaptureConfig's
    defaults (:28, :36-39). The expressions keep numpy's types: the RMS is a float32 scalar, so the
    background level turns float32 at its first update (Python float times np.float32)."""

    def __init__(self, fs: int = 48000, chunk: int = 512, noise_floor: float = 0.001,
                 silence_threshold_seconds: float = 0.25, background_alpha: float = 0.001):
        self.chunk, self.noise_floor, self.alpha = chunk, noise_floor, background_alpha
        self.silence_samples = 0
        self.silence_threshold = int(fs * silence_threshold_seconds)
        self.background_level = 0.0

    def process(self, x: np.ndarray) -> np.ndarray:
        rms = np.sqrt(np.mean(x ** 2))
        if rms < self.noise_floor * 2:
            self.background_level = (1 - self.alpha) * self.background_level + self.alpha * rms
        if rms < max(self.noise_floor, self.background_level * 3):
            self.silence_samples += self.chunk
            if self.silence_samples > self.silence_threshold:
                return np.zeros_like(x)
        else:
            self.silence_samples = 0
        return x


def capture_stream(x: np.ndarray, fs: int = 48000, chunk: int = 512, gain: float = 4.0, gate: bool = True) -> np.ndarray:
    """One channel's analysed stream: whole capture chunks through the gate, times input_gain
    (float32 array times a Python float stays float32)."""
    g = CaptureGate(fs, chunk)
    n = len(x) // chunk * chunk
    y = np.concatenate([g.process(x[i:i + chunk]) if gate else x[i:i + chunk] for i in range(0, n, chunk)]) \
        if n else np.zeros(0, np.float32)
    return y * gain


def capture_stream_interleaved(x: np.ndarray, fs: int = 48000, chunk: int = 512, gain: float = 4.0,
                               gate: bool = True) -> np.ndarray:
    """The analysed streams of an interleaved capture x [n, C]: the capture loop reads chunk_size
    samples of the interleaved stream whatever the channel count (capture.py:549-550), so one gate
    (one RMS over all the chunk's channels, one state) runs over the flattened stream; then the
    input gain. Returns planar [C, n'] over the whole chunks, cut to whole frames."""
    x = np.asarray(x)
    C = x.shape[1]
    flat = x.reshape(-1)
    n = len(flat) // chunk * chunk
    g = CaptureGate(fs, chunk)
    y = np.concatenate([g.process(flat[i:i + chunk]) if gate else flat[i:i + chunk] for i in range(0, n, chunk)]) \
        if n else np.zeros(0, np.float32)
    y = y[:len(y) // C * C]
    return (y * gain).reshape(-1, C).T.copy()


def s16le_samples(data: bytes) -> np.ndarray:
    """capture.py:571-574 for s16le: int16 -> float32 / 32768.0."""
    return np.frombuffer(data, dtype=np.int16).astype(np.float32) / 32768.0


# ----------------------------------------------------------------------------------------------
# SURVEY.md §8(f) row 2 remainder: VU meter ballistics (omega4/panels/vu_meters.py:55-99)
# ----------------------------------------------------------------------------------------------


class VUState:
    """VUMetersPanel.update for one channel: the 300 ms sample deque (:28-30, :65-68), RMS (:71-72),
    dBFS + 18 (:76-81, :104-108), damping 0.94 (:84-85) and the 2 s peak hold with 10 dB/s decay
    stopping at -20 (:88-102)."""

    def __init__(self, fs: float = 48000):
        self.buf = deque(maxlen=int(300e-3 * fs))
        self.db, self.display, self.peak, self.peak_time = -60.0, -60.0, -60.0, 0.0

    def update(self, x: np.ndarray, dt: float):
        if x is None or len(x) == 0:
            return
        self.buf.extend(x)  # (the reference appends sample by sample)
        rms = np.sqrt(np.mean(np.array(self.buf) ** 2))
        dbfs = 20.0 * np.log10(rms) if rms > 0 else -60.0
        self.db = dbfs + 18.0
        self.display += (self.db - self.display) * (1.0 - 0.94)
        if self.display > self.peak:
            self.peak, self.peak_time = self.display, 0.0
        else:
            self.peak_time += dt
            if self.peak_time > 2.0:
                self.peak = max(self.peak - 10.0 * dt, -20.0)
        return self.db, self.display, self.peak


# ----------------------------------------------------------------------------------------------
# TransientAnalyzer.analyze_transients (omega4/analyzers/transient.py:19-108)
# ----------------------------------------------------------------------------------------------


class TransientState:
    """analyze_transients with the envelope history (transient.py:17, :33): scipy.signal.hilbert and
    savgol_filter (scipy 1.15.3 here), np.diff / np.std threshold, attack time and punch factor."""

    def __init__(self, fs: float = 48000):
        self.fs = fs
        self.envelope_history = deque(maxlen=int(0.5 * 60))

    def analyze(self, x: np.ndarray) -> Dict:
        from scipy import signal as ss
        if len(x) < 64:
            return {"transients_detected": 0, "attack_time": 0.0, "punch_factor": 0.0}
        env = np.abs(ss.hilbert(x))
        es = ss.savgol_filter(env, min(21, len(env) // 2 * 2 + 1), 3)
        self.envelope_history.append(np.mean(es))
        d = np.diff(es)
        pts = np.where(d > np.std(d) * 2.0)[0]
        times, punch = [], []
        for i in pts:
            if 10 < i < len(es) - 10:
                s0, pk = max(0, i - 10), es[i]
                ten = next((j for j in range(s0, i) if es[j] >= pk * 0.1), s0)
                ninety = next((j for j in range(ten, min(len(es), i + 10)) if es[j] >= pk * 0.9), i)
                times.append((ninety - ten) / self.fs * 1000)
            if 5 < i < len(es) - 5:
                punch.append(max(0.0, np.mean(es[i:i + 5]) - np.mean(es[i - 5:i])))
        return {"transients_detected": len(pts), "attack_time": np.mean(times) if times else 0.0,
                "punch_factor": np.mean(punch) if punch else 0.0, "envelope_peak": np.max(es),
                "envelope_rms": np.sqrt(np.mean(es ** 2))}
