"""App spectrum post-processing on the MI355X: what
omega4_main.ProfessionalLiveAudioAnalyzer does to each frame's combined spectrum after
combine_results_optimized -- the equal-loudness curve and bass boost of process_multi_resolution_fft
(omega4_main.py:748-752), update_content_type (:805-840, without voice detection), and
process_audio_spectrum's 98th-percentile normalisation (:991-997), apply_frequency_compensation
(:855-926), optional max normalisation (:1004-1005), band means -> sqrt -> clamp (:1011-1036) and
frequency-dependent band EMA (:1041-1056) -- for a block of consecutive frames of one stream in two
kernel launches (omega_post_process). The tables are the app's own precomputation, built here once.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict

import numpy as np

from . import _lib as L
from .engine import Engine, _is_torch

CONTENT_TYPES = ("instrumental", "vocal", "bass_heavy")
PSYCHO, FREQ_COMP, NORMALIZE, SMOOTH = 1, 2, 4, 8


def _band_table(fs, fft_base, bars, n_bins):
    """freq_mapper.py:83-124 band_indices, cut as the spectrum loop cuts them (:1011-1013, :1035), and
    the EMA factor by band start frequency (:1044-1052)."""
    width = fs / fft_base
    mel = np.linspace(2595 * np.log10(1 + 20 / 700), 2595 * np.log10(1 + 20000 / 700), bars + 1)
    edges = [700 * (10 ** (m / 2595) - 1) for m in mel]
    edges[0], edges[-1] = max(20, edges[0]), min(20000, edges[-1])
    starts, ends = [], []
    for i in range(bars):
        s, e = int(edges[i] / width), int(edges[i + 1] / width)
        if e <= s:
            e = s + 1
        s = max(0, min(s, fft_base // 2))
        e = max(s + 1, min(e, fft_base // 2 + 1))
        if e > n_bins:
            break
        starts.append(s), ends.append(e)
    hz = np.array(starts, np.float64) * fs / fft_base
    f = np.where(hz < 250, 0.6, np.where(hz < 2000, 0.75, 0.85))
    return np.array(starts, np.int32), np.array(ends, np.int32), f


class SpectrumPostProcessor:
    """One stream's post-processing of [F, T] combined spectra (T = bars, 512 in the app). Options are
    the app's toggles (omega4_main.py:158-161, :343-346). ``process`` returns (spectrum [F, T] float32,
    band_values [F, n_bands] float64 -- each row numpy's float32 or float64 band array exactly, see
    omega.h --, content [F]: indices into CONTENT_TYPES); the band EMA carries over between calls
    (``reset`` starts a new stream)."""

    def __init__(self, comb_frequencies, sample_rate: int = 48000, fft_size_base: int = 2048, bars: int = 512,
                 psychoacoustic_enabled: bool = True, psycho_bass_boost: float = 1.5,
                 freq_compensation_enabled: bool = True, normalization_enabled: bool = False,
                 smoothing_enabled: bool = True, vocal_suppression: float = 0.0, device: int = 0):
        self.sample_rate, self.fft_size_base, self.bars = sample_rate, fft_size_base, bars
        cf = np.asarray(comb_frequencies, np.float64)
        T = len(cf)
        self.n_bins = T
        f = np.fft.rfftfreq(fft_size_base, 1 / sample_rate)
        if T > len(f):
            raise ValueError(f"{T} spectrum bins exceed the base FFT's {len(f)} (the reference's tables by position)")
        f = f[:T]
        # _create_equal_loudness_curve :617-644, by position
        curve = np.ones(T)
        curve[f < 200] = 1 + (200 - f[f < 200]) / 50
        curve[(f > 500) & (f < 2000)] *= 0.85
        curve[(f > 2000) & (f < 5000)] *= 1.05
        curve[f > 6000] *= 0.5
        curve[f > 10000] *= 0.2
        # apply_frequency_compensation :872-919: one factor per bin (the ranges are disjoint)
        def comp(first):
            c = np.ones(T, np.float32)
            for (lo, hi), g in zip(((0, 60), (60, 250), (250, 500), (500, 2000), (2000, 6000), (6000, 10000),
                                    (10000, np.inf)), first + (1.2, 0.8, 0.3)):
                c[(f >= lo) & (f < hi)] = np.float32(g)
            return c
        vsup = np.ones(T, np.float32)
        if vocal_suppression > 0:
            vsup[(f >= 800) & (f < 4000)] = np.float32(1.0 - vocal_suppression * 0.5)
        w = sample_rate / (2 * T)
        ranges = np.array([int(250 / w), int(200 / w), int(4000 / w), int(6000 / w)], np.int32)
        # np.percentile(., 98), method 'linear', all in float32: numpy's virtual index is (n - 1) q
        # (numpy/lib/_function_base_impl.py 'linear' get_virtual_index), not n q + (1 - q) - 1
        q = np.float32(98) / np.float32(100)
        vi = np.float32(T - 1) * q
        lo = min(max(int(np.floor(vi)), 0), T - 1)
        hi = min(lo + 1, T - 1)
        gamma = np.float32(vi - np.float32(lo))
        bs, be, sf = _band_table(sample_rate, fft_size_base, bars, T)
        smooth = np.ascontiguousarray(sf, np.float64)
        self.n_bands = len(bs)
        self._flags = ((PSYCHO if psychoacoustic_enabled else 0) | (FREQ_COMP if freq_compensation_enabled else 0)
                       | (NORMALIZE if normalization_enabled else 0) | (SMOOTH if smoothing_enabled else 0))
        self._boost = float(np.float32(psycho_bass_boost))
        self._eng = Engine(sample_rate=sample_rate, device=device)
        bass = (cf < 250).astype(np.uint8)
        keep = [curve, bass, comp((0.8, 1.0, 1.1, 0.85)), comp((0.15, 0.2, 0.6, 1.5)), vsup, ranges, bs, be, smooth]
        ptr = [a.ctypes.data if len(a) else None for a in keep]
        self._eng._check(L.lib().omega_post_configure(
            self._eng._ctx, T, ptr[0], ptr[1], ptr[2], ptr[3], ptr[4], ptr[5], lo, hi, C.c_float(gamma),
            ptr[6], ptr[7], ptr[8], self.n_bands))

    def process(self, spectra):
        """spectra: [F, T] float32, host numpy or device torch (results come back the same way)."""
        import torch
        host = not _is_torch(spectra)
        dev = torch.device("cuda", self._eng.device)
        x = torch.as_tensor(np.ascontiguousarray(np.atleast_2d(spectra), np.float32)).to(dev) if host else spectra
        if x.dtype != torch.float32 or x.dim() != 2 or x.shape[1] != self.n_bins or x.stride(1) != 1:
            raise ValueError(f"spectra must be [F, {self.n_bins}] float32 rows")
        F = x.shape[0]
        spec = torch.empty((F, self.n_bins), dtype=torch.float32, device=x.device)
        bands = torch.empty((F, self.n_bands), dtype=torch.float64, device=x.device)
        content = torch.empty(F, dtype=torch.int32, device=x.device)
        self._eng._bind_stream(x)
        self._eng._check(L.lib().omega_post_process(self._eng._ctx, x.data_ptr(), F, x.stride(0), self._flags,
                                                    C.c_float(self._boost), spec.data_ptr(), bands.data_ptr(),
                                                    content.data_ptr()))
        if host:
            torch.cuda.current_stream(x.device).synchronize()
            return spec.cpu().numpy(), bands.cpu().numpy(), content.cpu().numpy()
        return spec, bands, content

    def process_dict(self, spectra) -> Dict[str, object]:
        s, b, c = self.process(spectra)
        return {"spectrum": s, "band_values": b, "content_type": c}

    def reset(self):
        self._eng._check(L.lib().omega_post_reset(self._eng._ctx))
