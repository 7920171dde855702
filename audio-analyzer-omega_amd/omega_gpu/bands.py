"""Band reductions over libomega.so.

``PipelineBands.map_to_bands`` mirrors AudioProcessingPipeline.map_to_bands (omega4/audio/pipeline.py:
295-335) with its band table (:165-230) and compensation (:145-163); ``PrecomputedFrequencyMapper``
mirrors omega4/optimization/freq_mapper.py:25-208. The tables are built host-side once (they are the
reference's own precomputation); every reduction runs on the device.
"""
from __future__ import annotations

import logging
from typing import Dict, List, Tuple

import numpy as np

from . import _lib as L
from .engine import BandTable, Engine, Resolution

logger = logging.getLogger(__name__)


def _table_engine(sample_rate: int, device: int) -> Engine:
    return Engine([Resolution((20, 20000), 512, 256, 1.0)], sample_rate, min(20000, sample_rate / 2), target_bins=2,
                  frame_size=512, device=device)


def pipeline_band_table(sample_rate=48000, num_bands=768, fft_size=4096, min_frequency=20.0,
                        max_frequency=20000.0, transition_frequency=1000.0, low_freq_band_ratio=0.5):
    """pipeline.py:165-230 and :145-163 -> (starts, ends, compensation); num_bands-1 bands."""
    nyq = sample_rate / 2
    if fft_size <= 0 or (fft_size & (fft_size - 1)) != 0:
        fft_size = 4096
    width = nyq / (fft_size // 2)
    max_f = min(max_frequency, nyq)
    tb = int(num_bands * low_freq_band_ratio)
    lows = np.logspace(np.log10(min_frequency), np.log10(transition_frequency), tb)
    highs = np.linspace(transition_frequency, max_f, num_bands - tb + 1)[1:]
    allf = np.concatenate([lows, highs])
    starts, ends, fs0, fs1 = [], [], [], []
    for i in range(min(len(allf) - 1, num_bands)):
        a, b = allf[i], allf[i + 1]
        s, e = int(a / width), int(b / width)
        if e <= s:
            e = s + 1
        s = max(0, min(s, fft_size // 2 - 1))
        e = max(s + 1, min(e, fft_size // 2))
        starts.append(s), ends.append(e), fs0.append(a), fs1.append(b)
    centers = (np.array(fs0) + np.array(fs1)) / 2
    comp = np.ones_like(centers)
    comp[centers < 100] = 2.0
    comp[(centers >= 100) & (centers < 250)] = 1.5
    comp[(centers >= 250) & (centers < 1000)] = 1.2
    comp[centers >= 10000] = 1.3
    return np.array(starts, np.int32), np.array(ends, np.int32), comp


class PipelineBands:
    """The band-mapping half of AudioProcessingPipeline (max-reduce x compensation + EMA)."""

    def __init__(self, sample_rate=48000, num_bands=768, fft_size=4096, smoothing_factor=0.7, device=0, **kw):
        self.sample_rate, self.num_bands, self.fft_size = sample_rate, num_bands, fft_size
        self.smoothing_factor = smoothing_factor
        self.starts, self.ends, self.freq_compensation = pipeline_band_table(sample_rate, num_bands, fft_size, **kw)
        self.band_indices = {"starts": list(self.starts), "ends": list(self.ends)}
        self.smoothing_buffer = np.zeros(num_bands, np.float32)
        self._eng = _table_engine(sample_rate, device)
        self._tables: Dict[int, BandTable] = {}

    def _table(self, n_bins: int) -> BandTable:
        t = self._tables.get(n_bins)
        if t is None:
            t = BandTable(self._eng, L.BANDS_MAX, self.starts, self.ends, self.num_bands, n_bins,
                          scale=self.freq_compensation)
            self._tables[n_bins] = t
        return t

    def map_to_bands_batch(self, mags: np.ndarray) -> np.ndarray:
        """[F, n_bins] -> [F, num_bands] without smoothing (stateless per frame)."""
        mags = np.atleast_2d(mags)
        return self._table(mags.shape[1]).apply(mags)

    def map_to_bands(self, fft_magnitude: np.ndarray, apply_smoothing: bool = True) -> np.ndarray:
        """pipeline.py:295-335."""
        try:
            if fft_magnitude is None or len(fft_magnitude) == 0:
                return np.zeros(self.num_bands, np.float32)
            v = self.map_to_bands_batch(fft_magnitude)[0]
            if apply_smoothing:
                self.smoothing_buffer *= self.smoothing_factor
                self.smoothing_buffer += (1 - self.smoothing_factor) * v
                return self.smoothing_buffer.copy()
            return v.copy()
        except Exception as e:
            logger.error(f"Error in band mapping: {e}")
            return np.zeros(self.num_bands)


class PrecomputedFrequencyMapper:
    """freq_mapper.py:25-208 with the mel band mean on the device."""

    def __init__(self, sample_rate: int, fft_size: int, num_bars: int, device: int = 0):
        self.sample_rate, self.fft_size, self.num_bars = sample_rate, fft_size, num_bars
        self.freq_bin_width = sample_rate / fft_size
        self.band_indices = self._create_mel_band_mapping()
        nb = fft_size // 2 + 1
        f = np.arange(nb) * self.freq_bin_width
        self.compensation_curve = self._compute_compensation_curve(f)
        self.frequency_points = np.zeros(num_bars)
        for i, (s, e) in enumerate(self.band_indices[:num_bars]):
            self.frequency_points[i] = ((s + e) // 2) * self.freq_bin_width
        self._eng = _table_engine(sample_rate, device)
        self._tables: Dict[Tuple[int, bool], BandTable] = {}

    def _create_mel_band_mapping(self) -> List[Tuple[int, int]]:
        """freq_mapper.py:83-124."""
        mel = np.linspace(2595 * np.log10(1 + 20 / 700), 2595 * np.log10(1 + 20000 / 700), self.num_bars + 1)
        fp = [700 * (10 ** (m / 2595) - 1) for m in mel]
        fp[0] = max(20, fp[0])
        fp[-1] = min(20000, fp[-1])
        bands = []
        for i in range(self.num_bars):
            if i >= len(fp) - 1:
                break
            s, e = int(fp[i] / self.freq_bin_width), int(fp[i + 1] / self.freq_bin_width)
            if e <= s:
                e = s + 1
            s = max(0, min(s, self.fft_size // 2))
            e = max(s + 1, min(e, self.fft_size // 2 + 1))
            bands.append((s, e))
        return bands

    @staticmethod
    def _compute_compensation_curve(f: np.ndarray) -> np.ndarray:
        """freq_mapper.py:146-163 (vectorised, same piecewise values)."""
        c = np.ones_like(f)
        pos = f > 0
        c = np.where(pos & (f < 100), 1.0 + (100 - f) / 100 * 0.5, c)
        c = np.where(pos & (f >= 1000) & (f < 4000), 1.0 + (f - 1000) / 3000 * 0.3, c)
        c = np.where(pos & (f >= 4000), 1.3 - (f - 4000) / 16000 * 0.5, c)
        return c

    def _table(self, n_bins: int, comp: bool) -> BandTable:
        t = self._tables.get((n_bins, comp))
        if t is None:
            s = np.array([b[0] for b in self.band_indices], np.int32)
            e = np.array([b[1] for b in self.band_indices], np.int32)
            t = BandTable(self._eng, L.BANDS_MEAN, s, e, self.num_bars, n_bins,
                          bin_scale=self.compensation_curve if comp else None)
            self._tables[(n_bins, comp)] = t
        return t

    def map_spectrum_to_bars_batch(self, spectra: np.ndarray, apply_compensation: bool = True) -> np.ndarray:
        spectra = np.atleast_2d(spectra)
        comp = apply_compensation and spectra.shape[1] == len(self.compensation_curve)
        return self._table(spectra.shape[1], comp).apply(spectra)

    def map_spectrum_to_bars(self, spectrum: np.ndarray, apply_compensation: bool = True) -> np.ndarray:
        """freq_mapper.py:165-196."""
        return self.map_spectrum_to_bars_batch(spectrum, apply_compensation)[0]

    def get_frequency_for_bar(self, bar_index: int) -> float:
        return self.frequency_points[bar_index] if 0 <= bar_index < self.num_bars else 0.0

    def get_bar_for_frequency(self, frequency: float) -> int:
        idx = np.searchsorted(self.frequency_points, frequency)
        return max(0, min(idx, self.num_bars - 1))
