"""Drop-in MultiResolutionFFT over libomega.so (omega4/audio/multi_resolution_fft.py:135-457).

Same constructor, attributes, call signatures, result types, dtypes and error convention
(log and return ``{}`` / zeros; constructors raise ``ValueError``) as the reference. The per-resolution
CircularBuffers (:52-133) are kept as one host ring of the last max(N_r) samples: resolution r is
available once N_r samples were written and then sees the last N_r of them, which is exactly what
``read_latest(N_r)`` returns. Every FFT, magnitude, weighting and combine runs on the MI355X.
"""
from __future__ import annotations

import logging
import threading
import time
from dataclasses import dataclass
from enum import Enum
from typing import Dict, NamedTuple, Tuple

import ctypes as C

import numpy as np

from . import _lib as L
from .engine import Engine, Resolution

logger = logging.getLogger(__name__)


class WindowType(Enum):
    BLACKMAN = "blackman"
    HANN = "hann"
    HAMMING = "hamming"
    BLACKMAN_HARRIS = "blackman_harris"  # the reference falls back to blackman (:183-184)


@dataclass
class FFTConfig:
    """multi_resolution_fft.py:26-44 (same validation and messages)."""

    freq_range: Tuple[float, float]
    fft_size: int
    hop_size: int
    weight: float
    window_type: WindowType = WindowType.BLACKMAN

    def __post_init__(self):
        if self.freq_range[0] >= self.freq_range[1]:
            raise ValueError(f"Invalid frequency range: {self.freq_range}")
        if self.fft_size <= 0 or (self.fft_size & (self.fft_size - 1)) != 0:
            raise ValueError(f"FFT size must be power of 2: {self.fft_size}")
        if self.hop_size <= 0:
            raise ValueError(f"Hop size must be positive: {self.hop_size}")
        if self.weight <= 0:
            raise ValueError(f"Weight must be positive: {self.weight}")


class FFTResult(NamedTuple):
    magnitude: np.ndarray
    frequencies: np.ndarray
    config_index: int


def _win_name(w: WindowType) -> str:
    return {WindowType.HANN: "hann", WindowType.HAMMING: "hamming"}.get(w, "blackman")


class MultiResolutionFFT:
    """Multi-resolution FFT analysis (multi_resolution_fft.py:135)."""

    def __init__(self, sample_rate: int = 48000, max_freq: float = 20000, device: int = 0):
        if sample_rate <= 0:
            raise ValueError("Sample rate must be positive")
        if max_freq <= 0 or max_freq > sample_rate / 2:
            raise ValueError("Max frequency must be positive and <= Nyquist")
        self.sample_rate = sample_rate
        self.nyquist = sample_rate / 2
        self.max_freq = min(max_freq, self.nyquist)
        self.device = device
        self.configs = [
            FFTConfig((20, 200), 4096, 1024, 1.5),
            FFTConfig((200, 1000), 2048, 512, 1.2),
            FFTConfig((1000, 5000), 1024, 256, 1.0),
            FFTConfig((5000, 20000), 1024, 256, 1.5),
        ]
        self._engines: Dict[tuple, Engine] = {}
        # process_audio_chunk and combine_results_optimized share the ring, the prepared calls and the
        # last chunk's same-launch combine; the app may call them from different threads
        self._lock = threading.RLock()
        # combine target the next chunk forms in its own launch: the target_bins combine_results_optimized
        # was last asked for (the app's display bars, omega4_main.py:714-717), 1024 until then
        self._want_bins = 1024
        self._setup_windows()
        self._setup_buffers()
        self._setup_frequency_arrays()
        self._setup_working_arrays()
        self.processing_stats = {"total_calls": 0, "total_time": 0.0, "error_count": 0}

    # The reference builds per-config tables in these hooks; callers that replace ``configs`` call
    # them again. Here they invalidate the device contexts built from configs.
    def _setup_windows(self):
        self._engines = {}
        self._calls = {}

    def _setup_buffers(self):
        self._wmax = max(c.fft_size for c in self.configs)
        self._ring = np.zeros(max(512, self._wmax), np.float32)  # (the last _wmax samples at the end)
        self._written = 0
        self._calls = {}
        self._tfreqs = {}

    def _setup_frequency_arrays(self):
        self.freq_arrays = {i: np.fft.rfftfreq(c.fft_size, 1 / self.sample_rate) for i, c in enumerate(self.configs)}

    def _setup_working_arrays(self):
        self._engines = {}
        self._calls = {}

    def _resolutions(self):
        return [Resolution(tuple(c.freq_range), c.fft_size, c.hop_size, c.weight, _win_name(c.window_type))
                for c in self.configs]

    def _cfg_key(self):
        # everything an engine is built from: a caller may replace configs, max_freq or sample_rate
        return (self.sample_rate, self.max_freq,
                tuple((tuple(c.freq_range), c.fft_size, c.weight, c.window_type) for c in self.configs))

    def _engine(self, apply_weighting: bool, target_bins: int = 1024) -> Engine:
        key = (apply_weighting, target_bins, self._cfg_key())
        eng = self._engines.get(key)
        if eng is None:
            eng = Engine(self._resolutions(), self.sample_rate, self.max_freq, target_bins,
                         frame_size=max(512, self._wmax), apply_weighting=apply_weighting, device=self.device)
            self._engines[key] = eng
        return eng

    def _chunk_call(self, apply_weighting: bool, avail, full: bool, target_bins: int):
        """The per-chunk device call, prepared once per (configs, weighting, available resolutions, combine
        target): the C ABI's output struct over persistent host arrays (the results get copies), so a call
        is one ctypes call on the ring (host memory; omega_process_frames stages it page-locked and returns
        every output in one copy)."""
        key = (apply_weighting, tuple(avail), full, target_bins, self._cfg_key())
        prep = self._calls.get(key)
        if prep is None:
            eng = self._engine(apply_weighting, target_bins)
            outs = L.Outputs()
            mags = {i: np.empty((1, self.configs[i].fft_size // 2 + 1), np.float32) for i in avail}
            for i, a in mags.items():
                outs.mag[i] = a.ctypes.data
            comb = np.empty((1, eng.T), np.float32) if full else None
            if comb is not None:
                outs.combined = comb.ctypes.data
            prep = (eng, outs, mags, comb)
            self._calls[key] = prep
        return prep

    def process_audio_chunk(self, audio_chunk: np.ndarray, apply_weighting: bool = True) -> Dict[int, FFTResult]:
        """multi_resolution_fft.py:228-302."""
        if audio_chunk is None or len(audio_chunk) == 0:
            logger.warning("Empty audio chunk received")
            return {}
        try:
            start = time.perf_counter()
            # (float64 frames -- the app's Hann-windowed ring slice, omega4_main.py:952-980 -- are cast
            # by the copy into the float32 ring, not by a separate pass)
            chunk = np.asarray(audio_chunk).ravel()
            with self._lock:
                if self._wmax != max(c.fft_size for c in self.configs):
                    self._setup_buffers()
                ring, n = self._ring, len(chunk)
                if n >= self._wmax:
                    ring[-self._wmax:] = chunk[-self._wmax:]
                else:  # (in place: the ring's address stays what the prepared calls hold)
                    ring[:-n] = ring[n:]
                    ring[-n:] = chunk
                self._written = min(self._written + n, 1 << 62)
                avail = [i for i, c in enumerate(self.configs) if self._written >= c.fft_size]
                results: Dict[int, FFTResult] = {}
                self._last = None
                if avail:
                    # with the magnitudes of every resolution, the same launch also forms their combine
                    # (multi_resolution_fft.py:335-408) for the target_bins last asked for:
                    # combine_results_optimized of exactly these results then needs no second round trip
                    full = len(avail) == len(self.configs)
                    tb = self._want_bins
                    eng, outs, mags, comb = self._chunk_call(apply_weighting, avail, full, tb)
                    L.check(eng._ctx, L.lib().omega_process_frames(eng._ctx, ring.ctypes.data, 1, eng.W, eng.W,
                                                                    C.byref(outs), L.MEM_HOST))
                    for i in avail:
                        results[i] = FFTResult(magnitude=mags[i][0].copy(), frequencies=self.freq_arrays[i],
                                               config_index=i)
                    if full:
                        self._last = ({i: (results[i].magnitude, mags[i][0]) for i in avail}, comb[0], tb,
                                      self._cfg_key())
            self.processing_stats["total_calls"] += 1
            self.processing_stats["total_time"] += time.perf_counter() - start
            return results
        except Exception as e:  # the reference swallows and logs (:299-302)
            logger.error(f"Multi-resolution FFT processing failed: {e}")
            self.processing_stats["error_count"] += 1
            return {}

    def process_frames(self, frames: np.ndarray, apply_weighting: bool = True):
        """Batched stateless form: frames [F, W] -> {i: magnitudes [F, N_i/2+1]} for every resolution
        (each frame seen by a fresh instance)."""
        frames = np.ascontiguousarray(frames, dtype=np.float32)
        eng = self._engine(apply_weighting)
        if frames.shape[1] != eng.W:
            raise ValueError(f"frames must have {eng.W} samples")
        out = eng.process_frames(frames, frames.shape[0], eng.W, eng.W, combined=False, lufs=False,
                                 true_peak=False, mags=True)
        return {i: out[f"mag{i}"] for i in range(len(self.configs))}

    def combine_results_optimized(self, results: Dict[int, FFTResult],
                                  target_bins: int = 1024) -> Tuple[np.ndarray, np.ndarray]:
        """multi_resolution_fft.py:335-408."""
        if not results:
            logger.warning("No FFT results to combine")
            return np.zeros(target_bins), np.linspace(0, self.max_freq, target_bins)
        try:
            with self._lock:
                last = getattr(self, "_last", None)
                if (last is not None and target_bins == last[2] and last[3] == self._cfg_key()
                        and self._same_results(results, last[0])):
                    tf = self._tfreqs.get((self.max_freq, target_bins))
                    if tf is None:
                        tf = self._tfreqs[(self.max_freq, target_bins)] = np.linspace(0, self.max_freq, target_bins)
                    return last[1].copy(), tf.copy()
                # the next chunk forms this target in its own launch
                if isinstance(target_bins, (int, np.integer)) and target_bins > 0:
                    self._want_bins = int(target_bins)
                target_freqs = np.linspace(0, self.max_freq, target_bins)
                eng = self._engine(True, target_bins)
                mags = {r.config_index: r.magnitude for r in results.values()}
                out = eng.combine(mags, 1)
                return out[0].copy(), target_freqs
        except Exception as e:
            logger.error(f"FFT result combination failed: {e}")
            return np.zeros(target_bins), np.linspace(0, self.max_freq, target_bins)

    @staticmethod
    def _same_results(results, ref) -> bool:
        """results are the last process_audio_chunk's, unmodified: every resolution present with its own
        magnitude array object holding the values the device returned."""
        if len(results) != len(ref):
            return False
        for r in results.values():
            got = ref.get(getattr(r, "config_index", None))
            if got is None or r.magnitude is not got[0] or not np.array_equal(got[0], got[1]):
                return False
        return True

    def get_frequency_arrays(self) -> Dict[int, np.ndarray]:
        return self.freq_arrays.copy()

    def reset_all_buffers(self):
        with self._lock:
            self._ring.fill(0)
            self._last = None
            self._written = 0
        logger.info("All buffers reset")

    def get_processing_stats(self) -> Dict[str, float]:
        stats = self.processing_stats.copy()
        if stats["total_calls"] > 0:
            stats["avg_time_ms"] = stats["total_time"] / stats["total_calls"] * 1000
            stats["error_rate"] = stats["error_count"] / stats["total_calls"]
        else:
            stats["avg_time_ms"] = 0.0
            stats["error_rate"] = 0.0
        return stats

    def get_buffer_status(self) -> Dict[int, Dict[str, int]]:
        out = {}
        for i, c in enumerate(self.configs):
            size = max(c.fft_size * 2, c.fft_size + c.hop_size)
            w = min(self._written, size)
            out[i] = {"size": size, "write_pos": self._written % size, "samples_written": w,
                      "utilization_pct": int(w / size * 100)}
        return out

    def cleanup(self):
        self.reset_all_buffers()
        for e in self._engines.values():
            e.close()
        self._engines = {}


def create_default_multi_fft(sample_rate: int = 48000) -> MultiResolutionFFT:
    return MultiResolutionFFT(sample_rate=sample_rate)


def benchmark_multi_fft(sample_rate: int = 48000, chunk_size: int = 512, num_iterations: int = 1000,
                        device: int = 0) -> Dict[str, float]:
    """multi_resolution_fft.py:467-494: the default configs fed the same random 512-sample chunk,
    process_audio_chunk + combine_results_optimized per iteration (10 untimed warm-up calls), timed on
    the host clock; the reference's published figure for this loop is 0.20 ms per iteration
    (docs/MULTI_RESOLUTION_FFT_IMPROVEMENTS.md:193-195)."""
    fft_processor = MultiResolutionFFT(sample_rate=sample_rate, device=device)
    test_audio = np.random.random(chunk_size).astype(np.float32)
    for _ in range(10):
        fft_processor.process_audio_chunk(test_audio)
    start_time = time.perf_counter()
    for _ in range(num_iterations):
        results = fft_processor.process_audio_chunk(test_audio)
        if results:
            combined, freqs = fft_processor.combine_results_optimized(results)
    total_time = time.perf_counter() - start_time
    return {"total_time_s": total_time, "avg_time_ms": total_time / num_iterations * 1000,
            "iterations_per_second": num_iterations / total_time, "stats": fft_processor.get_processing_stats()}
