"""Drop-in ProfessionalMetering over libomega.so (omega4/panels/professional_meters.py:13-299).

``calculate_lufs`` returns the same (mutated, shared) ``current_lufs`` dict with the same keys; the
K-weighting, the instantaneous LUFS, the 4x true peak and the momentary / short-term / integrated /
range / peak-hold deques all run on the MI355X (the deques live in the context as device-side
per-stream history). Filter coefficients are derived in the library (closed forms of
scipy.signal.butter / lfilter_zi) and exposed here for inspection.

Frames of any length are metered, like the reference (its 4800-sample chunks included): the weighting
runs scipy's float64 filtfilt cascade on the device (omega_weighting, any length above filtfilt's
padlen of 9), the true peak the polyphase form of scipy's resample on the power-of-two kernels or, for
other lengths, the mixed-radix transform (anyfft.hip). Nothing here raises to the caller (the
reference's convention): errors (e.g. a frame of 9 samples or fewer, where scipy's filtfilt raises)
are logged and the previous values (or, for the weighted signal, zeros) returned. calculate_true_peak
supports oversampling 1, 2 and 4 (the reference's default; 1 and 2 are phase subsets of the 4x form).
"""
from __future__ import annotations

import logging
from typing import Dict

import numpy as np

from .engine import Engine, Resolution

logger = logging.getLogger(__name__)

def _butter2_highpass(fc: float, fs: float):
    k = np.tan(np.pi * fc / fs)
    n = 1 + np.sqrt(2) * k + k * k
    return np.array([1.0, -2.0, 1.0]) / n, np.array([1.0, 2 * (k * k - 1) / n, (1 - np.sqrt(2) * k + k * k) / n])


def _butter2_lowpass(fc: float, fs: float):
    k = np.tan(np.pi * fc / fs)
    n = 1 + np.sqrt(2) * k + k * k
    return np.array([k * k, 2 * k * k, k * k]) / n, np.array([1.0, 2 * (k * k - 1) / n, (1 - np.sqrt(2) * k + k * k) / n])


def _butter1(fc: float, fs: float, high: bool):
    k = np.tan(np.pi * fc / fs)
    b = np.array([1.0, -1.0]) / (1 + k) if high else np.array([k, k]) / (1 + k)
    return b, np.array([1.0, (k - 1) / (k + 1)])


class ProfessionalMetering:
    """Professional audio metering standards (LUFS, K-weighting, True Peak)."""

    def __init__(self, sample_rate: int = 48000, device: int = 0):
        self.sample_rate = sample_rate
        self.gate_threshold = -70.0
        self.weighting_mode = "K"
        self.k_weighting_filter = self.create_k_weighting_filter()
        self.current_lufs = {"momentary": -100.0, "short_term": -100.0, "integrated": -100.0, "range": 0.0,
                             "true_peak": -100.0}
        self.current_true_peak = -100.0
        self.a_weighting_filter = self.create_a_weighting_filter()
        self.c_weighting_filter = self.create_c_weighting_filter()
        # one context: its meter state is the four deques of :20-25 for one stream
        self._eng = Engine([Resolution((20, 20000), 512, 256, 1.0)], sample_rate, min(20000, sample_rate / 2),
                           target_bins=2, frame_size=512, n_channels=1, device=device)

    @staticmethod
    def _frame(audio_data):
        return np.asarray(audio_data, dtype=np.float32).ravel()

    @staticmethod
    def _tp_type(audio_data):
        """The dtype calculate_true_peak returns (professional_meters.py:289-299): scipy's resample
        keeps float32 (and computes float16 in float32) and gives float64 for every other input, int
        frames and lists included; ``20 * np.log10`` keeps that type. Silence is the Python float
        -100.0 the reference returns (:295-296)."""
        dt = np.asarray(audio_data).dtype
        t = np.float32 if dt in (np.float32, np.float16) else np.float64
        return lambda v: -100.0 if v == -100.0 else t(v)

    def apply_k_weighting(self, audio_data: np.ndarray) -> np.ndarray:
        """professional_meters.py:129-153 (returned as float64 like scipy's filtfilt)."""
        return self._weighted(audio_data, "K")

    def create_k_weighting_filter(self):
        """professional_meters.py:48-72: second-order Butterworth high-passes at 38 Hz and at 1500 Hz
        (the reference's "simplified shelf": iirfilter(2, ..., btype='high', ftype='butter')) and the
        +4 dB shelf gain it computes but never applies (:59). The device builds the same coefficients
        for the K-weighting it runs (omega_k_weighting / omega_weighting)."""
        hp_b, hp_a = _butter2_highpass(38.0, self.sample_rate)
        sh_b, sh_a = _butter2_highpass(1500.0, self.sample_rate)
        return {"hp_b": hp_b, "hp_a": hp_a, "shelf_b": sh_b, "shelf_a": sh_a, "shelf_gain": 10 ** (4.0 / 20)}

    def create_a_weighting_filter(self):
        """professional_meters.py:74-107: the four cascaded Butterworth sections (the device builds the
        same coefficients in omega_weighting)."""
        fs, nyq = self.sample_rate, self.sample_rate / 2
        return {"hp1": _butter2_highpass(20.598997, fs), "hp2": _butter1(107.65265, fs, True),
                "lp1": _butter1(737.86223, fs, False), "lp2": _butter2_lowpass(min(12194.217 / nyq, 0.99) * nyq, fs),
                "gain": 1.0}

    def create_c_weighting_filter(self):
        """professional_meters.py:109-127."""
        fs, nyq = self.sample_rate, self.sample_rate / 2
        return {"hp": _butter2_highpass(20.598997, fs), "lp": _butter2_lowpass(min(12194.217 / nyq, 0.99) * nyq, fs),
                "gain": 1.0}

    def _weighted(self, audio_data, mode: str) -> np.ndarray:
        try:
            w, _ = self._eng.weighting(self._frame(audio_data), mode)
            return w[0].astype(np.float64)
        except Exception as e:
            logger.error("apply_%s_weighting: %s", mode.lower(), e)
            return np.zeros(len(audio_data), np.float64)

    def apply_a_weighting(self, audio_data: np.ndarray) -> np.ndarray:
        """professional_meters.py:155-192: RMS gate, four cascaded filtfilt sections, times 2.5."""
        return self._weighted(audio_data, "A")

    def apply_c_weighting(self, audio_data: np.ndarray) -> np.ndarray:
        """professional_meters.py:194-218: RMS gate, two cascaded filtfilt sections."""
        return self._weighted(audio_data, "C")

    def apply_weighting(self, audio_data: np.ndarray) -> np.ndarray:
        """professional_meters.py:220-229: K, A and C on the device; any other mode is Z (unweighted)."""
        if self.weighting_mode not in ("K", "A", "C"):
            return audio_data
        return self._weighted(audio_data, self.weighting_mode)

    def calculate_true_peak(self, audio_data: np.ndarray, oversampling: int = 4) -> float:
        """professional_meters.py:283-299 (the result follows the input dtype like scipy's resample:
        float32 for float32 frames, float64 for the app's float64 Hann frames, omega4_main.py:1082)."""
        if len(audio_data) == 0:
            return -100.0
        try:
            tp = self._eng.true_peak(self._frame(audio_data), oversampling)[0]
            self.current_true_peak = self._tp_type(audio_data)(tp)
        except Exception as e:
            logger.error("calculate_true_peak: %s", e)
        return self.current_true_peak

    def calculate_lufs(self, audio_data: np.ndarray) -> Dict[str, float]:
        """professional_meters.py:231-281."""
        if len(audio_data) == 0:
            return self.current_lufs
        try:
            x = self._frame(audio_data)
            mode = "Z" if self.weighting_mode not in ("K", "A", "C") else self.weighting_mode
            m = self._eng.calculate_lufs(x, mode)[2][0]  # weighting + true peak + aggregates, one round trip
        except Exception as e:
            logger.error("calculate_lufs: %s", e)
            return self.current_lufs
        self.current_lufs["momentary"] = np.float64(m[0])
        self.current_lufs["short_term"] = np.float64(m[1])
        self.current_lufs["integrated"] = np.float64(m[2])
        self.current_lufs["range"] = np.float64(m[3])
        self.current_lufs["true_peak"] = self._tp_type(audio_data)(m[4])
        return self.current_lufs

    def calculate_lufs_batch(self, frames: np.ndarray) -> np.ndarray:
        """Batched form: frames [F, M] of one stream in order -> [F, 5] dict values per call."""
        frames = np.ascontiguousarray(frames, dtype=np.float32)
        mode = "Z" if self.weighting_mode not in ("K", "A", "C") else self.weighting_mode
        _, li = self._eng.weighting(frames, mode, weighted=False)
        tp = self._eng.true_peak(frames)
        return self._eng.meter_update(li, tp, frames.shape[0])

    def reset(self):
        self._eng.reset_meters()
        self.current_lufs.update({"momentary": -100.0, "short_term": -100.0, "integrated": -100.0, "range": 0.0,
                                  "true_peak": -100.0})
