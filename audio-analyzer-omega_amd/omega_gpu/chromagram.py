"""ChromagramAnalyzer.compute_chromagram over libomega.so (omega4/panels/chromagram.py:109-237).

The per-frame work (harmonic suppression, the 12 x K Gaussian pitch-class projection, smoothing,
normalisation) runs on the device; the genre-dependent temporal blend with the previous frame
(:215-237) is 12 multiply-adds and stays with the stateful caller object, as in the reference.
The tuning offset (:111-113, :128-129) is a whole number of semitones added to every bin's MIDI
number, so it rotates the 12 classes: the device computes the offset-0 chroma and the facade rolls it
(smoothing and normalisation commute with the rotation). The offset itself (detect_tuning_offset,
:581-639, metal / rock only) is a peak pick over the handful of 70-100 Hz bins of each frame plus a
30-deep mode -- scalar host logic, like the reference's.
Key/chord/mode detection (:239-935) is out of scope (scalar host logic on 12 numbers).
"""
from __future__ import annotations

import logging
from collections import Counter, deque

import numpy as np

from .engine import Engine, Resolution

_BLEND = {"metal": 0.7, "rock": 0.7, "jazz": 0.5}
_E2 = 82.41  # chromagram.py:592-599: E2 and the drop tunings' lowest-string references
_TUNINGS = ((0, _E2), (-1, _E2 * 0.944), (-2, _E2 * 0.891), (-3, _E2 * 0.841), (-4, _E2 * 0.794))
logger = logging.getLogger(__name__)


class ChromagramAnalyzer:
    def __init__(self, sample_rate: int = 48000, device: int = 0):
        self.sample_rate = sample_rate
        self.chroma_bins = 12
        self.transposition_offset = 0
        self.chroma_history = deque(maxlen=8)
        self.current_genre = "pop"
        self.tuning_history = []
        self._eng = Engine([Resolution((20, 20000), 512, 256, 1.0)], sample_rate, min(20000, sample_rate / 2),
                           target_bins=2, frame_size=512, device=device)

    def _raw(self, spectra: np.ndarray, freqs: np.ndarray) -> np.ndarray:
        spectra = np.atleast_2d(spectra)
        df = float(freqs[1] - freqs[0]) if len(freqs) > 1 else float(self.sample_rate) / 2
        return self._eng.chroma_raw(spectra, df)

    @staticmethod
    def _find_peaks(data: np.ndarray, prominence: float = 0.3) -> np.ndarray:
        """chromagram.py:641-654."""
        if len(data) < 3:
            return np.array([], int)
        thr = np.max(data) * prominence
        inner = data[1:-1]
        return np.nonzero((inner > data[:-2]) & (inner > data[2:]) & (inner > thr))[0] + 1

    def detect_tuning_offset(self, fft_data: np.ndarray, freqs: np.ndarray) -> int:
        """chromagram.py:581-639: the first 70-100 Hz peak against the tuning references (closest
        within 50 cents, else standard), then the mode of the last 30 detections once there are 5."""
        sel = (freqs > 70) & (freqs < 100)
        bass = np.asarray(fft_data)[sel]
        if len(bass) == 0:
            return self.transposition_offset
        pk = self._find_peaks(bass, 0.3)
        if len(pk) == 0:
            return self.transposition_offset
        pf = freqs[sel][pk[0]]
        best, dmin = 0, float("inf")
        for off, rf in _TUNINGS:
            if pf > 0 and rf > 0:
                d = abs(1200 * np.log2(pf / rf))
                if d < dmin and d < 50:
                    best, dmin = off, d
        self.tuning_history.append(best)
        if len(self.tuning_history) > 30:
            self.tuning_history.pop(0)
        if len(self.tuning_history) >= 5:
            return Counter(self.tuning_history).most_common(1)[0][0]
        return best

    def _offsets(self, spectra: np.ndarray, freqs: np.ndarray) -> np.ndarray:
        """The transposition offset in force for each frame, in order (state advanced)."""
        offs = np.empty(len(spectra), int)
        detect = self.current_genre.lower() in ("metal", "rock")
        for f in range(len(spectra)):
            if detect:
                self.transposition_offset = self.detect_tuning_offset(spectra[f], freqs)
            offs[f] = self.transposition_offset
        return offs

    def _chroma(self, spectra: np.ndarray, freqs: np.ndarray) -> np.ndarray:
        spectra = np.atleast_2d(np.asarray(spectra, np.float32))
        offs = self._offsets(spectra, freqs)
        raw = self._raw(spectra, freqs)
        for f in np.nonzero(offs)[0]:
            raw[f] = np.roll(raw[f], int(offs[f]))
        return raw

    def _blend(self):
        if len(self.chroma_history) == 0:
            return np.zeros(12)
        cur = self.chroma_history[-1]
        if len(self.chroma_history) == 1:
            return cur
        a = _BLEND.get(self.current_genre.lower(), 0.3)
        return self.chroma_history[-2] * (1 - a) + cur * a

    def compute_chromagram(self, fft_data: np.ndarray, freqs: np.ndarray) -> np.ndarray:
        """chromagram.py:109-159. Errors are logged and the last blended chroma returned."""
        try:
            raw = self._chroma(fft_data, np.asarray(freqs))[0]
        except Exception as e:
            logger.error("compute_chromagram failed: %s", e)
            return self._blend()
        self.chroma_history.append(raw.copy())
        return self._blend()

    def compute_chromagram_batch(self, spectra: np.ndarray, freqs: np.ndarray) -> np.ndarray:
        """Frames of one stream in order: [F, K] -> [F, 12] blended chroma, state advanced."""
        raw = self._chroma(spectra, np.asarray(freqs))
        out = np.empty_like(raw)
        for f in range(len(raw)):
            self.chroma_history.append(raw[f].copy())
            out[f] = self._blend()
        return out
