"""ChromagramAnalyzer.compute_chromagram over libomega.so (omega4/panels/chromagram.py:109-237).

The per-frame work (harmonic suppression, the 12 x K Gaussian pitch-class projection, smoothing,
normalisation) runs on the device; the genre-dependent temporal blend with the previous frame
(:215-237) is 12 multiply-adds and stays with the stateful caller object, as in the reference.
Key/chord/mode detection (:239-935) is out of scope (scalar host logic on 12 numbers).
"""
from __future__ import annotations

from collections import deque

import numpy as np

from .engine import Engine, Resolution

_BLEND = {"metal": 0.7, "rock": 0.7, "jazz": 0.5}


class ChromagramAnalyzer:
    def __init__(self, sample_rate: int = 48000, device: int = 0):
        self.sample_rate = sample_rate
        self.chroma_bins = 12
        self.transposition_offset = 0
        self.chroma_history = deque(maxlen=8)
        self.current_genre = "pop"
        self._eng = Engine([Resolution((20, 20000), 512, 256, 1.0)], sample_rate, min(20000, sample_rate / 2),
                           target_bins=2, frame_size=512, device=device)

    def _raw(self, spectra: np.ndarray, freqs: np.ndarray) -> np.ndarray:
        spectra = np.atleast_2d(spectra)
        df = float(freqs[1] - freqs[0]) if len(freqs) > 1 else float(self.sample_rate) / 2
        if self.current_genre.lower() in ("metal", "rock"):
            # the tuning-offset path (chromagram.py:112-113) shifts the pitch map per frame
            raise NotImplementedError("metal/rock tuning detection is not implemented on the device")
        return self._eng.chroma_raw(spectra, df)

    def _blend(self):
        if len(self.chroma_history) == 0:
            return np.zeros(12)
        cur = self.chroma_history[-1]
        if len(self.chroma_history) == 1:
            return cur
        a = _BLEND.get(self.current_genre.lower(), 0.3)
        return self.chroma_history[-2] * (1 - a) + cur * a

    def compute_chromagram(self, fft_data: np.ndarray, freqs: np.ndarray) -> np.ndarray:
        """chromagram.py:109-159."""
        raw = self._raw(np.asarray(fft_data, np.float32), freqs)[0]
        self.chroma_history.append(raw.copy())
        return self._blend()

    def compute_chromagram_batch(self, spectra: np.ndarray, freqs: np.ndarray) -> np.ndarray:
        """Frames of one stream in order: [F, K] -> [F, 12] blended chroma, state advanced."""
        raw = self._raw(np.asarray(spectra, np.float32), freqs)
        out = np.empty_like(raw)
        for f in range(len(raw)):
            self.chroma_history.append(raw[f].copy())
            out[f] = self._blend()
        return out
