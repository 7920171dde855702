"""TransientAnalyzer on the MI355X: analyze_transients
(omega4/analyzers/transient.py:19-108) -- Hilbert envelope, Savitzky-Golay (21, 3) smoothing, derivative
threshold, attack time and punch factor -- over libomega.so's omega_transients, in float64 like the
reference's scipy path. ``analyze_transients(frame)`` returns the reference's dict and appends the
smoothed envelope's mean to ``envelope_history`` (:17, :33); ``analyze_batch(frames)`` does a batch of
one stream's frames in one launch (history advanced in order).
"""
from __future__ import annotations

import logging
from collections import deque
from typing import Any, Dict, List

import numpy as np

from . import _lib as L
from .engine import Engine, Resolution, _is_torch

logger = logging.getLogger(__name__)
COLUMNS = ("transients_detected", "attack_time", "punch_factor", "envelope_peak", "envelope_rms", "envelope_mean")


class TransientAnalyzer:
    def __init__(self, sample_rate: int = 48000, device: int = 0):
        self.sample_rate = sample_rate
        self.envelope_history = deque(maxlen=int(0.5 * 60))
        self._eng = Engine([Resolution((20, 20000), 512, 256, 1.0)], sample_rate, min(20000, sample_rate / 2),
                           target_bins=2, frame_size=512, device=device)

    def analyze_batch(self, frames) -> np.ndarray:
        """frames [F, n] (float32 / float64; host numpy or device torch) -> [F, 6] float64 in COLUMNS order."""
        dev = _is_torch(frames)
        if not dev:
            frames = np.asarray(frames)
            frames = np.ascontiguousarray(frames if frames.dtype in (np.float32, np.float64) else frames.astype(np.float64))
        if frames.ndim != 2:
            raise ValueError("frames must be [F, n]")
        F, n = frames.shape
        f64 = 1 if str(frames.dtype).endswith("float64") else 0
        if dev:
            import torch
            out = torch.empty((F, len(COLUMNS)), dtype=torch.float64, device=frames.device)
            self._eng._bind_stream(frames)
            self._eng._check(L.lib().omega_transients(self._eng._ctx, frames.data_ptr(), f64, F, n, frames.stride(0),
                                                      out.data_ptr(), L.MEM_DEVICE))
            hist = out[:, 5].cpu().numpy()
        else:
            out = np.empty((F, len(COLUMNS)), np.float64)
            self._eng._check(L.lib().omega_transients(self._eng._ctx, frames.ctypes.data, f64, F, n, n,
                                                      out.ctypes.data, L.MEM_HOST))
            hist = out[:, 5]
        self.envelope_history.extend(float(v) for v in hist)
        return out

    def analyze_transients(self, audio_data: np.ndarray) -> Dict[str, Any]:
        """transient.py:19-55. Frames shorter than 64 samples give the reference's zero dict; errors are
        logged and give it too (the reference's analysis never raises here)."""
        if len(audio_data) < 64:
            return {"transients_detected": 0, "attack_time": 0.0, "punch_factor": 0.0}
        try:
            o = self.analyze_batch(np.asarray(audio_data)[None, :])[0]
        except Exception as e:
            logger.error("analyze_transients failed: %s", e)
            return {"transients_detected": 0, "attack_time": 0.0, "punch_factor": 0.0}
        return {"transients_detected": int(o[0]), "attack_time": float(o[1]), "punch_factor": float(o[2]),
                "envelope_peak": float(o[3]), "envelope_rms": float(o[4])}

    def get_envelope_history(self) -> List[float]:
        return list(self.envelope_history)
