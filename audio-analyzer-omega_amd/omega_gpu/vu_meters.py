"""VU meter ballistics on the MI355X (SURVEY.md §8(f) row 2 remainder): the processing half of
VUMetersPanel (omega4/panels/vu_meters.py:55-99) -- the 300 ms RMS window, dBFS + 18, needle damping and
the 2 s peak hold -- over libomega.so's omega_vu_update. The reference appends every sample to a deque in
a Python loop (one of the per-sample hot loops of SURVEY.md §3); here a batch of update calls is one
device launch sequence (window mean squares in parallel, then the damping / hold recurrence).

``VUMeters.update(audio_data, dt)`` keeps the panel's attribute names (mono input drives both needles,
as in the reference); ``update_batch(frames [n, C, chunk], dts)`` runs n consecutive updates of C
independent channels and returns [n, C, 3] (level, display, peak). Drawing stays with the panel.
"""
from __future__ import annotations

import ctypes as C
import logging

import numpy as np

from . import _lib as L
from .engine import Engine, Resolution, _is_torch

logger = logging.getLogger(__name__)


class VUMeters:
    def __init__(self, sample_rate: int = 48000, n_channels: int = 1, device: int = 0):
        self.sample_rate = sample_rate
        self.vu_integration_time = 300e-3
        self.vu_damping = 0.94
        self.vu_reference_level = 0.125
        self.vu_peak_hold_time = 2.0
        self.n_channels = n_channels
        self._eng = Engine([Resolution((20, 20000), 512, 256, 1.0)], sample_rate, min(20000, sample_rate / 2),
                           target_bins=2, frame_size=512, n_channels=n_channels, device=device)
        self._last = np.tile([-60.0, -60.0, -60.0], (n_channels, 1))
        self._publish()

    def _publish(self):
        lv, rv = self._last[0], self._last[min(1, self.n_channels - 1)]
        self.vu_left_db, self.vu_left_display, self.vu_left_peak_db = (float(v) for v in lv)
        self.vu_right_db, self.vu_right_display, self.vu_right_peak_db = (float(v) for v in rv)

    def update_batch(self, frames, dts) -> np.ndarray:
        """frames [n, C, chunk] (float32 or float64, host numpy or device torch), dts [n] seconds ->
        [n, C, 3] float64: level (dBFS + 18), damped display, peak hold; state advanced."""
        dev = _is_torch(frames)
        if not dev:
            frames = np.asarray(frames)
            if frames.dtype not in (np.float32, np.float64):
                frames = frames.astype(np.float32)
            frames = np.ascontiguousarray(frames)
        n, c, m = frames.shape
        if c != self.n_channels:
            raise ValueError(f"{self.n_channels} channels expected, got {c}")
        f64 = 1 if str(frames.dtype).endswith("float64") else 0
        dts = np.array(np.broadcast_to(np.asarray(dts, np.float64), (n,)))
        if dev:
            import torch
            dt_dev = torch.as_tensor(dts, device=frames.device)
            out = torch.empty((n, c, 3), dtype=torch.float64, device=frames.device)
            self._eng._bind_stream(frames)
            self._eng._check(L.lib().omega_vu_update(self._eng._ctx, frames.data_ptr(), f64, n, m, frames.stride(0),
                                                     frames.stride(1), dt_dev.data_ptr(), out.data_ptr(), L.MEM_DEVICE))
            return out
        out = np.empty((n, c, 3), np.float64)
        self._eng._check(L.lib().omega_vu_update(self._eng._ctx, frames.ctypes.data, f64, n, m, c * m, m,
                                                 dts.ctypes.data, out.ctypes.data, L.MEM_HOST))
        if n:
            self._last = out[-1].copy()
            self._publish()
        return out

    def update(self, audio_data, dt: float):
        """vu_meters.py:55-99 for one call; errors are logged and the previous values kept."""
        if audio_data is None or len(audio_data) == 0:
            return
        try:
            x = np.asarray(audio_data)
            x = x if x.dtype in (np.float32, np.float64) else x.astype(np.float32)
            self.update_batch(np.broadcast_to(x, (1, self.n_channels, len(x))), [dt])
        except Exception as e:
            logger.error("VUMeters.update failed: %s", e)

    def reset(self):
        self._eng._check(L.lib().omega_vu_reset(self._eng._ctx))
        self._last = np.tile([-60.0, -60.0, -60.0], (self.n_channels, 1))
        self._publish()
