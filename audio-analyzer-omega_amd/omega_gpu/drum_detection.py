"""Drum-detection spectral features on the MI355X: the data-parallel part of
omega4/analyzers/drum_detection.py -- EnhancedKickDetector band flux (:47-67) + adaptive thresholds
(:69-78) over 20-60 / 60-120 / 2000-5000 Hz (:20-22, :85-103) and EnhancedSnareDetector band flux
(:231-266) over 150-400 / 400-1000 / 2000-8000 / 8000-15000 Hz, thresholds (:290-305) and spectral
centroid (:212-229) -- computed for a whole block of consecutive frames of one stream in two kernel
launches (omega_drum_features). The onset decisions and display persistence read the wall clock
(time.time(), :82, :270) and stay with the caller.
"""
from __future__ import annotations

from typing import Dict

import numpy as np

from .engine import Engine

COLUMNS = ("kick_sub_flux", "kick_body_flux", "kick_click_flux",
           "kick_sub_threshold", "kick_body_threshold", "kick_click_threshold",
           "snare_fundamental_flux", "snare_body_flux", "snare_snap_flux", "snare_rattle_flux",
           "snare_fundamental_threshold", "snare_body_threshold", "snare_snap_threshold",
           "snare_centroid")


class DrumFeatures:
    """One stream's kick + snare features. ``process(mags)`` takes [F, n_bins] magnitude frames (the
    spectra the reference's detectors receive, one per call there) and returns [F, 14] float64 in
    COLUMNS order; state (previous frame, 21-deep flux histories) carries over between calls."""

    def __init__(self, sample_rate: int = 48000, sensitivity: float = 1.0, device: int = 0):
        self.sample_rate = sample_rate
        self.sensitivity = sensitivity
        # any valid engine config: only the sample rate matters to the drum features
        self._eng = Engine(sample_rate=sample_rate, device=device)

    def process(self, mags) -> np.ndarray:
        mags = np.atleast_2d(mags) if isinstance(mags, np.ndarray) else mags
        return self._eng.drum_features(mags, self.sensitivity)

    def process_dict(self, mags) -> Dict[str, np.ndarray]:
        o = self.process(mags)
        return {k: o[:, i] for i, k in enumerate(COLUMNS)}

    def reset(self):
        self._eng.reset_drums()
