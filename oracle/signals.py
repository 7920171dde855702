"""Deterministic synthetic inputs shared by the golden generator, the tests and bench.py's
cpu_baseline leg (SURVEY.md §8(c) recipe step 1, §8(d) config table).

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``). bench.py builds the device-side workload
with the same formulas so that its CPU-baseline sample sees identical frames.
"""
from __future__ import annotations

import numpy as np

FS = 48000


def sine(freq: float, amp: float, n: int, fs: float = FS, start: int = 0) -> np.ndarray:
    t = (np.arange(n) + start) / fs
    return (amp * np.sin(2 * np.pi * freq * t)).astype(np.float32)


def noise(seed: int, n: int, scale: float = 1.0) -> np.ndarray:
    return (scale * np.random.default_rng(seed).standard_normal(n)).astype(np.float32)


def triad(n: int, amp: float = 1.0, fs: float = FS) -> np.ndarray:
    """C-major triad as in test_chromagram_fix.py:28-32 (on an arange time base)."""
    t = np.arange(n) / fs
    x = np.sin(2 * np.pi * 261.63 * t) + np.sin(2 * np.pi * 329.63 * t) + np.sin(2 * np.pi * 392.00 * t)
    return (amp * x).astype(np.float32)


def composite(n: int, seed: int = 7, fs: float = FS) -> np.ndarray:
    """test_enhanced_meters.py:10-38: 1 kHz @0.1 + 100 Hz @0.03 + 10 kHz @0.01 + 10-sample click at
    100 ms + 0.001 noise (seeded here; the reference used the global RNG)."""
    t = np.arange(n) / fs
    x = 0.1 * np.sin(2 * np.pi * 1000 * t) + 0.03 * np.sin(2 * np.pi * 100 * t) \
        + 0.01 * np.sin(2 * np.pi * 10000 * t)
    k = int(0.1 * fs)
    if k < n:
        x[k:k + 10] = x[k:k + 10] + 0.5
    x = x + 0.001 * np.random.default_rng(seed).standard_normal(n)
    return x.astype(np.float32)


def square(n: int, amp: float = 0.9, freq: float = 1000, fs: float = FS) -> np.ndarray:
    """test_enhanced_meters.py:66-71 (0.9-amplitude 1 kHz square)."""
    t = np.arange(n) / fs
    return (amp * np.sign(np.sin(2 * np.pi * freq * t))).astype(np.float32)


def cfg2_batch(frames: int, w: int = 16384, seed_l: int = 0, seed_r: int = 1) -> np.ndarray:
    """BASELINE cfg2 materialized input f32[frames, 2, W]: consecutive frames of
    L = 0.25 sin(2 pi 440 t) + 0.05 N(0,1) (seed 0), R = 0.25 sin(2 pi 997 t) + 0.05 N(0,1) (seed 1)."""
    n = frames * w
    left = sine(440, 0.25, n) + noise(seed_l, n, 0.05)
    right = sine(997, 0.25, n) + noise(seed_r, n, 0.05)
    return np.stack([left.reshape(frames, w), right.reshape(frames, w)], axis=1).astype(np.float32)


def cfg3_batch(frames: int, w: int = 8192, seed: int = 1234) -> np.ndarray:
    """BASELINE cfg3 input f32[frames, W]: frames alternate a 0.5 C-major triad and 0.1 N(0,1)."""
    out = np.empty((frames, w), np.float32)
    tri = triad(w, 0.5)
    nz = noise(seed, (frames // 2 + 1) * w, 0.1).reshape(-1, w)
    for f in range(frames):
        out[f] = tri if f % 2 == 0 else nz[f // 2]
    return out


def level_steps(frames: int, m: int, seed: int = 3) -> np.ndarray:
    """A meter stream whose level moves between loud, quiet and silent frames so the -70 LUFS
    gate, the 24/180/3600 windows and the 60-frame peak hold all see changes
    (test_enhanced_meters.py:82-180 style level steps + gating)."""
    rng = np.random.default_rng(seed)
    base = noise(seed + 100, frames * m, 1.0).reshape(frames, m)
    lv = np.empty(frames, np.float32)
    for f in range(frames):
        ph = (f // 37) % 5
        lv[f] = (0.3, 0.03, 0.0, 0.0001, 0.9)[ph] * (1 + 0.1 * rng.random())
    return (base * lv[:, None]).astype(np.float32)


def cfg5_stream(n: int, channels: int = 8, fs: float = 96000) -> np.ndarray:
    """BASELINE cfg5 surround stream, planar [C, n] float32: channel c =
    0.2 sin(2 pi 110 (c + 1) t) + 0.02 N(0, 1) (seed c)."""
    t = np.arange(n) / fs
    return np.stack([(0.2 * np.sin(2 * np.pi * 110 * (c + 1) * t)).astype(np.float32) + noise(c, n, 0.02)
                     for c in range(channels)]).astype(np.float32)


def dc_meter_frames(n: int = 8, m: int = 16384) -> dict:
    """DC-biased 16384-sample meter frames (the capture path passes raw samples with no DC removal,
    capture.py:571-574, :620-641): large constant offsets under low-level content, where a float32
    IIR's state rounding at the DC level is amplified by the high-pass poles (radius ~0.9965).
    Returns {name: f32[n, m]}; ``hann_dc05`` is the app's Hann-windowed form (omega4_main.py:1082)
    rounded to float32 (its float64 product is ``dc05_n1e3 * np.hanning(m)``)."""
    t = np.arange(n * m)
    rng = np.random.default_rng(77)
    seqs = {
        "dc09_n1e4": 0.9 + 1e-4 * rng.standard_normal(n * m),
        "dc05_n1e3": 0.5 + 1e-3 * rng.standard_normal(n * m),
        "dcm07_n3e4": -0.7 + 3e-4 * rng.standard_normal(n * m),
        "dc03_sine": 0.3 + 0.25 * np.sin(2 * np.pi * 997 * t / FS) + 1e-3 * rng.standard_normal(n * m),
        "dc09_sine1e3": 0.9 + 1e-3 * np.sin(2 * np.pi * 60 * t / FS),
        # a step of the offset inside frame 3
        "dc_step": np.where(t < 3 * m + 5000, 0.2, 0.8) + 2e-4 * rng.standard_normal(n * m),
    }
    out = {k: v.astype(np.float32).reshape(n, m) for k, v in seqs.items()}
    out["hann_dc05"] = (out["dc05_n1e3"].astype(np.float64) * np.hanning(m)).astype(np.float32)
    return out
