#!/usr/bin/env python3
"""App post-processing outputs of one build, for bitwise A/B of post.hip variants:
python tools/post_outputs.py [--lib libomega_x.so] --out f.npz (random, tied and short frames)."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "audio-analyzer-omega_amd"))
import numpy as np  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=None)
ap.add_argument("--out", required=True)
a = ap.parse_args()
from omega_gpu import _lib as L  # noqa: E402
if a.lib:
    L.use_development_library(a.lib)
from omega_gpu.app_post import SpectrumPostProcessor  # noqa: E402

rng = np.random.default_rng(21)
res = {}
for T in (512, 300, 40, 1024):
    x = (rng.random((600, T)) * rng.random((600, 1)) ** 2).astype(np.float32)
    x[::7] = (np.round(x[::7] * 8) / 8).astype(np.float32)
    x[1::7, : T // 2] = -0.0
    x[2::7] = rng.standard_normal((len(x[2::7]), T)).astype(np.float32)
    s, b, c = SpectrumPostProcessor(np.linspace(20, 20000, T)).process(x)
    res[f"s{T}"], res[f"b{T}"], res[f"c{T}"] = s, b, c
np.savez(a.out, **res)
print("saved", a.out)
