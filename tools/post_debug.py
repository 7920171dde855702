#!/usr/bin/env python3
"""Dump omega_post_process outputs for the app_post golden configs (GPU box) to gpurun_out/post_<cfg>.npz
for offline comparison with the golden frames and the numpy emulation."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "audio-analyzer-omega_amd"))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402

from omega_gpu.app_post import SpectrumPostProcessor  # noqa: E402

CFG = {"default": {}, "vocal_supp_norm": dict(vocal_suppression=0.4, normalization_enabled=True),
       "flat": dict(psychoacoustic_enabled=False, freq_compensation_enabled=False, smoothing_enabled=False)}
g = np.load(os.path.join(REPO, "tests", "golden", "app_post.npz"))
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
for name, kw in CFG.items():
    pp = SpectrumPostProcessor(g[f"{name}/freqs"], **kw)
    s, b, c = pp.process(g[f"{name}/combined"])
    np.savez(os.path.join(REPO, "gpurun_out", f"post_{name}.npz"), spectrum=s, bands=b, content=c)
    print(name, "mismatch", int((s != g[f"{name}/spectrum"]).sum()))
