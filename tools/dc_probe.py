"""LUFS_inst error of the float32 K-weighting scan on DC-biased frames (tests/golden/meters_dc.npz,
the reference's calculate_lufs), through the batch launch (omega_process_frames) and kweight_kernel
(omega_k_weighting). Development tool: --lib picks another build (tools/ab_build.sh)."""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "audio-analyzer-omega_amd")]

ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=None)
a = ap.parse_args()
from omega_gpu import _lib as L  # noqa: E402
if a.lib:
    L.use_development_library(a.lib)
import torch  # noqa: E402
from omega_gpu import Engine, NORTHSTAR_RESOLUTIONS, Resolution  # noqa: E402
from oracle import signals as S  # noqa: E402

g = np.load(os.path.join(REPO, "tests", "golden", "meters_dc.npz"))
for name, fr in S.dc_meter_frames().items():
    eng = Engine(NORTHSTAR_RESOLUTIONS, 48000, 20000, target_bins=512, n_channels=1)
    out = eng.process_frames(torch.from_numpy(fr).cuda(), len(fr), 16384, 16384, meters=True)
    torch.cuda.synchronize()
    li = out["lufs_inst"].cpu().numpy()
    e = Engine([Resolution((20, 20000), 512, 256, 1.0)], 48000, 20000, 2, frame_size=512)
    _, li2 = e.k_weighting_scan(fr, weighted=False)
    want = g[f"{name}/lufs_inst"]
    print(f"{a.lib or 'libomega.so'} {name:14s} batch max|dLU| {np.abs(li - want).max():.4f}  "
          f"kweight {np.abs(li2 - want).max():.4f}")
