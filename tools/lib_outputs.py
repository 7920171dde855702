"""Outputs of one build over three consecutive cfg2 batches with meters, direct and pipelined (and a 1500-frame cfg4 shard),
saved for a bitwise comparison between builds (tools/ab.sh: a scheduling variant must not change a
single bit). Development tool: --lib picks another build in lib/."""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "audio-analyzer-omega_amd")]
ap = argparse.ArgumentParser()
ap.add_argument("--lib", default=None)
ap.add_argument("--out", required=True)
a = ap.parse_args()
from omega_gpu import _lib as L  # noqa: E402
if a.lib:
    L.use_development_library(a.lib)
import torch  # noqa: E402
from omega_gpu import Engine, NORTHSTAR_RESOLUTIONS  # noqa: E402
from oracle import signals as S  # noqa: E402

res = {}
x = torch.from_numpy(S.cfg2_batch(768)).cuda()
eng = Engine(NORTHSTAR_RESOLUTIONS, 48000, 20000, target_bins=512, n_channels=2)
for i in range(3):
    o = eng.process_frames(x[256 * i:256 * (i + 1)], 256, 2 * 16384, 16384, meters=True)
    for k, v in o.items():
        res[f"{k}{i}"] = v.cpu().numpy()
# the same batches through a pipelined context (each call's meter segment runs in the next launch):
# every output, including the deferred meters once flushed
eng = Engine(NORTHSTAR_RESOLUTIONS, 48000, 20000, target_bins=512, n_channels=2)
eng.set_meter_pipelining(True)
outs = [eng.process_frames(x[256 * i:256 * (i + 1)], 256, 2 * 16384, 16384, meters=True) for i in range(3)]
eng.synchronize()
for i, o in enumerate(outs):
    for k, v in o.items():
        res[f"{k}{i}_pipe"] = v.cpu().numpy()
x4 = torch.from_numpy(S.cfg2_batch(1500, seed_l=4, seed_r=5)).cuda()
o = Engine(NORTHSTAR_RESOLUTIONS, 48000, 20000, target_bins=512, n_channels=2).process_frames(
    x4, 1500, 2 * 16384, 16384, meters=True)
for k, v in o.items():
    res[f"{k}_big"] = v.cpu().numpy()
np.savez(a.out, **res)
print("saved", a.out, len(res))
