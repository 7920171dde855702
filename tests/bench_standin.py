"""CPU stand-in compute backend for bench.py (test infrastructure only): `bench.py --standin
tests.bench_standin` runs bench's own launcher, step loop, packed-output layout and gather over gloo
with the oracle computing each rank's channel-frames, so the N>1 path is exercised without a GPU
(tests/test_bench_launch.py). Never used by a measurement."""
import numpy as np
import torch

from oracle import omega_ref as R
from oracle import signals as S

FS = 48000


class Backend:
    dist_backend = "gloo"

    def __init__(self, local):
        self.dev = torch.device("cpu")
        self.states = {}

    def input(self, frames, seed_l, seed_r):
        return torch.from_numpy(S.cfg2_batch(frames, seed_l=seed_l, seed_r=seed_r))

    def alloc(self, layout):
        return layout.alloc(self.dev)

    def reset(self):
        self.states = {}

    def process(self, x, frames, out):
        xn = x.numpy()
        C = xn.shape[1]
        for f in range(frames):
            for c in range(C):
                cf = f * C + c
                _, comb, li, tp = R.full_frame(xn[f, c])
                m = self.states.setdefault(c, R.MeterState(FS)).update(xn[f, c], li, tp)
                out["combined"][cf] = torch.from_numpy(np.asarray(comb, np.float32))
                out["lufs_inst"][cf] = float(li)
                out["true_peak_db"][cf] = float(tp)
                out["meters"][cf] = torch.tensor([m[k] for k in R.AGG_KEYS], dtype=torch.float64)

    def sync(self):
        pass
