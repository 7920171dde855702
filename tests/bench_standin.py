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
    # meter pipelining as the device does it (omega_set_meter_pipelining): a call's meter aggregates
    # land in its buffer during the NEXT call (or flush), so bench.py's gather of a step must follow the
    # next step's launch -- a wrong lag shows up as stale meters in the gathered blocks
    pipelined = True

    def __init__(self, local):
        self.dev = torch.device("cpu")
        self.states = {}
        self.pend = None

    def input(self, frames, seed_l, seed_r):
        return torch.from_numpy(S.cfg2_batch(frames, seed_l=seed_l, seed_r=seed_r))

    def alloc(self, layout):
        return layout.alloc(self.dev)

    def reset(self):
        self.flush()
        self.states = {}

    def flush(self):
        if self.pend is not None:
            dst, vals = self.pend
            dst.copy_(vals)
            self.pend = None

    def process(self, x, frames, out):
        self.flush()
        xn = x.numpy()
        C = xn.shape[1]
        met = torch.empty_like(out["meters"])
        out["meters"].fill_(float("nan"))  # (not yet: the next call writes them)
        for f in range(frames):
            for c in range(C):
                cf = f * C + c
                _, comb, li, tp = R.full_frame(xn[f, c])
                m = self.states.setdefault(c, R.MeterState(FS)).update(xn[f, c], li, tp)
                out["combined"][cf] = torch.from_numpy(np.asarray(comb, np.float32))
                out["lufs_inst"][cf] = float(li)
                out["true_peak_db"][cf] = float(tp)
                met[cf] = torch.tensor([m[k] for k in R.AGG_KEYS], dtype=torch.float64)
        self.pend = (out["meters"], met)

    def sync(self):
        pass
