#!/usr/bin/env python3
"""Time bench.py's cfg1 line alone, after the cfg3 line, and with extra live engines (why the
full bench's cfg1 number differs from cfg1 alone).

  python tools/side_order_probe.py [lib]   (lib: another build in lib/, e.g. libomega_ab.so)
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "audio-analyzer-omega_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

if len(sys.argv) > 1:
    from omega_gpu import _lib as _L
    _L.use_development_library(sys.argv[1])
import bench  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    print("cfg1 alone        ", round(bench.cfg1_line(dev, cpu=False)["ms_per_call"], 4), "ms", flush=True)
    from omega_gpu import Engine, NORTHSTAR_RESOLUTIONS
    engs = []
    for k in range(3):
        engs.append(Engine(NORTHSTAR_RESOLUTIONS, 48000, 20000, target_bins=512, n_channels=2))
        print(f"cfg1 + {k + 1} engines ", round(bench.cfg1_line(dev, cpu=False)["ms_per_call"], 4), "ms", flush=True)
    del engs
    c3 = bench.cfg3_line(dev)
    print("cfg3              ", round(c3["ms_per_batch"], 4), "ms", flush=True)
    print("cfg1 after cfg3   ", round(bench.cfg1_line(dev, cpu=False)["ms_per_call"], 4), "ms", flush=True)
    import gc
    gc.collect()
    torch.cuda.empty_cache()
    print("cfg1 after gc     ", round(bench.cfg1_line(dev, cpu=False)["ms_per_call"], 4), "ms", flush=True)


if __name__ == "__main__":
    main()
