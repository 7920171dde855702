import sys, os, json
sys.path.insert(0, "/root/repo/audio-analyzer-omega_amd"); sys.path.insert(0, "/root/repo")
import torch, bench
from omega_gpu import Engine, Resolution
from omega_gpu import _lib as L
from omega_gpu.engine import BandTable
x = torch.from_numpy(bench.cfg3_input(4096, 8192)).cuda()
e3 = Engine([Resolution((20, 20000), 8192, 2048, 1.0)], 48000, 20000, 512)
st_, en_, comp_ = bench.band_table_512()
bt = BandTable(e3, L.BANDS_MAX, st_, en_, 512, 4097, scale=comp_)
for n in (256, 512, 768, 1024, 1280, 2048, 3072, 4096):
    xs = x[:n]
    so = {"bands": torch.empty(n, 512, device="cuda"), "chroma": torch.empty(n, 12, dtype=torch.float64, device="cuda")}
    for chroma in (True, False):
        for _ in range(3): e3.spectra(xs, "hann", bands=bt, chroma=chroma, out=so)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20): e3.spectra(xs, "hann", bands=bt, chroma=chroma, out=so)
        e.record(); torch.cuda.synchronize()
        print(n, "chroma" if chroma else "bands", round(s.elapsed_time(e) / 20 * 1e3, 1), "us", flush=True)
