#!/usr/bin/env python3
"""Benchmark: BASELINE cfg2 -- per GPU, 256 stereo frames x 16384 samples (512 channel-frames), the
full hot path per step: 16k/8k/4k/1k multi-resolution FFT + weighting + combine(512), K-weighted
LUFS, 4x true peak and the meter aggregates. One process per GPU; frames shard
across ranks (weak scaling) and each step's per-frame outputs are gathered to rank 0 over RCCL
(overlapped with the next step). Prints ONE JSON line on rank 0.

  python bench.py [--gpus N] [--steps K] [--warmup W]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

With --gpus N > 1 and no WORLD_SIZE in the environment, this process starts the N rank processes
itself (before touching any GPU) and exits with their status. Every run also measures cfg4's per-GPU
shard (4096 stereo frames per GPU = BASELINE cfg4's 32768 at N = 8) as the `cfg4` object.
"""
import argparse
import importlib
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "audio-analyzer-omega_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

FS = 48000
W = 16384
FRAMES = 256          # stereo frames per GPU (BASELINE cfg2)
FRAMES_CFG4 = 4096    # stereo frames per GPU (BASELINE cfg4: 32768 over 8 GPUs)
C = 2
T = 512
PEAK_FP32_TFLOPS = 157.3   # MI355X_MICROARCH.md: FP32 vector peak
PEAK_HBM_GBS = 8000.0
# SURVEY.md §8(d), per channel-frame (cfg2)
FLOP_TP = 2.5 * W * np.log2(W) + 2.5 * 4 * W * np.log2(4 * W) + 8 * W          # 3.33 MFLOP (reference algorithm)
FLOP_FFT = sum(2.5 * n * np.log2(n) + 3.5 * n for n in (16384, 8192, 4096, 1024))  # 1.09 MFLOP
FLOP_KW = 4 * (W + 18) * 9 + 5 * W                                                 # 0.67 MFLOP
# the true peak as the kernel executes it (polyphase form, rfkern.hip): four K = W/2-point complex FFTs
# (5 K log2 K each: the forward rfft and three phase inverses), three phase rotations + Hermitian packs
# (16 flops per bin), one untangle (10 per bin) -- 2.60 MFLOP against the reference algorithm's 3.33
FLOP_TP_EXEC = 4 * 5 * (W // 2) * np.log2(W // 2) + 3 * 16 * (W // 2) + 10 * (W // 2)
BYTES_CF = 4 * W + 4 * (T + 2)                                                     # 67,592 B
METRIC = "audio frames/sec (multi-res FFT + LUFS + TruePeak) at 1/2/4/8 MI355X"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU-baseline budget (rank 0, N=1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-procs", type=int, default=min(16, os.cpu_count() or 1),
                    help="processes of the all-cores CPU baseline (the GPU box's CPU share is 16)")
    ap.add_argument("--no-cfg3", action="store_true", help="skip the cfg3 / drums / app_post lines")
    ap.add_argument("--no-cfg4", action="store_true", help="skip the cfg4 per-GPU-shard line")
    ap.add_argument("--cfg4-steps", type=int, default=20)
    ap.add_argument("--no-rotating", action="store_true", help="skip the rotating-input variant of the headline")
    ap.add_argument("--no-cfg5", action="store_true", help="skip the cfg5 sustained-stream line")
    ap.add_argument("--cfg5-seconds", type=float, default=60.0)
    # test hooks (tests/test_bench_launch.py): a stand-in compute backend on the CPU over gloo, a
    # smaller per-rank batch, and rank 0 dumping the last gathered blocks
    ap.add_argument("--standin", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--frames", type=int, default=FRAMES, help=argparse.SUPPRESS)
    ap.add_argument("--dump", default=None, help=argparse.SUPPRESS)
    return ap.parse_args(argv)


def cfg2_input(frames=FRAMES, w=W, seed_l=0, seed_r=1):
    """BASELINE cfg2 synthetic input f32[frames, 2, W]: consecutive frames of
    L = 0.25 sin(2 pi 440 t) + 0.05 N(0,1), R = 0.25 sin(2 pi 997 t) + 0.05 N(0,1) (seeded). Same formula
    as oracle/signals.cfg2_batch (checked equal in tests/test_bench_contract.py)."""
    n = frames * w
    t = np.arange(n) / FS
    left = (0.25 * np.sin(2 * np.pi * 440 * t)).astype(np.float32) + \
        (0.05 * np.random.default_rng(seed_l).standard_normal(n)).astype(np.float32)
    right = (0.25 * np.sin(2 * np.pi * 997 * t)).astype(np.float32) + \
        (0.05 * np.random.default_rng(seed_r).standard_normal(n)).astype(np.float32)
    return np.stack([left.reshape(frames, w), right.reshape(frames, w)], axis=1).astype(np.float32)


def cfg5_input(n, channels=8, fs=96000):
    """BASELINE cfg5 surround stream, planar [C, n]: channel c = 0.2 sin(2 pi 110 (c + 1) t)
    + 0.02 N(0, 1) (seed c). Same formula as oracle/signals.cfg5_stream (tests/test_bench_contract.py)."""
    t = np.arange(n) / fs
    return np.stack([(0.2 * np.sin(2 * np.pi * 110 * (c + 1) * t)).astype(np.float32) +
                     (0.02 * np.random.default_rng(c).standard_normal(n)).astype(np.float32)
                     for c in range(channels)]).astype(np.float32)


# ---------------------------------------------------------------------------------------------
# rank launcher
# ---------------------------------------------------------------------------------------------


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n, argv):
    """Start n rank processes of this script (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* as
    torch.distributed.run sets them, rendezvous on 127.0.0.1) and return the first non-zero exit
    status, or 0. Called before this process touches any GPU; a failing rank stops the others."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 128 - code
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


# ---------------------------------------------------------------------------------------------
# compute backends: the product path (libomega on this rank's GPU) -- tests inject a CPU stand-in
# ---------------------------------------------------------------------------------------------


class DeviceBackend:
    """libomega.so on this rank's MI355X through the omega_gpu Engine (the product path)."""

    dist_backend = "nccl"

    def __init__(self, local):
        torch.cuda.set_device(local)
        self.dev = torch.device("cuda", local)
        from omega_gpu import NORTHSTAR_RESOLUTIONS, Engine
        self.eng = Engine(NORTHSTAR_RESOLUTIONS, FS, 20000, target_bins=T, n_channels=C, device=local)

    def input(self, frames, seed_l, seed_r):
        return torch.from_numpy(cfg2_input(frames, W, seed_l=seed_l, seed_r=seed_r)).to(self.dev)

    def alloc(self, layout):
        return layout.alloc(self.dev)

    # meter pipelining (omega_set_meter_pipelining): each step's launch computes the previous step's
    # meter aggregates first in its grid; measure() gathers a step's block after the next launch and
    # flushes the last step's meters inside the timed region
    pipelined = True

    def reset(self):
        self.eng.reset_meters()
        self.eng.set_meter_pipelining(self.pipelined)

    def flush(self):
        self.eng.flush_meters()

    def process(self, x, frames, out):
        self.eng.process_frames(x, frames, C * W, W, meters=True, out=out)

    def sync(self):
        torch.cuda.synchronize(self.dev)

    def check_queues(self):
        # RCCL's streams exist now (communicator init, the warmup's gathers): re-probe that the
        # context's stream and its side stream still sit on different hardware queues
        if not self.eng.check_queues():
            print(f"bench.py: {self.dev}: the side stream shares a hardware queue (omega_check_queues)",
                  file=sys.stderr)


def prepare(be, rank, world, frames, seed_base=None):
    """The inputs and output buffers of one measurement, made ahead of it (see main: no GPU idle between
    the cfg4 line and the headline)."""
    from omega_gpu import dist as D
    sb = 2 * rank if seed_base is None else seed_base
    x = be.input(frames, sb, sb + 1)
    lay = D.PackedLayout(frames * C, T)
    bufs = [be.alloc(lay) for _ in range(2)]
    recv = [[be.alloc(lay) for _ in range(world)] if rank == 0 else None for _ in range(2)]
    return x, lay, bufs, recv


def measure(be, rank, world, frames, steps, warmup, gather, seed_base=None, prep=None):
    """Time `steps` passes of the hot path over this rank's batch of `frames` stereo frames (after
    `warmup` untimed ones), each step's packed outputs gathered to rank 0 asynchronously
    (double-buffered: step i waits only for the gather of step i - 2). Returns (max-over-ranks
    seconds, rank 0's last gathered blocks or None, layout)."""
    from omega_gpu import dist as D
    x, lay, bufs, recv = prep if prep is not None else prepare(be, rank, world, frames, seed_base)
    # x: one resident batch, or a list of distinct batches rotated per step (the cache-cold variant)
    xs = x if isinstance(x, (list, tuple)) else [x]
    views = [lay.views(b) for b in bufs]
    pending = [None, None]
    be.reset()
    # pipelined meters: step i's block is complete once step i + 1's launch (or the flush) is enqueued
    lag = 1 if getattr(be, "pipelined", False) else 0

    def step(i, first):
        b = i % 2
        if pending[b] is not None:
            pending[b].wait()
            pending[b] = None
        be.process(xs[i % len(xs)], frames, views[b])
        j = i - lag
        if gather and j >= first:
            pending[j % 2] = D.gather_to_root(bufs[j % 2], recv[j % 2], async_op=True)

    def drain(last):
        if lag:  # the last step's meters, then its gather
            be.flush()
            if gather:
                pending[last % 2] = D.gather_to_root(bufs[last % 2], recv[last % 2], async_op=True)
        for k in range(2):
            if pending[k] is not None:
                pending[k].wait()
                pending[k] = None

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()
        be.sync()

    for i in range(warmup):
        step(i, 0)
    if warmup:
        drain(warmup - 1)
    if world > 1 and hasattr(be, "check_queues"):
        be.check_queues()
    barrier()
    t0 = time.perf_counter()
    for i in range(warmup, warmup + steps):
        step(i, warmup)
    drain(warmup + steps - 1)
    be.sync()
    t1 = time.perf_counter()
    barrier()
    dt = t1 - t0
    if world > 1:
        import torch.distributed as dist
        tt = torch.tensor([dt], dtype=torch.float64, device=getattr(be, "dev", None))
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    last = (warmup + steps - 1) % 2
    got = recv[last] if (gather and rank == 0) else None
    return dt, got, lay


# ---------------------------------------------------------------------------------------------
# per-kernel timings and the other BASELINE configs (rank 0 / N = 1 lines)
# ---------------------------------------------------------------------------------------------


def kernel_time_ms(eng, xd, reps=20):
    """Average duration of the dominant kernel: batch_kernel, the one launch that carries all the
    per-channel-frame work of a step (K-weighting + LUFS_inst, the four resolutions + combine, 4x true
    peak; omega_process_frames on device memory without meters launches exactly that kernel), from
    HIP events on the stream it is launched on (torch's current stream, bound to the context), through
    the C ABI so the host cost per call stays below the kernel's."""
    import ctypes
    from omega_gpu import _lib as L
    ncf = xd.numel() // W
    keep = [torch.empty(ncf, T, device=xd.device), torch.empty(ncf, device=xd.device),
            torch.empty(ncf, device=xd.device)]
    outs = L.Outputs()
    outs.combined, outs.lufs_inst, outs.true_peak_db = (t.data_ptr() for t in keep)
    lib = L.lib()
    eng._bind_stream(xd)

    def call():
        eng._check(lib.omega_process_frames(eng._ctx, xd.data_ptr(), ncf // C, C * W, W, ctypes.byref(outs),
                                            L.MEM_DEVICE))
    for _ in range(3):
        call()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        call()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps, ncf


def cfg3_line(dev, reps=100, n_batches=4):
    """BASELINE cfg3, the HBM-roofline run: 4096 mono frames x 8192 samples, fused windowed rfft ->
    512 log bands + 12-bin chromagram (omega_spectra), one launch per batch, inputs resident in HBM.
    The launches rotate over n_batches distinct input batches (134 MB each: 4 x 134 MB = 537 MB, past
    the 256 MiB Infinity Cache), so every launch reads its frames from HBM, not from on-die cache.
    Bytes per frame from SURVEY.md §8(d): 4 * 8192 in + 4 * (512 + 12) out = 34,864."""
    from omega_gpu import Engine, Resolution
    from omega_gpu import _lib as L
    from omega_gpu.engine import BandTable
    n, m = 4096, 8192
    x0 = torch.from_numpy(cfg3_input(n, m)).to(dev)
    # distinct batches: the same frames scaled per batch (distinct bytes, same workload)
    xs = [x0] + [x0 * (1.0 + 0.125 * k) for k in range(1, n_batches)]
    eng = Engine([Resolution((20, 20000), m, m // 4, 1.0)], FS, 20000, 512, device=dev.index or 0)
    st, en, comp = band_table_512()
    bt = BandTable(eng, L.BANDS_MAX, st, en, 512, m // 2 + 1, scale=comp)
    out = {"bands": torch.empty(n, 512, device=dev), "chroma": torch.empty(n, 12, dtype=torch.float64, device=dev)}
    rot = [0]

    def call():
        eng.spectra(xs[rot[0] % n_batches], "hann", bands=bt, chroma=True, out=out)
        rot[0] += 1
    warm_clock(call)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(reps):
        eng.spectra(xs[i % n_batches], "hann", bands=bt, chroma=True, out=out)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / reps
    bpf = 4 * m + 4 * (512 + 12)
    gbs = n * bpf / (ms * 1e-3) / 1e9
    traffic, src = kernel_traffic("cfg3")
    # the same batches alternating over two contexts on two streams: one launch's drain (its last
    # workgroups on a mostly idle chip) overlaps the next launch's start
    eng2 = Engine([Resolution((20, 20000), m, m // 4, 1.0)], FS, 20000, 512, device=dev.index or 0)
    bt2 = BandTable(eng2, L.BANDS_MAX, st, en, 512, m // 2 + 1, scale=comp)
    out2 = {"bands": torch.empty(n, 512, device=dev), "chroma": torch.empty(n, 12, dtype=torch.float64, device=dev)}
    lanes = [(eng, bt, out, torch.cuda.Stream(device=dev)), (eng2, bt2, out2, torch.cuda.Stream(device=dev))]

    def call2(i):
        eg, b, o, st_ = lanes[i % 2]
        with torch.cuda.stream(st_):
            eg.spectra(xs[i % n_batches], "hann", bands=b, chroma=True, out=o)
    warm_clock(lambda: [call2(i) for i in range(2)])
    s.record()
    for _, _, _, st_ in lanes:
        st_.wait_event(s)
    for i in range(reps):
        call2(i)
    for _, _, _, st_ in lanes:
        ev = torch.cuda.Event()
        ev.record(st_)
        torch.cuda.current_stream().wait_event(ev)
    e.record()
    torch.cuda.synchronize()
    ms2 = s.elapsed_time(e) / reps
    return {"workload": "cfg3: 4096 mono frames x 8192, Hann rfft -> 512 log bands (A10) + chromagram (A12), fused",
            "value": n / (ms * 1e-3), "unit": "frames/s", "ms_per_batch": ms,
            "two_streams": {"value": n / (ms2 * 1e-3), "ms_per_batch": ms2,
                            "achieved_gbs": n * bpf / (ms2 * 1e-3) / 1e9,
                            "frac": n * bpf / (ms2 * 1e-3) / 1e9 / PEAK_HBM_GBS,
                            "note": "consecutive batches alternating over two contexts on two streams (one launch's "
                                    "drain overlaps the next one's start); the roofline below is the one-stream "
                                    "launch interval"},
            "working_set": f"{n_batches} distinct input batches of {n * m * 4 / 1e6:.0f} MB rotated per launch "
                           f"({n_batches * n * m * 4 / 2**20:.0f} MiB > the 256 MiB Infinity Cache)",
            "roofline": {"bound": "hbm", "kernel": "spectra_rf_kernel<4096>", "achieved": gbs, "peak": PEAK_HBM_GBS,
                         "unit": "GB/s", "frac": gbs / PEAK_HBM_GBS, "traffic": traffic, "traffic_source": src,
                         "bytes_per_frame": bpf, "algorithmic_bytes_per_launch": n * bpf}}


PUBLISHED_MRFFT_MS = 0.20  # MultiResolutionFFT 0.20 ms per iteration (docs/MULTI_RESOLUTION_FFT_IMPROVEMENTS.md:193-195)


def latency_line(dev, iters=1000, lufs_iters=300, cpu=True):
    """The drop-in surfaces the app calls once per display frame, per-call latency on the host clock:
    (a) benchmark_multi_fft (multi_resolution_fft.py:467-494: default configs, 512-sample chunks,
    process_audio_chunk + combine_results_optimized per iteration) -- the reference's only published
    on-path figure is 0.20 ms per iteration; (b) ProfessionalMetering.calculate_lufs at the app's shape
    (omega4_main.py:1082: 2048-sample Hann-windowed float64 frames; professional_meters.py:231-281);
    (c) the app's MRFFT call pair on those frames (app_frame_ms). Beside each, the oracle's equivalent
    on this host (one core)."""
    from omega_gpu.multi_resolution_fft import benchmark_multi_fft
    from omega_gpu.professional_meters import ProfessionalMetering
    mr = benchmark_multi_fft(FS, 512, iters, device=dev.index or 0)
    rng = np.random.default_rng(8)
    frames = [(0.3 * np.sin(2 * np.pi * 440 * np.arange(2048) / FS + 0.1 * k) + 0.01 * rng.standard_normal(2048))
              * np.hanning(2048) for k in range(64)]
    # (c) the app's own per-display-frame MRFFT call pair (omega4_main.py:707-717): process_audio_chunk
    # on the 2048-sample Hann-windowed float64 frame, then combine_results_optimized at target_bins =
    # the display bars (512): after the first frame the chunk's launch forms the 512-target combine, so
    # the pair is one device round trip
    from omega_gpu.multi_resolution_fft import MultiResolutionFFT
    app = MultiResolutionFFT(FS, device=dev.index or 0)
    for k in range(10):
        res = app.process_audio_chunk(frames[k % 64], apply_weighting=True)
        app.combine_results_optimized(res, target_bins=512)
    t0 = time.perf_counter()
    for k in range(iters):
        res = app.process_audio_chunk(frames[k % 64], apply_weighting=True)
        if res:
            spectrum, freqs = app.combine_results_optimized(res, target_bins=512)
    app_ms = (time.perf_counter() - t0) / iters * 1e3
    app.cleanup()
    pm = ProfessionalMetering(FS, device=dev.index or 0)
    for k in range(10):
        pm.calculate_lufs(frames[k % 64])
    t0 = time.perf_counter()
    for k in range(lufs_iters):
        pm.calculate_lufs(frames[k % 64])
    lufs_ms = (time.perf_counter() - t0) / lufs_iters * 1e3
    line = {"workload": "drop-in per-call latency: benchmark_multi_fft (default configs, 512-sample chunks, "
                        "process_audio_chunk + combine_results_optimized) and calculate_lufs on 2048-sample Hann "
                        "float64 frames (the app's per-display-frame calls), host clock",
            "mrfft_ms_per_iteration": mr["avg_time_ms"], "mrfft_published_ms": PUBLISHED_MRFFT_MS,
            "mrfft_vs_published": PUBLISHED_MRFFT_MS / mr["avg_time_ms"],
            "calculate_lufs_ms_per_call": lufs_ms,
            "app_frame_ms": app_ms,
            "app_frame_workload": "process_audio_chunk(2048-sample Hann float64 frame, apply_weighting=True) + "
                                  "combine_results_optimized(target_bins=512), omega4_main.py:707-717"}
    if cpu:
        os.environ.setdefault("OMP_NUM_THREADS", "1")
        from oracle import omega_ref as R
        st = R.MRFFTStream()
        x = np.random.random(512).astype(np.float32)
        for _ in range(10):
            st.process(x)
        n = max(100, iters // 5)
        t0 = time.perf_counter()
        for _ in range(n):
            res = st.process(x)
            if res:
                R.combine(res)
        line["mrfft_oracle_ms_per_iteration"] = (time.perf_counter() - t0) / n * 1e3
        st = R.MRFFTStream()
        for k in range(10):
            st.process(frames[k % 64])
        n = max(100, iters // 5)
        t0 = time.perf_counter()
        for k in range(n):
            res = st.process(frames[k % 64])
            if res:
                R.combine(res, target_bins=512)
        line["app_frame_oracle_ms"] = (time.perf_counter() - t0) / n * 1e3
        ms = R.MeterState(FS)
        t0 = time.perf_counter()
        for k in range(lufs_iters):
            ms.update(frames[k % 64])
        line["calculate_lufs_oracle_ms_per_call"] = (time.perf_counter() - t0) / lufs_iters * 1e3
    return line


def cfg1_line(dev, reps=100, cpu=True):
    """BASELINE cfg1 (configs[0], the plumbing config): one 48 kHz mono stream, hop 512, W = 1024, one
    1024-point resolution + combine(512), K-weighted LUFS + true peak + meters (momentary over 24
    frames), 600 frames of 0.5 sin(2 pi 1000 t); the whole stream in one omega_process_stream call
    (device-resident), beside the oracle's per-frame loop over the same 600 frames on one core."""
    from omega_gpu import Engine, Resolution
    W1, H1, F1 = 1024, 512, 600
    n = W1 + H1 * (F1 - 1)
    t = np.arange(n) / FS
    x = (0.5 * np.sin(2 * np.pi * 1000 * t)).astype(np.float32)
    xd = torch.from_numpy(x).to(dev)
    eng = Engine([Resolution((20, 20000), W1, H1, 1.0)], FS, 20000, target_bins=T, frame_size=W1,
                 device=dev.index or 0)
    out = eng.process_stream(xd, n, H1, combined=True, meters=True)
    # (without the warm-up the per-call time read 0.21-0.27 ms on some runs instead of 0.07 ms)
    warm_clock(lambda: eng.process_stream(xd, n, H1, combined=True, meters=True, out=out))
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        eng.process_stream(xd, n, H1, combined=True, meters=True, out=out)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / reps
    line = {"workload": "cfg1: 48 kHz mono stream, hop 512, W 1024, one 1024-pt resolution + combine(512), K-LUFS + "
                        "4x TP + meters (momentary over 24 frames), 600 frames of 0.5 sin(2 pi 1000 t), one call",
            "value": F1 / (ms * 1e-3), "unit": "frames/s", "ms_per_call": ms, "frames": F1}
    if cpu:
        os.environ.setdefault("OMP_NUM_THREADS", "1")
        from oracle import omega_ref as R
        st = R.MeterState(FS)
        cfgs = (R.FFTConfig((20, 20000), W1, H1, 1.0),)
        t0 = time.perf_counter()
        for f in range(F1):
            fr = x[f * H1:f * H1 + W1]
            _, _, li, tp = R.full_frame(fr, configs=cfgs, target_bins=T)
            st.update(fr, li, tp)
        dt = time.perf_counter() - t0
        line["cpu_baseline"] = {"value": F1 / dt, "unit": "frames/s", "cores": 1, "kind": "port",
                                "sample": f"the same {F1} frames through the oracle's per-frame loop, {dt:.2f} s"}
    return line


def drums_line(dev, reps=100, n=4096, bins=1025):
    """SURVEY.md §8(f) row 1 (drum-detection features): one call over n consecutive magnitude frames
    of one stream (kick/snare band flux, adaptive thresholds, centroid), device-resident. Bytes per
    frame: the magnitude row in + 14 float64 out."""
    from omega_gpu import Engine
    rng = np.random.default_rng(5)
    mags = torch.from_numpy(np.abs(rng.standard_normal((n, bins))).astype(np.float32)).to(dev)
    eng = Engine(sample_rate=FS, device=dev.index or 0)
    out = torch.empty(n, 14, dtype=torch.float64, device=dev)
    warm_clock(lambda: eng.drum_features(mags, out=out))
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        eng.drum_features(mags, out=out)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / reps
    bpf = 4 * bins + 8 * 14
    gbs = n * bpf / (ms * 1e-3) / 1e9
    traffic, src = kernel_traffic("drums")
    return {"workload": f"drum features: {n} consecutive frames x {bins} bins of one stream (kick 3 + snare 4 band "
                        "flux, adaptive thresholds, spectral centroid)",
            "value": n / (ms * 1e-3), "unit": "frames/s", "ms_per_call": ms,
            "roofline": {"bound": "latency", "kernel": "drum_flux_kernel + drum_thr_kernel", "achieved": gbs,
                         "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": gbs / PEAK_HBM_GBS, "traffic": traffic,
                         "traffic_source": src, "bytes_per_frame": bpf}}


def post_line(dev, reps=100, n=4096, bins=512):
    """SURVEY.md §8(f) row 2 (the app's spectrum post-processing): one call over n consecutive
    combined spectra of one stream (equal-loudness, content type, p98 normalisation, compensation,
    band means + EMA), device-resident. Bytes per frame: the spectrum in, spectrum + bands + content out."""
    from omega_gpu.app_post import SpectrumPostProcessor
    rng = np.random.default_rng(6)
    x = torch.from_numpy(rng.random((n, bins)).astype(np.float32)).to(dev)
    pp = SpectrumPostProcessor(np.linspace(20, 20000, bins), device=dev.index or 0)
    warm_clock(lambda: pp.process(x))
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        pp.process(x)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / reps
    bpf = 4 * (2 * bins + 1) + 8 * pp.n_bands
    gbs = n * bpf / (ms * 1e-3) / 1e9
    traffic, src = kernel_traffic("post")
    return {"workload": f"app post-processing: {n} consecutive combined spectra x {bins} bins of one stream "
                        f"({pp.n_bands} bands)",
            "value": n / (ms * 1e-3), "unit": "frames/s", "ms_per_call": ms,
            "roofline": {"bound": "latency", "kernel": "post_frame_kernel + post_ema_kernel", "achieved": gbs,
                         "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": gbs / PEAK_HBM_GBS, "traffic": traffic,
                         "traffic_source": src, "bytes_per_frame": bpf}}


def cfg5_line(rank, world, dev, seconds=60.0):
    """BASELINE cfg5, the sustained stream: 96 kHz 8-channel surround, 60 s (SURVEY.md §8(d) signal),
    pushed as interleaved float32le capture bytes in 512-sample chunks through the ingest
    (omega_ingest_*: page-locked staging, async H2D, capture noise gate, stream layout), 16384-point
    frames every 1024 samples with 4x true peak, K-weighted LUFS and the meter aggregates (integrated
    window 3600 frames, reached at 38 s). One channel per GPU: rank r takes channels r, r + N, ...
    Wall time from the first push to the last result polled on the host, so it includes the host
    push, PCIe both ways and the analysis; max over ranks."""
    from omega_gpu import NORTHSTAR_RESOLUTIONS, Engine
    from omega_gpu.ingest import StreamIngest
    fs, C_all, W5, H5 = 96000, 8, 16384, 1024
    chans = list(range(rank, C_all, world))
    n = int(fs * seconds)
    x = cfg5_input(n, C_all, fs)[chans]
    inter = np.ascontiguousarray(x.T)
    eng = Engine(NORTHSTAR_RESOLUTIONS, fs, 20000, target_bins=T, n_channels=len(chans), device=dev.index or 0)
    ing = StreamIngest(eng, hop=H5, batch_hops=64, ring_slots=4, gain=1.0)
    # warm-up: one batch through a separate ingest
    w = StreamIngest(Engine(NORTHSTAR_RESOLUTIONS, fs, 20000, target_bins=T, n_channels=len(chans),
                            device=dev.index or 0), hop=H5, batch_hops=64)
    w.push(inter[:W5 + 64 * H5])
    w.flush()
    w.poll(wait=True)
    w.close()
    frames = 0
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    t0 = time.perf_counter()
    for i in range(0, n, 512):
        ing.push(inter[i:i + 512])
        if (i // 512) % 128 == 127:
            frames += len(ing.poll()["lufs_inst"])
    ing.flush()
    got = ing.poll(wait=True)
    frames += len(got["lufs_inst"])
    dt = time.perf_counter() - t0
    meters = got["meters"]
    st = ing.stats()
    ing.close()
    if world > 1:
        import torch.distributed as dist
        tt = torch.tensor([dt, frames], dtype=torch.float64, device=dev)
        dist.all_reduce(tt[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(tt[1:], op=dist.ReduceOp.SUM)
        dt, frames = float(tt[0]), int(tt[1])
    per_ch = (n - W5) // H5 + 1
    return {"workload": f"cfg5: 96 kHz x {C_all} ch x {seconds:.0f} s sustained stream, float32le capture bytes in "
                        "512-sample chunks -> ingest (page-locked staging, async H2D, noise gate) -> 16384-pt frames "
                        f"every {H5} samples (MRFFT 16k/8k/4k/1k + combine(512) + K-LUFS + 4x TP + meters, "
                        "integrated window 3600 frames); one channel per GPU",
            "value": frames / dt, "unit": "channel-frames/s", "wall_s": dt, "channel_frames": frames,
            "expected_channel_frames": per_ch * C_all, "dropped_frames": st["dropped_frames"],
            "realtime_factor": seconds / dt, "integrated_reached": bool(np.all(meters[-len(chans):, 2] > -100)),
            "note": "host push + PCIe H2D/D2H + analysis, wall-clock on the host (not the HBM-resident headline)"}


def cfg3_input(n, m):
    """BASELINE cfg3 synthetic frames (same generator as oracle/signals.cfg3_batch): even frames a
    0.5-amplitude C-major triad, odd frames 0.1 N(0,1) (seed 1234)."""
    t = np.arange(m) / FS
    tri = (0.5 * (np.sin(2 * np.pi * 261.63 * t) + np.sin(2 * np.pi * 329.63 * t) +
                  np.sin(2 * np.pi * 392.00 * t))).astype(np.float32)
    nz = (0.1 * np.random.default_rng(1234).standard_normal((n // 2 + 1) * m)).astype(np.float32).reshape(-1, m)
    out = np.empty((n, m), np.float32)
    out[0::2] = tri
    out[1::2] = nz[: n // 2]
    return out


def band_table_512(fs=FS, num_bands=512, fft_size=8192):
    """AudioProcessingPipeline band table (pipeline.py:165-230) via the product facade."""
    from omega_gpu.bands import pipeline_band_table
    return pipeline_band_table(fs, num_bands, fft_size)


def warm_clock(fn, seconds=0.1):
    """fn back to back for `seconds` of wall clock before a side line's timed loop. The shader clock
    drops within milliseconds of idle and takes ~30 ms of load to come back; a side line
    follows the host work of building its inputs and engine, and its 20 timed calls (1-6 ms) would
    otherwise run inside the ramp -- the clock of an idle GPU, not of the continuous stream the line
    stands for (cfg3 at continuous load: 50 us per launch at 2297 MHz, profiles/r05_power_cfg3.txt)."""
    t_end = time.perf_counter() + seconds
    while time.perf_counter() < t_end:
        for _ in range(10):
            fn()
        torch.cuda.synchronize()


def kernel_traffic(kind="batch"):
    """HBM bytes per launch of the dominant kernel from the newest committed counter passes
    (profiles/rNN_<kind>_traffic.json, written by tools/profile_round.sh + tools/summarize_round.py),
    or None."""
    import glob
    fs = sorted(glob.glob(os.path.join(REPO, "profiles", f"r*_{kind}_traffic.json")))
    if not fs:
        return None, None
    d = json.load(open(fs[-1]))
    return d["traffic_bytes"], os.path.relpath(fs[-1], REPO)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_calibration():
    """The restatement-vs-reference time ratio measured in the build container
    (tools/cpu_calibrate.py -> profiles/cpu_calibration.json), so the GPU host's port number is
    traceable to the reference's own CPU cost."""
    p = os.path.join(REPO, "profiles", "cpu_calibration.json")
    if not os.path.exists(p):
        return None
    return json.load(open(p))


def cpu_baseline(seconds):
    """The oracle (numpy/scipy restatement of the reference path, one core) on the first frames of
    the same workload until the time budget is spent -- the reference's steady state: windows, weight
    tables and filter coefficients are computed once (as MultiResolutionFFT._setup_windows and
    ProfessionalMetering.__init__ do), the meter deques carried frame to frame. `calibration` holds the
    restatement-vs-reference ratio measured in the build container (tools/cpu_calibrate.py: the
    reference with one MultiResolutionFFT and reset_all_buffers() per frame)."""
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    from oracle import omega_ref as R
    x = cfg2_input(64)
    st = [R.MeterState(FS), R.MeterState(FS)]
    n = 0
    t0 = time.perf_counter()
    while True:
        f, c = divmod(n, 2)
        fr = x[f % 64, c]
        _, _, li, tp = R.full_frame(fr)
        st[c].update(fr, li, tp)
        n += 1
        if time.perf_counter() - t0 > seconds and n >= 8:
            break
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "channel-frames/s", "cores": 1, "kind": "port", "cpu_model": cpu_model(),
            "sample": f"{n} channel-frames of cfg2 (oracle, steady state: MRFFT 16k/8k/4k/1k + combine(512) + "
                      f"K-LUFS + 4x TP + meter deques), {dt:.1f} s, OMP_NUM_THREADS=1",
            "calibration": cpu_calibration()}


def _cpu_worker(args):
    """One CPU-baseline process: its own channel of the cfg2 frames (oracle loop with meter state)."""
    seconds, c, seed = args
    os.environ["OMP_NUM_THREADS"] = "1"
    from oracle import omega_ref as R
    x = cfg2_input(16, seed_l=seed, seed_r=seed + 1)
    st = R.MeterState(FS)
    n = 0
    t0 = time.perf_counter()
    while True:
        fr = x[n % 16, c]
        _, _, li, tp = R.full_frame(fr)
        st.update(fr, li, tp)
        n += 1
        if time.perf_counter() - t0 > seconds and n >= 4:
            break
    return n, time.perf_counter() - t0


def cpu_baseline_all_cores(seconds, procs):
    """SURVEY.md §8(d)'s second CPU mode: the same oracle loop in `procs` processes (one stream each),
    forked before this process touches the GPU; aggregate channel-frames/s."""
    import multiprocessing as mp
    with mp.get_context("fork").Pool(procs) as pool:
        res = pool.map(_cpu_worker, [(seconds, i % 2, 2 * (i // 2)) for i in range(procs)])
    n = sum(r[0] for r in res)
    wall = max(r[1] for r in res)
    return {"value": n / wall, "unit": "channel-frames/s", "cores": procs, "kind": "port", "cpu_model": cpu_model(),
            "sample": f"{n} channel-frames of cfg2 over {procs} processes (one stream each, oracle loop with "
                      f"meter state), {wall:.1f} s, OMP_NUM_THREADS=1"}


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    if a.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU, started here before any GPU call (no exec from a GPU process)
        sys.exit(launch_ranks(a.gpus, argv))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {a.gpus}")
    standin = a.standin is not None
    cpu_all = None
    if world == 1 and not a.no_cpu_baseline and a.cpu_procs > 1 and not standin:
        # before any GPU call: the workers are forked from this process
        cpu_all = cpu_baseline_all_cores(a.cpu_seconds, a.cpu_procs)
    be = importlib.import_module(a.standin).Backend(local) if standin else DeviceBackend(local)
    if world > 1:
        import torch.distributed as dist
        if standin:
            dist.init_process_group(be.dist_backend)
        else:
            dist.init_process_group(be.dist_backend, device_id=be.dev)
            be.check_queues()
    gather = world > 1 and not a.no_gather

    frames = a.frames
    prep_main = prepare(be, rank, world, frames) if not standin else None
    # The cfg4 line (every rank: the per-GPU shard, ~25 ms of the same path) runs right before the
    # headline, its inputs and the headline's made beforehand so the GPU does not idle in between:
    # MI355X lowers its clock after a few ms of idle and takes ~30 ms of load to raise it again
    # (tools/ramp_probe.py: 89.8 us per step in the first 20 steps out of idle, 79.7 after 350; after
    # a 5 ms pause 90.0 again; after 25 cfg4 steps instead of the pause 79.9 -- DESIGN.md §5), so the
    # headline's K steps are timed at the clock the path runs at in continuous service.
    cfg4 = None
    if not standin and not a.no_cfg4:
        dt4, _, _ = measure(be, rank, world, FRAMES_CFG4, a.cfg4_steps, 3, gather)
        ncf4 = FRAMES_CFG4 * C
        cfg4 = {"workload": f"cfg4 per-GPU shard: {FRAMES_CFG4} stereo frames x 16384 per GPU "
                            f"({FRAMES_CFG4 * world} stereo frames over {world} GPU(s); BASELINE cfg4 = 32768 "
                            "over 8), same per-step path as the headline line" +
                            (", packed outputs gathered to rank 0 over RCCL each step" if gather else "") +
                            "; measured first, out of idle (its steps include the clock ramp)",
                "value": ncf4 * world * a.cfg4_steps / dt4, "unit": "channel-frames/s",
                "ms_per_step": dt4 / a.cfg4_steps * 1e3, "steps": a.cfg4_steps,
                "channel_frames_per_gpu": ncf4, "global_stereo_frames": FRAMES_CFG4 * world}
    dt, got, lay = measure(be, rank, world, frames, a.steps, a.warmup, gather, prep=prep_main)
    ncf = frames * C
    value = ncf * world * a.steps / dt
    if a.dump and rank == 0 and got is not None:
        np.save(a.dump, torch.stack([g.cpu() for g in got]).numpy())

    rotating = None
    if not standin and not a.no_rotating:
        # the same step over 8 distinct input batches rotated per step (8 x 33.5 MB = 268 MB, past the
        # 256 MiB Infinity Cache): the headline reads one resident batch, whose second read by the
        # true-peak role is an Infinity-Cache hit either way; this line shows what cold input costs
        x0 = prep_main[0]
        xr = [x0] + [x0 * (1.0 + 0.0625 * k) for k in range(1, 8)]
        # (800 untimed steps, ~55 ms: the clock back at the continuous-load level after building xr)
        dtr, _, _ = measure(be, rank, world, frames, a.steps, max(a.warmup, 800), gather,
                            prep=(xr,) + tuple(prep_main[1:]))
        rotating = {"workload": f"cfg2 step over 8 distinct resident input batches rotated per step "
                                f"({8 * frames * C * W * 4 / 2**20:.0f} MiB > the 256 MiB Infinity Cache)",
                    "value": frames * C * world * a.steps / dtr, "unit": "channel-frames/s",
                    "ms_per_step": dtr / a.steps * 1e3}
        del xr
    in_call = None
    if not standin and not a.no_rotating and getattr(be, "pipelined", False):
        # the same step with every call completing its own meter aggregates (no pipelining: the
        # contract of the drop-in facades), on the headline's input
        be.pipelined = False
        dti, _, _ = measure(be, rank, world, frames, a.steps, max(a.warmup, 400), gather, prep=prep_main)
        be.pipelined = True
        be.reset()
        in_call = {"workload": "cfg2 step with each call's meter aggregates computed in its own launch "
                               "(omega_set_meter_pipelining off: the contract the drop-in facades use)",
                   "value": frames * C * world * a.steps / dti, "unit": "channel-frames/s",
                   "ms_per_step": dti / a.steps * 1e3}
    roof = None
    if not standin:
        # (right after the headline, on its input: no idle in between, see above)
        kt_ms, kcf = kernel_time_ms(be.eng, prep_main[0])
        flop_launch = (FLOP_FFT + FLOP_KW + FLOP_TP) * kcf
        achieved = flop_launch / (kt_ms * 1e-3) / 1e12
        traffic, traffic_src = kernel_traffic("batch")
        roof = {"bound": "valu", "kernel": "batch_kernel (K-weighting + LUFS, 16k/8k/4k/1k FFT + combine, "
                                           "4x true peak; fp32)",
                "achieved": achieved, "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                "frac": achieved / PEAK_FP32_TFLOPS, "traffic": traffic,
                "kernel_ms": kt_ms, "flop_per_launch": flop_launch,
                "executed": {"flop_per_launch": (FLOP_FFT + FLOP_KW + FLOP_TP_EXEC) * kcf,
                             "achieved": (FLOP_FFT + FLOP_KW + FLOP_TP_EXEC) * kcf / (kt_ms * 1e-3) / 1e12,
                             "frac": (FLOP_FFT + FLOP_KW + FLOP_TP_EXEC) * kcf / (kt_ms * 1e-3) / 1e12
                             / PEAK_FP32_TFLOPS,
                             "note": "the flops the kernel executes: the true peak in its polyphase form "
                                     "(FLOP_TP_EXEC, 2.60 M per channel-frame) instead of the reference's "
                                     "resample algorithm; frac above is SURVEY.md §8(d)'s count"},
                "traffic_unit": "bytes per launch (HBM, FETCH_SIZE x2 + WRITE_SIZE)",
                "traffic_source": traffic_src,
                "algorithmic_bytes_per_launch": kcf * BYTES_CF,
                "note": "fp32 VALU-bound (no MFMA: nothing here is a dense contraction); algorithmic flops per "
                        "channel-frame = SURVEY.md §8(d) FFT 1.09 M + KW 0.67 M + TP 3.33 M (the reference's "
                        "resample algorithm); kernel_ms = HIP-event average of 20 back-to-back launches on the "
                        "launch stream"}
    cfg5 = None
    if not standin and not a.no_cfg5:
        cfg5 = cfg5_line(rank, world, be.dev, a.cfg5_seconds)
    if rank == 0:
        cpu = None
        if world == 1 and not a.no_cpu_baseline and not standin:
            cpu = cpu_baseline(a.cpu_seconds)
        line = {
            "metric": METRIC,
            "value": value, "unit": "channel-frames/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": dt / a.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32",
            "data": "synthetic cfg2 frames (0.25 sine 440/997 Hz + 0.05 N(0,1), seeds per rank)",
            "config": {"workload": f"cfg2: {frames} stereo frames x 16384 samples per GPU; MRFFT 16k/8k/4k/1k + "
                                   "combine(512) + K-weighted LUFS + 4x true peak + meter aggregates",
                       "channel_frames_per_gpu": ncf, "frame_samples": W, "target_bins": T,
                       "parallelism": f"frames sharded over {world} GPU(s)" +
                                      (", packed outputs gathered to rank 0 over RCCL each step" if gather else "")},
            "roofline": roof,
            "cpu_baseline": cpu,
            "cpu_baseline_all_cores": cpu_all,
            "meters": ("pipelined (omega_set_meter_pipelining): each step's meter aggregates are computed by "
                       "the next step's launch, the last step's by a flush inside the timed region; every "
                       "step's outputs are complete before the closing synchronize"
                       if getattr(be, "pipelined", False) else "computed in each step's own launch"),
        }
        if standin:
            line["backend"] = f"stand-in {a.standin} (CPU, {be.dist_backend}); not a measurement"
        if cfg4 is not None:
            line["cfg4"] = cfg4
        if rotating is not None:
            line["cfg2_rotating_inputs"] = rotating
        if in_call is not None:
            line["cfg2_meters_in_call"] = in_call
        if cfg5 is not None:
            line["cfg5"] = cfg5
        if world == 1 and not a.no_cfg3 and not standin:
            line["cfg3"] = cfg3_line(be.dev)
            line["cfg1"] = cfg1_line(be.dev, cpu=not a.no_cpu_baseline)
            line["latency"] = latency_line(be.dev, cpu=not a.no_cpu_baseline)
            line["drums"] = drums_line(be.dev)
            line["app_post"] = post_line(be.dev)
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
