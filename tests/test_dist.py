"""The N>1 path on CPU: world_size-2 gloo process group, frames sharded in contiguous blocks, each
rank computing its shard (the oracle stands in for the device here), packing the per-frame output
vectors and gathering them to rank 0 exactly as bench.py does over RCCL; rank 0 checks the gathered
batch against a single-process run."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "audio-analyzer-omega_amd"))
sys.path.insert(0, REPO)

from omega_gpu import dist as D  # noqa: E402

T = 512


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard_outputs(x, a, b):
    """Oracle outputs for channel-frames [a, b) of x [F, C, W], with per-stream meter state."""
    from oracle import omega_ref as R
    F, C, W = x.shape
    n = b - a
    comb = np.zeros((n, T), np.float32)
    li = np.zeros(n, np.float32)
    tp = np.zeros(n, np.float32)
    met = np.zeros((n, 5), np.float64)
    states = {}
    for i, cf in enumerate(range(a, b)):
        f, c = divmod(cf, C)
        _, cb, l, t = R.full_frame(x[f, c])
        st = states.setdefault(c, R.MeterState(48000))
        m = st.update(x[f, c], l, t)
        comb[i], li[i], tp[i] = cb, l, t
        met[i] = list(m.values())
    return {"combined": torch.from_numpy(comb), "lufs_inst": torch.from_numpy(li),
            "true_peak_db": torch.from_numpy(tp), "meters": torch.from_numpy(met)}


def _worker(rank, world, port, x, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        F, C, _ = x.shape
        # whole streams per rank: shard the frame axis, every rank keeps all channels of its frames
        fa, fb = D.shard_range(F, rank, world)
        out = _shard_outputs(x, fa * C, fb * C)
        lay = D.PackedLayout((fb - fa) * C, T)
        p = lay.pack(out)
        recv = [torch.empty_like(p) for _ in range(world)] if rank == 0 else None
        D.gather_to_root(p, recv, async_op=True).wait()
        if rank == 0:
            g = D.unpack_gathered(recv, lay)
            q.put({k: v.numpy() for k, v in g.items()})
    finally:
        dist.destroy_process_group()


def test_shard_range_covers():
    for n in (0, 1, 7, 256, 1000):
        for w in (1, 2, 3, 8):
            blocks = [D.shard_range(n, r, w) for r in range(w)]
            assert blocks[0][0] == 0 and blocks[-1][1] == n
            assert all(blocks[i][1] == blocks[i + 1][0] for i in range(w - 1))
            assert max(b - a for a, b in blocks) - min(b - a for a, b in blocks) <= 1
    with pytest.raises(ValueError):
        D.shard_range(4, 2, 2)


def test_pack_roundtrip():
    n = 3
    out = {"combined": torch.rand(n, T), "lufs_inst": torch.rand(n), "true_peak_db": torch.rand(n),
           "meters": torch.rand(n, 5, dtype=torch.float64)}
    lay = D.PackedLayout(n, T)
    u = lay.views(lay.pack(out))
    for k in out:
        assert torch.equal(u[k], out[k])


def test_gloo_world2_gather_matches_single_process():
    from oracle import signals as S
    # 4 stereo frames, shards of 2 frames (= whole streams of 2 frames each rank)
    x = S.cfg2_batch(4)
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, x, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single process, same sharding of streams (meter state restarts per shard, as per rank)
    shards = [_shard_outputs(x, a * 2, b * 2) for a, b in (D.shard_range(4, r, world) for r in range(world))]
    for k in got:
        np.testing.assert_array_equal(got[k], np.concatenate([s[k].numpy() for s in shards]), err_msg=k)
    assert got["combined"].shape == (8, T) and got["meters"].shape == (8, 5)
