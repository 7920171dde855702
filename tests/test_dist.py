"""The N>1 path on CPU: gloo process groups, frames sharded in contiguous blocks, each rank computing
its shard (the oracle stands in for the device here), packing the per-frame output vectors and
gathering them to rank 0 exactly as bench.py does over RCCL; rank 0 checks the gathered batch against
a single-process run. Two stream layouts: independent streams per rank (bench.py's cfg4), and one
stream split over the ranks in time, whose meter history the ranks exchange (TimeShardExchange) --
checked against ONE meter state over the whole stream."""
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
    # single process over the same layout: every rank's frames are an independent stream (bench.py's
    # cfg4 generates one stream per rank), so the meter state starts fresh per shard; the time-sharded
    # layout of ONE stream is test_gloo_time_sharded_stream_meters_match_one_stream below
    shards = [_shard_outputs(x, a * 2, b * 2) for a, b in (D.shard_range(4, r, world) for r in range(world))]
    for k in got:
        np.testing.assert_array_equal(got[k], np.concatenate([s[k].numpy() for s in shards]), err_msg=k)
    assert got["combined"].shape == (8, T) and got["meters"].shape == (8, 5)


class _OracleMeters:
    """The engine's meter interface (reset_meters / meter_update over [n, C] rows) on the oracle's
    per-stream MeterState (float64 deques), standing in for the device on the CPU."""

    def __init__(self, C):
        from oracle import omega_ref as R
        self.C, self.R = C, R
        self.reset_meters()

    def reset_meters(self):
        self.st = [self.R.MeterState(48000) for _ in range(self.C)]

    def meter_update(self, li, tp, n):
        out = np.zeros((n * self.C, 5))
        for f in range(n):
            for c in range(self.C):
                out[f * self.C + c] = list(self.st[c].update(np.ones(1), float(li[f, c]), float(tp[f, c])).values())
        return torch.from_numpy(out)


def _stream_values(n, C, seed=9):
    """LUFS_inst / true-peak rows of one C-channel stream: gated and ungated stretches, a silent run
    longer than the 3600-frame window's gate margin, ties (the aggregates depend on these alone)."""
    rng = np.random.default_rng(seed)
    li = rng.uniform(-85, -5, (n, C)).astype(np.float32)
    li[1200:1500] = -95.0
    li[2600:2700] = np.float32(-23.0)
    tp = rng.uniform(-40, 0, (n, C)).astype(np.float32)
    return li, tp


def _ts_worker(rank, world, port, batches, C, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        eng = _OracleMeters(C)
        ex = D.TimeShardExchange(C)
        res = []
        for li, tp in batches:  # consecutive global batches of the one stream
            a, b = D.shard_range(li.shape[0], rank, world)
            sl, st = torch.from_numpy(li[a:b]), torch.from_numpy(tp[a:b])
            hist = ex.exchange(sl, st)
            res.append(D.meter_time_shard(eng, sl, st, hist))
        q.put((rank, [r.numpy() for r in res]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,sizes", [(2, (4100, 2300)), (3, (900, 700, 4000))])
def test_gloo_time_sharded_stream_meters_match_one_stream(world, sizes):
    """ONE stereo stream split over the ranks in time (SURVEY §8(e)'s second layout), over several
    global batches (shards both longer and shorter than the 3599-frame history, so a rank's history
    can span several earlier ranks and the previous batch): each rank's meters, after the all-gather of
    the shard tails, equal one meter state fed the whole stream frame by frame -- bitwise."""
    C = 2
    li, tp = _stream_values(sum(sizes), C)
    cuts = np.cumsum((0,) + sizes)
    batches = [(li[a:b], tp[a:b]) for a, b in zip(cuts[:-1], cuts[1:])]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ts_worker, args=(r, world, port, batches, C, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=600) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    one = _OracleMeters(C).meter_update(li, tp, li.shape[0]).numpy().reshape(-1, C, 5)
    for bi, (a0, b0) in enumerate(zip(cuts[:-1], cuts[1:])):
        for r in range(world):
            a, b = D.shard_range(b0 - a0, r, world)
            np.testing.assert_array_equal(got[r][bi].reshape(-1, C, 5), one[a0 + a:a0 + b], err_msg=f"batch {bi} rank {r}")


def test_stream_history_spans_short_shards():
    """stream_history takes the last rows across several short tails and the carried history."""
    prev = torch.arange(5, dtype=torch.float32)[:, None]
    tails = [(torch.tensor([[10.0], [11.0]]), torch.tensor([[10.0], [11.0]])), (torch.tensor([[20.0]]), torch.tensor([[20.0]]))]
    li, tp = D.stream_history(prev, prev, tails, 2, nl=4, nt=2)
    assert li[:, 0].tolist() == [4.0, 10.0, 11.0, 20.0] and tp[:, 0].tolist() == [11.0, 20.0]
    hl, ht = D.history_frames(li, tp)
    assert ht[:, 0].tolist() == [-100.0, -100.0, 11.0, 20.0]
