"""bench.py's N>1 path on the CPU: `bench.py --gpus 2` starts its own two rank processes (no
WORLD_SIZE in the environment), runs its own step loop with the packed zero-copy outputs and the
async gather to rank 0 over gloo, with the oracle stand-in (tests/bench_standin.py) computing each
rank's shard; rank 0's JSON line reports n_gpus 2 and its last gathered blocks equal a
single-process oracle run of the same shards."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "audio-analyzer-omega_amd"))

from omega_gpu import dist as D  # noqa: E402

T = 512


def _run(args, tmp_path, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["PYTHONPATH"] = REPO + os.pathsep + env.get("PYTHONPATH", "")
    env["OMP_NUM_THREADS"] = "1"
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, cwd=REPO, env=env,
                          capture_output=True, text=True, timeout=600)


def test_bench_gpus2_launches_two_ranks_and_gathers(tmp_path):
    from tests.bench_standin import Backend
    dump = str(tmp_path / "gathered.npy")
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--frames", "1", "--standin", "tests.bench_standin",
              "--dump", dump], tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["steps"] == 1 and line["scaling"] == "weak"
    assert line["config"]["channel_frames_per_gpu"] == 2
    assert "gathered to rank 0" in line["config"]["parallelism"]
    got = np.load(dump)
    lay = D.PackedLayout(2, T)
    assert got.shape == (2, lay.nbytes)
    g = D.unpack_gathered([torch.from_numpy(b) for b in got], lay)
    # single process: the same per-rank shards (seeds 2r, 2r + 1), meter state fresh per shard
    be = Backend(0)
    for rank in range(2):
        x = be.input(1, 2 * rank, 2 * rank + 1)
        buf = lay.alloc()
        be.reset()
        be.process(x, 1, lay.views(buf))
        be.flush()  # (pipelined meters: the stand-in writes them at the next call or flush, like the device)
        ref = lay.views(buf)
        for k in ref:
            np.testing.assert_array_equal(g[k][2 * rank:2 * rank + 2].numpy(), ref[k].numpy(), err_msg=k)


def test_bench_gpus2_pipelined_meters_over_steps(tmp_path):
    """Several warmup and timed steps: with the stand-in's pipelined meters (written by the next call,
    like omega_set_meter_pipelining) the last gathered block carries the last step's complete meters --
    bench.py gathers each step after the next launch and flushes the last one."""
    from tests.bench_standin import Backend
    dump = str(tmp_path / "gathered.npy")
    r = _run(["--gpus", "2", "--steps", "3", "--warmup", "2", "--frames", "1", "--standin", "tests.bench_standin",
              "--dump", dump], tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    lay = D.PackedLayout(2, T)
    g = D.unpack_gathered([torch.from_numpy(b) for b in np.load(dump)], lay)
    be = Backend(0)
    for rank in range(2):
        x = be.input(1, 2 * rank, 2 * rank + 1)
        be.reset()
        for _ in range(5):  # one meter stream over warmup + timed steps
            buf = lay.alloc()
            be.process(x, 1, lay.views(buf))
        be.flush()
        ref = lay.views(buf)
        for k in ref:
            np.testing.assert_array_equal(g[k][2 * rank:2 * rank + 2].numpy(), ref[k].numpy(), err_msg=k)


def test_bench_rejects_world_mismatch(tmp_path):
    r = _run(["--gpus", "2", "--standin", "tests.bench_standin"], tmp_path,
             {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=1 but --gpus 2" in r.stderr


def test_launcher_propagates_rank_failure(tmp_path):
    # a stand-in module that does not exist: every rank fails, the launcher reports it
    r = _run(["--gpus", "2", "--standin", "tests.no_such_module", "--steps", "1", "--warmup", "0"], tmp_path)
    assert r.returncode != 0


@pytest.mark.parametrize("n", [0, 1, 3, 512])
def test_packed_layout_views_alias_buffer(n):
    lay = D.PackedLayout(n, T)
    buf = lay.alloc()
    v = lay.views(buf)
    assert v["combined"].shape == (n, T) and v["meters"].shape == (n, 5) and v["meters"].dtype == torch.float64
    if n:
        v["combined"].fill_(1.5)
        v["lufs_inst"].fill_(-3.0)
        v["true_peak_db"].fill_(-1.0)
        v["meters"].fill_(2.25)
        w = lay.views(buf)
        assert float(w["combined"].sum()) == 1.5 * n * T and float(w["meters"].sum()) == 2.25 * 5 * n
        assert float(w["lufs_inst"].sum()) == -3.0 * n and float(w["true_peak_db"].sum()) == -1.0 * n
    assert lay.off_meters % 8 == 0 and lay.nbytes >= lay.off_meters + 40 * n
