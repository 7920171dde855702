"""Multi-GPU layout for the per-frame path: one process per GPU, channel-frames
sharded in contiguous blocks of the batch axis (weak scaling: every rank owns whole streams, so the
meter aggregates need no exchange), and the per-frame output vectors gathered to rank 0 over RCCL
(backend "nccl") -- the only collective, overlapped with the next batch by the caller.

Packed per-channel-frame vector (float32, T + 7 values):
    [0, T)   combined spectrum          T     LUFS_inst        T + 1  true peak (dBTP)
    T + 2 .. T + 6  meter aggregates (momentary, short_term, integrated, range, true_peak)
The aggregates are float64 on the device; the packed form carries them as float32 (0.1 LU bars are
far above float32 resolution in the -100..+10 dB range).

Pure torch: the same code runs over gloo on the CPU (tests/test_dist.py) and over RCCL on the box.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch

N_EXTRA = 7


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous block [a, b) of n items for `rank` (the first n % world ranks get one more)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} of world {world}")
    q, r = divmod(n, world)
    a = rank * q + min(rank, r)
    return a, a + q + (1 if rank < r else 0)


def pack_width(T: int) -> int:
    return T + N_EXTRA


def pack_outputs(out: Dict[str, torch.Tensor], T: int, dst: Optional[torch.Tensor] = None) -> torch.Tensor:
    """process_frames outputs (combined [n, T], lufs_inst [n], true_peak_db [n], meters [n, 5]) ->
    one [n, T + 7] float32 tensor (written into dst when given)."""
    comb = out["combined"]
    n = comb.shape[0]
    p = dst if dst is not None else torch.empty(n, pack_width(T), dtype=torch.float32, device=comb.device)
    p[:, :T].copy_(comb)
    p[:, T].copy_(out["lufs_inst"])
    p[:, T + 1].copy_(out["true_peak_db"])
    p[:, T + 2:].copy_(out["meters"])
    return p


def unpack_outputs(p: torch.Tensor, T: int) -> Dict[str, torch.Tensor]:
    return {"combined": p[:, :T], "lufs_inst": p[:, T], "true_peak_db": p[:, T + 1], "meters": p[:, T + 2:]}


def gather_to_root(p: torch.Tensor, recv: Optional[List[torch.Tensor]], async_op: bool = False):
    """Gather every rank's packed block (equal shapes) to rank 0. recv: world tensors on rank 0, None
    elsewhere. Returns the work handle when async_op."""
    import torch.distributed as dist
    return dist.gather(p, recv if dist.get_rank() == 0 else None, dst=0, async_op=async_op)
