"""Multi-GPU layout for the per-frame path: one process per GPU, channel-frames
sharded in contiguous blocks of the batch axis (weak scaling: every rank owns whole streams, so the
meter aggregates need no exchange), and each rank's per-frame outputs gathered to rank 0 over RCCL
(backend "nccl") -- the only collective, overlapped with the next batch by the caller.

Packed block of one rank (PackedLayout): ONE flat byte buffer holding the outputs planar, so the
engine writes straight into it (the output dict is a set of views) and the gather moves it as it is,
with no pack kernel in between:

    [0, 4·n·T)            combined spectrum   float32 [n, T]
    next 4·n              LUFS_inst           float32 [n]
    next 4·n              true peak (dBTP)    float32 [n]
    next 40·n (8-aligned) meter aggregates    float64 [n, 5] (momentary, short_term, integrated, range, true_peak)

= 4T + 48 bytes per channel-frame (+ alignment). Pure torch: the same code runs over gloo on the CPU
(tests/test_dist.py, tests/test_bench_launch.py) and over RCCL on the box.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch

N_METERS = 5


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous block [a, b) of n items for `rank` (the first n % world ranks get one more)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} of world {world}")
    q, r = divmod(n, world)
    a = rank * q + min(rank, r)
    return a, a + q + (1 if rank < r else 0)


def _align(v: int, a: int) -> int:
    return (v + a - 1) // a * a


class PackedLayout:
    """Byte offsets of one rank's output block for n channel-frames and T combined bins."""

    def __init__(self, n: int, T: int):
        if n < 0 or T < 1:
            raise ValueError(f"packed layout of {n} channel-frames x {T} bins")
        self.n, self.T = int(n), int(T)
        self.off_combined = 0
        self.off_lufs = 4 * n * T
        self.off_tp = self.off_lufs + 4 * n
        self.off_meters = _align(self.off_tp + 4 * n, 8)
        self.nbytes = _align(self.off_meters + 8 * N_METERS * n, 8)

    def alloc(self, device=None) -> torch.Tensor:
        return torch.empty(self.nbytes, dtype=torch.uint8, device=device)

    def views(self, buf: torch.Tensor) -> Dict[str, torch.Tensor]:
        """The process_frames output dict over a packed byte buffer (no copies)."""
        if buf.dtype != torch.uint8 or buf.dim() != 1 or buf.numel() < self.nbytes:
            raise ValueError(f"packed buffer must be uint8[{self.nbytes}]")
        n, T = self.n, self.T
        return {"combined": buf[self.off_combined:self.off_lufs].view(torch.float32).view(n, T),
                "lufs_inst": buf[self.off_lufs:self.off_tp].view(torch.float32),
                "true_peak_db": buf[self.off_tp:self.off_tp + 4 * n].view(torch.float32),
                "meters": buf[self.off_meters:self.off_meters + 8 * N_METERS * n].view(torch.float64).view(n, N_METERS)}

    def pack(self, out: Dict[str, torch.Tensor], dst: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Copy separately allocated outputs into a packed buffer (the zero-copy path writes views)."""
        buf = dst if dst is not None else self.alloc(out["combined"].device)
        v = self.views(buf)
        for k in v:
            v[k].copy_(out[k])
        return buf


def gather_to_root(buf: torch.Tensor, recv: Optional[List[torch.Tensor]], async_op: bool = False):
    """Gather every rank's packed block (equal sizes) to rank 0. recv: world buffers on rank 0, None
    elsewhere. Returns the work handle when async_op."""
    import torch.distributed as dist
    return dist.gather(buf, recv if dist.get_rank() == 0 else None, dst=0, async_op=async_op)


def unpack_gathered(recv: List[torch.Tensor], layout: PackedLayout) -> Dict[str, torch.Tensor]:
    """Rank 0: the gathered blocks as one output dict in global channel-frame order (rank-major)."""
    vs = [layout.views(b) for b in recv]
    return {k: torch.cat([v[k] for v in vs]) for k in vs[0]}
