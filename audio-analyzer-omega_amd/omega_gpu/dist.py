"""Multi-GPU layout for the per-frame path: one process per GPU, channel-frames
sharded in contiguous blocks of the batch axis (weak scaling), and each rank's per-frame outputs
gathered to rank 0 over RCCL (backend "nccl"), overlapped with the next batch by the caller. Two
stream layouts: every rank owns whole streams (bench.py: one independent stream per rank, the meter
aggregates need no exchange), or one stream's frames are split over the ranks in time
(TimeShardExchange below: the meters' history is all-gathered before the local meter update).

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


# ---- time-sharded streams: the meter aggregates' history exchange ----
#
# When one stream's consecutive frames are split over the ranks (rank r holds frames [a_r, b_r) of the
# same stream, for every channel), the aggregates of a frame read the LUFS_inst of the 3599 frames
# before it and the true peaks of the 59 before it (the deques of professional_meters.py:20-25, used
# at :249-279) -- frames other ranks computed. Per global batch every rank (1) computes its shard's
# LUFS_inst and true peaks (the batch launch without meters), (2) all-gathers its shard's last 3599 /
# 59 values (~30 KB per channel), (3) loads the stream's history before a_r into its meter state (reset,
# then the history fed through omega_meter_update with its outputs discarded: the device state ends
# exactly as if it had metered those frames) and (4) meters its shard. The tails of all ranks also
# carry the stream into the next global batch. The result equals one context metering the whole
# stream, bitwise (tests/test_dist.py over gloo, tests/test_gpu_parity.py on the device).

LUFS_HIST = 3599  # the 3600-deep integrated deque minus the frame itself
TP_HIST = 59      # the 60-deep peak-hold deque minus the frame itself


def stream_history(prev_li: torch.Tensor, prev_tp: torch.Tensor, tails: List[Tuple[torch.Tensor, torch.Tensor]],
                   upto: int, nl: int = LUFS_HIST, nt: int = TP_HIST) -> Tuple[torch.Tensor, torch.Tensor]:
    """The stream's last nl LUFS_inst / nt true-peak rows before shard `upto` of this global batch:
    prev (the stream before the batch) ++ the tails of shards 0..upto-1, cut to the last nl / nt rows.
    Each tail holds the last <= nl / nt rows of its shard, so nothing earlier than a cut tail is needed."""
    li = torch.cat([prev_li] + [t[0] for t in tails[:upto]])[-nl:] if nl > 0 else prev_li[:0]
    tp = torch.cat([prev_tp] + [t[1] for t in tails[:upto]])[-nt:] if nt > 0 else prev_tp[:0]
    return li, tp


def history_frames(li: torch.Tensor, tp: torch.Tensor, fill: float = -100.0) -> Tuple[torch.Tensor, torch.Tensor]:
    """LUFS_inst / true-peak rows to feed through the meter update as pseudo-frames: one frame per
    LUFS row, the true peaks aligned to the last rows (older frames get `fill`: they leave the 60-deep
    peak hold before any real frame is metered)."""
    n = li.shape[0]
    full = torch.full_like(li, fill)
    k = min(n, tp.shape[0])
    if k:
        full[n - k:] = tp[tp.shape[0] - k:]
    return li, full


class TimeShardExchange:
    """Per-rank carrier of the stream history across global batches for a time-sharded stream of C
    channels (rows = frames, columns = channels; float32 like the device's LUFS_inst / true peaks)."""

    def __init__(self, channels: int, device=None, nl: int = LUFS_HIST, nt: int = TP_HIST):
        self.C, self.nl, self.nt = int(channels), int(nl), int(nt)
        self.prev_li = torch.empty(0, self.C, dtype=torch.float32, device=device)
        self.prev_tp = torch.empty(0, self.C, dtype=torch.float32, device=device)

    def _block(self, li: torch.Tensor, tp: torch.Tensor) -> torch.Tensor:
        """Fixed-size message: nl LUFS rows, nt true-peak rows, two count rows (all_gather needs equal
        sizes; a shard shorter than nl / nt sends fewer rows)."""
        blk = torch.zeros(self.nl + self.nt + 2, self.C, dtype=torch.float32, device=li.device)
        tl, tt = li[-self.nl:] if self.nl else li[:0], tp[-self.nt:] if self.nt else tp[:0]
        blk[:tl.shape[0]] = tl
        blk[self.nl:self.nl + tt.shape[0]] = tt
        blk[-2, 0], blk[-1, 0] = float(tl.shape[0]), float(tt.shape[0])
        return blk

    def _unblock(self, blk: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        cnt = blk[-2:, 0].cpu()
        nl, nt = int(cnt[0]), int(cnt[1])
        return blk[:nl], blk[self.nl:self.nl + nt]

    def exchange(self, li: torch.Tensor, tp: torch.Tensor, group=None) -> Tuple[torch.Tensor, torch.Tensor]:
        """li, tp: this rank's shard [n, C] in time order. All-gathers every rank's tail and returns the
        stream's history before this rank's first frame (LUFS rows, true-peak rows); advances the
        carried history past the whole global batch."""
        import torch.distributed as dist
        if li.dim() != 2 or li.shape[1] != self.C or tp.shape != li.shape:
            raise ValueError(f"shard values must be [n, {self.C}] (LUFS_inst and true peak alike)")
        world, rank = dist.get_world_size(group), dist.get_rank(group)
        blk = self._block(li, tp)
        got = [torch.empty_like(blk) for _ in range(world)]
        dist.all_gather(got, blk, group=group)
        tails = [self._unblock(b) for b in got]
        hist = stream_history(self.prev_li, self.prev_tp, tails, rank, self.nl, self.nt)
        self.prev_li, self.prev_tp = stream_history(self.prev_li, self.prev_tp, tails, world, self.nl, self.nt)
        return hist


def meter_time_shard(engine, li: torch.Tensor, tp: torch.Tensor, hist: Tuple[torch.Tensor, torch.Tensor]):
    """Step (3)-(4) on one rank: load the exchanged history into the engine's meter state, then meter
    the shard. `engine` offers load_meter_history(li, tp) (omega_gpu.Engine: omega_meter_load_history,
    one kernel writing the state) or else reset_meters() + meter_update(li, tp, n_frames) over [n, C]
    rows (the history replayed as pseudo-frames; the CPU stand-in of the tests). Returns the shard's
    meters [n * C, 5]."""
    hl, ht = hist
    if hasattr(engine, "load_meter_history"):
        k = min(ht.shape[0], hl.shape[0])
        engine.load_meter_history(hl.contiguous(), ht[ht.shape[0] - k:].contiguous())
    else:
        engine.reset_meters()
        hl, ht = history_frames(*hist)
        if hl.shape[0]:
            engine.meter_update(hl.contiguous(), ht.contiguous(), hl.shape[0])
    return engine.meter_update(li.contiguous(), tp.contiguous(), li.shape[0])
