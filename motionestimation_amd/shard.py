"""Row-stripe sharding of one frame search across ranks (one process per GPU).

SURVEY §8e: every macroblock is independent, so rank r searches block rows
[b_r, b_{r+1}) (balanced by the kernels' cost model ``me_plan_stripes``:
nbx * (3 (2S+1) + ny) per block row, include/me.h) from
the planes it holds: cur rows [b_r*B, b_{r+1}*B) and ref rows with an S-row
halo.  The only exchange is one gather of the per-stripe MV records to rank 0
(RCCL over xGMI with the ``nccl`` backend, gloo on CPU in the tests).

Record layout on every rank: int32 tensor [2, max_blocks]; row 0 holds the
(mvx, mvy) int16 pair of each block, row 1 the uint32 cost bits.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .engine import plan_stripes


@dataclass(frozen=True)
class Stripe:
    rank: int
    row_begin: int   # block rows [row_begin, row_end)
    row_end: int
    ref_y0: int      # frame rows of the ref halo window [ref_y0, ref_y1)
    ref_y1: int
    cur_y0: int      # frame rows of the cur stripe [cur_y0, cur_y1)
    cur_y1: int
    nbx: int
    max_blocks: int  # padded record count (largest stripe)

    @property
    def nblocks(self) -> int:
        return (self.row_end - self.row_begin) * self.nbx


def plan(width: int, height: int, blk: int, span: int, world: int) -> list:
    bounds = plan_stripes(width, height, blk, span, world)
    nbx = (width + blk - 1) // blk
    max_rows = max(max(bounds[i + 1] - bounds[i] for i in range(world)), 1)
    out = []
    for r in range(world):
        r0, r1 = bounds[r], bounds[r + 1]
        out.append(Stripe(r, r0, r1,
                          max(0, r0 * blk - span), min(height, r1 * blk + span),
                          r0 * blk, min(height, r1 * blk), nbx, max_rows * nbx))
    return out


def pack_records(mv, cost, max_blocks: int):
    """numpy/torch (mv int16 [n,2], cost uint32 [n]) -> int32 [2, max_blocks]."""
    try:
        import torch
        if isinstance(mv, torch.Tensor):
            rec = torch.zeros((2, max_blocks), dtype=torch.int32, device=mv.device)
            n = mv.shape[0]
            rec[0, :n] = mv.contiguous().view(torch.int32).view(-1)
            rec[1, :n] = cost.contiguous().view(torch.int32)
            return rec
    except ImportError:
        pass
    rec = np.zeros((2, max_blocks), np.int32)
    n = mv.shape[0]
    rec[0, :n] = np.ascontiguousarray(mv, np.int16).view(np.int32).reshape(-1)
    rec[1, :n] = np.ascontiguousarray(cost, np.uint32).view(np.int32)
    return rec


def assemble(gathered, stripes) -> tuple:
    """Rank-0 side: list/array of [2, max_blocks] int32 per rank -> full
    (mv int16 [N,2], cost uint32 [N]) in raster order."""
    mvs, costs = [], []
    for st, rec in zip(stripes, gathered):
        rec = np.asarray(rec.cpu() if hasattr(rec, "cpu") else rec)
        n = st.nblocks
        mvs.append(rec[0, :n].copy().view(np.int16).reshape(n, 2))
        costs.append(rec[1, :n].copy().view(np.uint32))
    return np.concatenate(mvs), np.concatenate(costs)


def gather_to_root(rec, stripes, group=None):
    """One torch.distributed gather of every rank's padded records to rank 0.
    Returns the assembled (mv, cost) on rank 0, None elsewhere."""
    import torch
    import torch.distributed as dist
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    bufs = [torch.empty_like(rec) for _ in range(world)] if rank == 0 else None
    dist.gather(rec, bufs, dst=0, group=group)
    if rank != 0:
        return None
    return assemble(bufs, stripes)
