"""Multi-GPU partitioning of the hot path: one process per GPU, independent
partitions, no collective on the data path.

The reference parallelises with dask: every target tile (reproject.py:230-252,
rectify.py:337-370) and every output chunk (affine.py via dask-image) is an
independent task, and a dim-0 axis (time / band) maps block-wise
(reproject.py:196-205).  On MI355X a single launch already covers all tiles of
a raster, so ranks split the work along the two axes that need no exchange:

* ``slice_shard``  — dim-0 slices of an (n, H, W) cube; each rank owns whole
                     rasters (weak scaling; ``bench.py --shard slices``);
* ``band_shard``   — target rows of ONE raster (row granularity, balanced by
                     rows or by algorithmic bytes); each rank holds only the
                     source rows its band reads (``ReprojectPlan.
                     source_rows_read``) and writes disjoint target rows —
                     the bench's partition of config 5 (strong scaling).

Collectives appear only around the data path: ``max_over_ranks`` (the bench's
clock) and ``gather_rows`` (assembling a result on one rank when asked).
"""

from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np


def balanced_range(n: int, world: int, rank: int) -> tuple[int, int]:
    """[a, b) of `n` items for `rank` (first n % world ranks get one more)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"invalid rank {rank} for world size {world}")
    q, r = divmod(n, world)
    a = rank * q + min(rank, r)
    return a, a + q + (1 if rank < r else 0)


def slice_shard(n_slices: int, world: int, rank: int) -> tuple[int, int]:
    """dim-0 slices [i0, i1) owned by `rank`."""
    return balanced_range(n_slices, world, rank)


@dataclass(frozen=True)
class BandShard:
    rank: int
    world: int
    row0: int       # target rows [row0, row1)
    row1: int
    src_row0: int   # global source rows [src_row0, src_row1) the band reads
    src_row1: int

    @property
    def rows(self) -> tuple[int, int]:
        return self.row0, self.row1

    @property
    def src_rows(self) -> tuple[int, int]:
        return self.src_row0, self.src_row1


# K1 time per band on MI355X ~ rows + COST_SRC_ROW_WEIGHT x source rows read
# + COST_DUP_ROW_WEIGHT x target rows whose floor source row repeats the
# previous row's (their requests duplicate lines still in flight: the bands
# near 70 N, where a source row serves ~1.6 target rows, ran 3-5 % above the
# two-term model).  Least-squares fit over the per-rank kernel times of the
# one-GPU rehearsals of 2/4/8-way splits with the round-2 kernel
# (3.45e-5 ms per target row, 2.56e-5 per source row, 1.55e-5 per repeated
# row, 0.023 ms per launch; profiles/r02_band_rehearsal*.jsonl).
COST_SRC_ROW_WEIGHT = 0.74
COST_DUP_ROW_WEIGHT = 0.45


BALANCE_MODELS = ("rows", "bytes", "cost")


def _cumulative_cost(plan, balance: str, out_itemsize: int) -> np.ndarray:
    """F(r), r = 0..H: predicted cost of target rows [0, r) under one model."""
    h = plan.dst_height
    if balance == "rows":
        return np.arange(h + 1, dtype=np.float64)
    if balance == "bytes":
        row_w, src_w = out_itemsize * plan.dst_width, 4 * plan.source_cols_read()
    elif balance == "cost":
        row_w, src_w = 1.0, COST_SRC_ROW_WEIGHT
    else:
        raise ValueError(f"balance must be one of {BALANCE_MODELS}, was {balance!r}")
    lo, hi = plan.row_source_extent()
    valid = hi >= lo
    # cumulative cost F(r) of target rows [0, r): rows + distinct source rows
    # (source rows grow monotonically with target rows here; the running max
    # of the last row read bounds them)
    first = int(lo[valid].min()) if valid.any() else 0
    run_hi = np.maximum.accumulate(np.where(valid, hi, first - 1))
    src_rows = np.concatenate([[0], np.maximum(run_hi - first + 1, 0)])
    f = row_w * np.arange(h + 1) + src_w * src_rows
    if balance == "cost":   # + repeated floor rows (see COST_DUP_ROW_WEIGHT)
        dup = np.zeros(h, bool)
        dup[1:] = (lo[1:] == lo[:-1]) & valid[1:] & valid[:-1]
        f = f + COST_DUP_ROW_WEIGHT * np.concatenate([[0], np.cumsum(dup)])
    return f


def band_splits(plan, world: int, balance: str = "rows", out_itemsize: int = 4) -> list[int]:
    """Target-row boundaries r_0 = 0 <= r_1 <= ... <= r_world = H of a
    `world`-way split of one raster at ROW granularity (K1 takes arbitrary
    row bands: ``xrs_reproject(row_begin, row_end)``; SURVEY §8(e) — whole
    tile rows give a 3/3/3/3/2/2/2/2 split of config 5's 20 tile rows).

    balance="rows":  equal target rows (equal output bytes and gather work);
    balance="bytes": equal algorithmic bytes per band (output + the distinct
                     source rows it reads: at config 5 a target row near 30 N
                     reads 2.6x the source rows of one near 70 N) — the
                     unfitted HBM-bound model, kept as the guard of "cost";
    balance="cost":  equal predicted K1 time: rows + COST_SRC_ROW_WEIGHT x
                     source rows + COST_DUP_ROW_WEIGHT x rows repeating the
                     previous row's floor source row (weights fitted to
                     one-GPU rehearsals; ``split_predictions`` reports every
                     model's balance of a split, so a multi-GPU run shows
                     which one held)."""
    h = plan.dst_height
    if world < 1:
        raise ValueError(f"invalid world size {world}")
    if balance == "rows":
        return [balanced_range(h, world, r)[0] for r in range(world)] + [h]
    f = _cumulative_cost(plan, balance, out_itemsize)
    targets = f[-1] * np.arange(1, world) / world
    cuts = np.searchsorted(f, targets, side="left")
    return [0] + [int(c) for c in cuts] + [h]


def split_predictions(plan, cuts: list[int], out_itemsize: int = 4) -> dict:
    """Per-band cost of the split `cuts` predicted by every balance model,
    relative to the model's mean over the bands, plus each model's max/mean
    (a measured per-rank time series is compared against these)."""
    out = {}
    for m in BALANCE_MODELS:
        f = _cumulative_cost(plan, m, out_itemsize)
        per = np.array([f[b] - f[a] for a, b in zip(cuts[:-1], cuts[1:])], np.float64)
        mean = per.mean() if per.size and per.mean() > 0 else 1.0
        out[m] = {"relative": [round(float(x), 4) for x in per / mean],
                  "max_over_mean": round(float(per.max() / mean), 4) if per.size else 1.0}
    return out


def band_shard(plan, world: int, rank: int, balance: str = "rows",
               out_itemsize: int = 4) -> BandShard:
    """Target rows of `rank` in a row-granular split of one raster
    (``band_splits``) and the global source rows they read
    (``ReprojectPlan.source_rows_read``: exactly the rows K1 touches, so a
    device holds nothing more).  Ranks beyond the number of rows get an
    empty band."""
    if not 0 <= rank < world:
        raise ValueError(f"invalid rank {rank} for world size {world}")
    cuts = band_splits(plan, world, balance, out_itemsize)
    r0, r1 = cuts[rank], cuts[rank + 1]
    if r1 <= r0:
        return BandShard(rank, world, r0, r0, 0, 0)
    j0, j1 = plan.source_rows_read(r0, r1)
    return BandShard(rank, world, r0, r1, j0, j1)


def env_rank() -> tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torchrun environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def max_over_ranks(value: float, device=None) -> float:
    """max of a host scalar over all ranks (the bench's wall clock)."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    if dist.get_backend() == "gloo":
        device = None   # gloo reduces host tensors
    t = torch.tensor([float(value)], dtype=torch.float64,
                     device=device if device is not None else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_rows(local, dst_rows: int, dst: int = 0):
    """Assemble the (n, rows, W) band results of all ranks (in rank order) into
    the whole (n, dst_rows, W) raster on rank `dst` (None elsewhere).  Bands
    differ in height, so they are padded to the tallest band for one
    all_gather."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size()
    n, h, w = local.shape
    sizes = [torch.zeros(1, dtype=torch.int64, device=local.device) for _ in range(world)]
    dist.all_gather(sizes, torch.tensor([h], dtype=torch.int64, device=local.device))
    heights = [int(s.item()) for s in sizes]
    pad = torch.zeros((n, max(heights), w), dtype=local.dtype, device=local.device)
    pad[:, :h] = local
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad)
    if dist.get_rank() != dst:
        return None
    out = torch.cat([p[:, :k] for p, k in zip(parts, heights)], dim=1)
    if out.shape[1] != dst_rows:
        raise ValueError(f"bands cover {out.shape[1]} rows, expected {dst_rows}")
    return out
