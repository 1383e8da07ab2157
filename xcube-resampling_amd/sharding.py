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
                     the bench's partition of config 5 (strong scaling);
* ``coarsen_shard`` — the affine / coarsen path (configs 1 and 3): output
                     chunk rows of ONE array, balanced by output rows; each
                     rank holds only the source rows its chunks' dask-image
                     footprints read (the chunk-edge halo included), and runs
                     the same kernel on them (affine.py:277-313);
* ``rectify_shard`` — the rectify path (config 4): target tiles dealt as
                     contiguous raster-order runs balanced by predicted cost
                     (source quads the claim pass scans + target pixels);
                     coordinates and variables are replicated per rank, tiles
                     are independent (rectify.py:347-370, dask.py:41-135).

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


def cost_splits(costs, world: int) -> list[int]:
    """Boundaries 0 = b_0 <= ... <= b_world = n of `world` contiguous runs of
    the n work units with (as nearly as unit granularity allows) equal summed
    cost."""
    if world < 1:
        raise ValueError(f"invalid world size {world}")
    c = np.concatenate([[0.0], np.cumsum(np.asarray(costs, np.float64))])
    n = len(c) - 1
    if c[-1] <= 0:
        return [balanced_range(n, world, r)[0] for r in range(world)] + [n]
    out = [0]
    for target in c[-1] * np.arange(1, world) / world:
        k = int(np.searchsorted(c, target, side="left"))   # nearest boundary to the target
        if k > 0 and (k > n or target - c[k - 1] <= c[k] - target):
            k -= 1
        out.append(min(max(k, out[-1]), n))
    return out + [n]


# ---- affine / coarsen (configs 1 and 3) ------------------------------------------
@dataclass(frozen=True)
class CoarsenShard:
    rank: int
    world: int
    chunk0: int     # output y-chunks [chunk0, chunk1)
    chunk1: int
    row0: int       # output rows [row0, row1)
    row1: int
    src_row0: int   # source rows [src_row0, src_row1) their footprints read
    src_row1: int
    plan: object    # the AffinePlan restricted to the chunks, source rows re-based to src_row0

    @property
    def rows(self) -> tuple[int, int]:
        return self.row0, self.row1

    @property
    def src_rows(self) -> tuple[int, int]:
        return self.src_row0, self.src_row1


def coarsen_shard(plan, world: int, rank: int) -> CoarsenShard:
    """Output chunk rows of `rank` for an affine / coarsen plan
    (``affine.plan_affine``) split over `world` ranks, balanced by output rows.
    Every output pixel depends only on its chunk's dask-image input slice
    (affine.py:336-343: rows [rel_y, rel_y + len_y), which already carries the
    chunk-edge halo the order-1 taps and the NaN dilation of the coarsen need),
    so a rank runs the unchanged kernel on the source rows of its chunks:
    the plan's rel_y is re-based to the first of them.  Plans with a separate
    coarsen pass (median, mode, std, var) or chunks that do not hold whole
    coarsen windows are not split (NotImplementedError)."""
    import dataclasses

    if not 0 <= rank < world:
        raise ValueError(f"invalid rank {rank} for world size {world}")
    if plan.post_agg is not None or plan.chunk_y % plan.div_y != 0:
        raise NotImplementedError("this affine plan cannot be split into output row bands")
    nchunks = len(plan.rel_y)
    rows_per_chunk = plan.chunk_y // plan.div_y
    rows = [min(plan.out_h, (k + 1) * rows_per_chunk) - k * rows_per_chunk
            for k in range(nchunks)]
    cuts = cost_splits(rows, world)
    k0, k1 = cuts[rank], cuts[rank + 1]
    r0 = k0 * rows_per_chunk
    r1 = min(plan.out_h, k1 * rows_per_chunk) if k1 > k0 else r0
    if k1 <= k0:
        return CoarsenShard(rank, world, k0, k0, r0, r0, 0, 0, None)
    rel, ln = plan.rel_y[k0:k1], plan.len_y[k0:k1]
    j0, j1 = int(rel.min()), int((rel + ln).max())
    sub = dataclasses.replace(plan, out_h=r1 - r0, rel_y=(rel - j0).astype(plan.rel_y.dtype),
                              len_y=ln, off_y=plan.off_y[k0:k1], _cache={})
    return CoarsenShard(rank, world, k0, k1, r0, r1, j0, j1, sub)


# ---- rectify (config 4) ----------------------------------------------------------
# predicted K5 + K6 cost of a target tile, in target-pixel units: one source
# quad scanned by the claim pass costs about RECT_QUAD_WEIGHT target pixels of
# resolve + sampling (config 4, round 2: claim 0.60 ms for 19.2 M quads,
# resolve + K6 0.51 ms for 44.6 M pixels)
RECT_QUAD_WEIGHT = 2.7


def rectify_tile_costs(tiles) -> np.ndarray:
    """Predicted cost of every target tile (TILE_INFO records, kernels.py)."""
    quads = np.where(tiles["si0"] >= 0,
                     np.maximum(tiles["swin"].astype(np.int64) - 1, 0) *
                     np.maximum(tiles["shin"].astype(np.int64) - 1, 0), 0)
    return RECT_QUAD_WEIGHT * quads + tiles["th"].astype(np.int64) * tiles["tw"]


@dataclass(frozen=True)
class RectifyShard:
    rank: int
    world: int
    tile0: int      # target tiles [tile0, tile1) in raster (row-major) order
    tile1: int
    row0: int       # target rows [row0, row1) those tiles cover
    row1: int

    @property
    def rows(self) -> tuple[int, int]:
        return self.row0, self.row1


def rectify_shard(tiles, world: int, rank: int) -> RectifyShard:
    """The contiguous run of target tiles `rank` rectifies (``cost_splits``
    over ``rectify_tile_costs``).  Tiles are independent (each reads only its
    source bbox and writes only its pixels), so no exchange is needed."""
    if not 0 <= rank < world:
        raise ValueError(f"invalid rank {rank} for world size {world}")
    cuts = cost_splits(rectify_tile_costs(tiles), world)
    t0, t1 = cuts[rank], cuts[rank + 1]
    if t1 <= t0:
        return RectifyShard(rank, world, t0, t0, 0, 0)
    r0 = int(tiles["r0"][t0])
    r1 = int((tiles["r0"][t0:t1] + tiles["th"][t0:t1]).max())
    return RectifyShard(rank, world, t0, t1, r0, r1)


def merge_tile_runs(parts, tiles, dst_shape, fill):
    """Assemble per-rank rectify results: part = (shard, band (n, r1-r0, W));
    each tile's pixels come from the rank that owns it."""
    n = parts[0][1].shape[0] if parts else 1
    out = np.full((n,) + tuple(dst_shape), fill, dtype=parts[0][1].dtype if parts else float)
    for shard, band in parts:
        for t in range(shard.tile0, shard.tile1):
            r, c = int(tiles["r0"][t]), int(tiles["c0"][t])
            th, tw = int(tiles["th"][t]), int(tiles["tw"][t])
            out[:, r:r + th, c:c + tw] = band[:, r - shard.row0:r - shard.row0 + th, c:c + tw]
    return out


def env_rank() -> tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torchrun environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def max_over_ranks(value: float, device=None) -> float:
    """max of a host scalar over all ranks (the bench's wall clock)."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
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
