"""Multi-GPU partitioning of the hot path: one process per GPU, independent
partitions, no collective on the data path.

The reference parallelises with dask: every target tile (reproject.py:230-252,
rectify.py:337-370) and every output chunk (affine.py via dask-image) is an
independent task, and a dim-0 axis (time / band) maps block-wise
(reproject.py:196-205).  On MI355X a single launch already covers all tiles of
a raster, so ranks split the work along the two axes that need no exchange:

* ``slice_shard``  — dim-0 slices of an (n, H, W) cube; each rank owns whole
                     rasters (weak scaling; the bench's partition);
* ``band_shard``   — target tile rows of one raster; each rank holds only the
                     source rows its tiles read (``ReprojectPlan.source_rows_for``)
                     and writes disjoint target rows (strong scaling of one
                     raster; a 40960^2 f32 source needs 6.7 GB, so this is for
                     rasters that exceed one GPU or for latency).

Collectives appear only around the data path: ``max_over_ranks`` (the bench's
clock) and ``gather_rows`` (assembling a result on one rank when asked).
"""

from __future__ import annotations

import os
from dataclasses import dataclass


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


def band_shard(plan, world: int, rank: int) -> BandShard:
    """Target rows of `rank`, aligned to whole tile rows (so every rank runs
    the same per-tile windows as the single-GPU launch), and the source rows
    they read.  Ranks beyond the number of tile rows get an empty band."""
    nty = plan.num_tiles[1]
    t0, t1 = balanced_range(nty, world, rank)
    r0 = min(t0 * plan.tile_height, plan.dst_height)
    r1 = min(t1 * plan.tile_height, plan.dst_height)
    if r1 <= r0:
        return BandShard(rank, world, r0, r0, 0, 0)
    j0, j1 = plan.source_rows_for(r0, r1)
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
