"""Multi-GPU driver: one process per GPU, sample (path-id) sharding, one
RCCL all-reduce of the framebuffer.

Why this decomposition: paths are independent and the only
shared output is the additive fp32 framebuffer.  With the RNG bound to the
path id, a path renders the same on any rank, so splitting the path-id range
[0, n_paths) into contiguous shards changes nothing but the order of the fp32
sums.  The only exchange is one sum-reduce of W*H*4 floats over xGMI (16 MiB
at 1024^2) per render.  Image tiles are not used for the split because tile
costs are very uneven (background vs volume).

Weak scaling (bench.py): each rank renders its own `iterations` samples per
pixel; the job renders iterations*world samples per pixel in total.

Tile sharding (BASELINE C4, `--number-of-tiles 4 2` over 8 GPUs, tile k ->
GPU k) is the reference's own decomposition and is kept as the second mode:
rank r renders tiles r, r+world, ... of the tile loop with the seeds those
tiles have in the sequential loop (cvr_render_tiles), into a zeroed full
image, and the same one all-reduce concatenates the disjoint tiles.  Total
work is fixed (strong scaling); its balance depends on the scene (C4 on
8 GPUs: 6.9x, the four centre tiles take 40 ms and the outer ones 30 ms;
on 4 GPUs 3.5x).

Tiles x paths (the third mode, `bench.py --shard tilepaths`): every rank
renders its path-id shard of every tile, each tile with its sequential-loop
seed, so the work splits evenly whatever the tile costs; the all-reduce sums
the ranks' partial images (linear in the paths).
"""
from __future__ import annotations

from typing import Callable, Tuple


def shard_range(n_paths: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous path-id shard [first, first+count) of rank `rank`."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError(f"bad rank/world {rank}/{world}")
    base, rem = divmod(n_paths, world)
    first = rank * base + min(rank, rem)
    count = base + (1 if rank < rem else 0)
    return first, count


def render_sharded(render_range: Callable[[int, int], "object"], n_paths: int, rank: int, world: int,
                   all_reduce: Callable[["object"], None] | None):
    """Render this rank's shard into an accumulator, then sum over ranks.

    `render_range(first, count)` returns the rank's unnormalised accumulator
    (a torch tensor on the rank's device, or any tensor the reducer accepts);
    `all_reduce(acc)` sums it in place across ranks (torch.distributed
    all_reduce over RCCL on the GPU box, gloo in the CPU tests)."""
    first, count = shard_range(n_paths, rank, world)
    acc = render_range(first, count)
    if world > 1 and all_reduce is not None:
        all_reduce(acc)
    return acc


def tile_shard(n_tiles: int, rank: int, world: int) -> Tuple[int, int]:
    """(first_tile, tile_stride) of rank `rank`: tiles rank, rank+world, ...
    (tile k -> GPU k when n_tiles == world)."""
    if world < 1 or not (0 <= rank < world) or n_tiles < 0:
        raise ValueError(f"bad rank/world/tiles {rank}/{world}/{n_tiles}")
    return rank, world


def tiles_of(n_tiles: int, rank: int, world: int):
    first, stride = tile_shard(n_tiles, rank, world)
    return list(range(first, n_tiles, stride))


def render_tiles_sharded(render_tiles: Callable[[int, int], "object"], n_tiles: int, rank: int, world: int,
                         all_reduce: Callable[["object"], None] | None):
    """Render this rank's tiles into a full, zeroed, normalised image, then
    sum over ranks (tiles are disjoint, so the sum is the whole image).

    `render_tiles(first_tile, tile_stride)` returns the rank's image."""
    first, stride = tile_shard(n_tiles, rank, world)
    img = render_tiles(first, stride)
    if world > 1 and all_reduce is not None:
        all_reduce(img)
    return img


def render_tile_paths_sharded(render_tiles_range: Callable[[int, int], "object"], n_paths_per_tile: int, rank: int,
                              world: int, all_reduce: Callable[["object"], None] | None):
    """Render this rank's path-id shard of every tile into a full, zeroed,
    normalised image, then sum over ranks.

    `render_tiles_range(first, count)` renders all tiles with the path range
    [first, first+count) of each tile (cvr_set_path_range + cvr_render_tiles)
    and returns the rank's image."""
    first, count = shard_range(n_paths_per_tile, rank, world)
    img = render_tiles_range(first, count)
    if world > 1 and all_reduce is not None:
        all_reduce(img)
    return img
