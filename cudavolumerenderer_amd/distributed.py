"""Multi-GPU driver: one process per GPU; by default pixel-block shards with
no collective in the data path.

Why this decomposition: paths are independent and the only
shared output is the additive fp32 framebuffer.  With the RNG bound to the
path id, a path renders the same on any rank, so any partition of the
path-id set changes nothing but the order of the fp32 sums.  The default
(block shards, below) partitions it by 8x8 pixel blocks, so the ranks' pixels
are disjoint and there is nothing to sum: RCCL carries only barriers and the
max-over-ranks time.  The other modes, which share pixels between ranks, sum
the framebuffers with one RCCL reduce-scatter per render.

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

Block shards (cvr_set_block_shard; bench.py's default strong-scaling mode):
rank r renders the 8x8 pixel blocks r, r+world, ... of the tile with all
their samples, so every rank keeps the pixel-block work order of the single-
GPU kernel and sees the whole image (balanced whatever the scene); the ranks'
path-id sets partition the launch (block_shard_path_ids).  Their pixels are
disjoint too, so there is nothing to reduce: each rank normalises its own
blocks straight into the node's shared pinned host image (blocks_to_host,
cvr_blocks_to_host), and the data path has no collective at all.
"""
from __future__ import annotations

import ctypes
import os
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


def init_process_group(dist, backend: str, device=None):
    """One process per GPU: the node's ranks over RCCL ("nccl" on ROCm, one
    device each) or gloo.  RCCL's collectives run on a high-priority stream:
    the renders in flight keep every CU busy with persistent wave pools, so
    the reduce-scatter's workgroups should be dispatched ahead of the next
    render's as CU slots free up (the same reason the copy stream is high
    priority in bench.py)."""
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend == "nccl":
        opts = dist.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = True
        dist.init_process_group("nccl", device_id=device, pg_options=opts)
    else:
        dist.init_process_group("gloo")


def block_shard_path_ids(tile_w: int, tile_h: int, samples: int, rank: int, world: int, first_sample: int = 0):
    """Path ids rank `rank` renders under cvr_set_block_shard(rank, world) for
    a launch of samples [first_sample, first_sample + samples) of a tile whose
    sides are multiples of 8 (the pixel-block order): the pixels of blocks
    rank, rank + world, ... (blocks row-major, 8x8 pixels each), every sample.
    A restatement of fill_launch / unit_to_path for tests (numpy array)."""
    import numpy as np
    if tile_w % 8 or tile_h % 8:
        raise ValueError("block shards need tile sides that are multiples of 8")
    bx = tile_w // 8
    nb = bx * (tile_h // 8)
    blocks = np.arange(rank, nb, world)
    lane = np.arange(64)
    px = (blocks[:, None] % bx) * 8 + (lane[None, :] & 7)
    py = (blocks[:, None] // bx) * 8 + (lane[None, :] >> 3)
    pix = (py * tile_w + px).reshape(-1)
    s = np.arange(first_sample, first_sample + samples)
    return (s[:, None] * (tile_w * tile_h) + pix[None, :]).reshape(-1)


def render_block_sharded(render_shard: Callable[[int, int], "object"], rank: int, world: int,
                         reduce: Callable[["object"], "object"] | None):
    """Render this rank's block shard (`render_shard(rank, world)` returns the
    rank's unnormalised accumulator) and combine the ranks' accumulators with
    `reduce` (a sum: all-reduce, reduce or reduce-scatter)."""
    acc = render_shard(rank, world)
    if world > 1 and reduce is not None:
        return reduce(acc)
    return acc


class HostImage:
    """The render's host image (the reference's buffer_out, Image.cpp:9-11
    cudaHostAlloc): pinned memory.  With N ranks it is one /dev/shm mapping
    shared by the node's processes, registered as pinned memory in each, and
    rank r writes its slice [r*chunk, (r+1)*chunk) of the flat float array."""

    def __init__(self, torch, dist, n_floats, rank, world, tag=None, pin=True):
        import numpy as np
        self.n = n_floats
        self.chunk = -(-n_floats // world)
        self.world = world
        self.rank = rank
        self.path = None
        self._registered = False
        if world == 1:
            self.flat = torch.empty(n_floats, dtype=torch.float32, pin_memory=pin)
            self.pinned = pin
            return
        run = tag or (os.environ.get("TORCHELASTIC_RUN_ID", "x") + "_" + os.environ.get("MASTER_PORT", "0"))
        self.path = f"/dev/shm/cvr_bench_image_{run}"
        nbytes = self.chunk * world * 4
        if rank == 0:
            mm = np.memmap(self.path, dtype=np.float32, mode="w+", shape=(self.chunk * world,))
        dist.barrier()
        if rank != 0:
            mm = np.memmap(self.path, dtype=np.float32, mode="r+", shape=(self.chunk * world,))
        self._mm = mm
        self.flat = torch.from_numpy(mm)
        self.pinned = False
        if not pin:  # host tensors only (the gloo CPU tests)
            return
        # hipHostRegister the mapping: the ranks' kernels store their blocks into it over PCIe.
        # An unpinned image would turn every render's output step into a synchronous host-side
        # gather inside the timed region, so a failure here ends the run instead.
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
        self._hip = hip
        rc = hip.hipHostRegister(ctypes.c_void_p(self.flat.data_ptr()), nbytes, 2)  # hipHostRegisterMapped
        if rc != 0:
            # no barrier here (the other ranks may have registered and moved on): drop this rank's
            # view and, on rank 0, the /dev/shm file, so that a failed run leaves no shared memory
            self.flat = None
            self._mm = None
            del mm
            if rank == 0:
                try:
                    os.unlink(self.path)
                except OSError:
                    pass
            raise RuntimeError(f"rank {rank}: hipHostRegister of the shared host image {self.path} failed "
                               f"(hipError {rc}); refusing to run with an unpinned image")
        self.pinned = self._registered = True

    def slice(self, r):
        return self.flat[r * self.chunk:(r + 1) * self.chunk]

    def close(self, dist):
        if self._registered:
            self._hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
            self._hip.hipHostUnregister(ctypes.c_void_p(self.flat.data_ptr()))
        if self.path:
            dist.barrier()
            if self.rank == 0:
                try:
                    os.unlink(self.path)
                except OSError:
                    pass


def block_pixel_index(width: int, height: int, rank: int, world: int):
    """Flat pixel indices of block shard (rank, world) of a width x height
    image (8x8 blocks rank, rank + world, ..., row-major), block by block,
    each block's 64 pixels row-major: k_blocks_to_host's store order."""
    import numpy as np
    if width % 8 or height % 8:
        raise ValueError("block shards need sides that are multiples of 8")
    bx = width // 8
    blocks = np.arange(rank, bx * (height // 8), world)
    lane = np.arange(64)
    px = (blocks[:, None] % bx) * 8 + (lane[None, :] & 7)
    py = (blocks[:, None] // bx) * 8 + (lane[None, :] >> 3)
    return (py * width + px).reshape(-1)


def blocks_to_host(acc_flat, host: "HostImage", width: int, height: int, scale: float):
    """The end of one block-sharded render on this rank: its pixels (the
    blocks of shard (host.rank, host.world)) / scale into their places in the
    shared host image.  No reduction: the ranks' blocks are disjoint.  On the
    GPU one kernel on the current stream stores into the pinned / registered
    image (cvr_blocks_to_host); host tensors (the gloo CPU tests) are indexed."""
    n = width * height * 4
    if acc_flat.is_cuda:
        if not host.pinned:
            raise RuntimeError("blocks_to_host: a device framebuffer needs a pinned host image")
        import torch
        from . import _lib
        _lib.blocks_to_host(acc_flat.data_ptr(), host.flat.data_ptr(), width, height, host.rank, host.world,
                            float(scale), torch.cuda.current_stream().cuda_stream)
        return
    import torch
    idx = torch.from_numpy(block_pixel_index(width, height, host.rank, host.world))
    src = acc_flat[:n].view(-1, 4)
    src = src[idx]
    host.flat[:n].view(-1, 4)[idx] = src / scale


KERNEL_COPY_MAX_BYTES = int(os.environ.get("CVR_KERNEL_COPY_MAX_BYTES", 4 << 20))


def reduce_to_host(acc_flat, part, host: HostImage, scale: float, dist):
    """The end of one render over N ranks: sum the ranks' framebuffers
    (`acc_flat`, padded to host.chunk * world floats) with one reduce-scatter,
    normalise this rank's slice by `scale` (UtilityFunctors::Scale, x / scale,
    Utilities.h:6-15) and copy it into its slice of the host image.  With one
    rank: normalise and copy the whole framebuffer."""
    if host.world > 1:
        if acc_flat.is_cuda and dist.get_backend() == "gloo":
            # gloo (the GPU tests' two ranks on one device): the collective on host copies
            p = part.cpu()
            dist.reduce_scatter_tensor(p, acc_flat.cpu())
            part.copy_(p)
        else:
            dist.reduce_scatter_tensor(part, acc_flat)
        mine = part
    else:
        mine = acc_flat
    dst = host.slice(host.rank)
    if host.pinned and mine.is_cuda and min(dst.numel(), mine.numel()) * 4 <= KERNEL_COPY_MAX_BYTES:
        # small images: normalise + store into the pinned host image in one kernel on the
        # current stream (cvr_image_to_host).  torch's copy_ of a small image into pinned memory
        # blocked the host until the render finished (tools/step_probe.py: 0.5 ms per 256^2
        # render), which serialised the pipelined renders; large images go through the copy
        # engine asynchronously, and the kernel would take CU slots from the renders for longer
        # (C2 1024^2: 4168 Msamples/s with the kernel vs 4353 with the copy engine)
        import torch
        from . import _lib
        n = min(dst.numel(), mine.numel())
        _lib.image_to_host(mine.data_ptr(), dst.data_ptr(), n, float(scale), torch.cuda.current_stream().cuda_stream)
    else:
        if scale != 1.0:
            mine.div_(scale)
        dst.copy_(mine, non_blocking=host.pinned)
