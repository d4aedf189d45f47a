"""Multi-rank path on CPU: world_size 2 over gloo.

The GPU ranks render a contiguous path-id shard each and sum the framebuffer
with one all-reduce (cudavolumerenderer_amd/distributed.py).  Here the
per-rank renderer is the CPU oracle (test infrastructure, standing in for
the HIP kernel that -m gpu tests cover), so the test checks the sharding and
the reduction: the 2-rank sum equals the 1-rank render up to fp32
summation order, and the counters add up exactly.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cudavolumerenderer_amd.distributed import (render_sharded, render_tile_paths_sharded, render_tiles_sharded,
                                                shard_range, tiles_of)

W = H = 24
ITERS = 3


@pytest.mark.parametrize("n,world", [(10, 3), (7, 8), (0, 2), (1 << 20, 8), (12345, 1)])
def test_shard_range_partitions(n, world):
    seen = 0
    sizes = []
    for r in range(world):
        a, c = shard_range(n, r, world)
        assert a == seen
        seen += c
        sizes.append(c)
    assert seen == n and max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(n, world, world)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _scene_and_launch():
    import cudavolumerenderer_amd as cvr
    import oracle
    s = cvr.Scene.synthetic("bucky")
    orc = oracle.Oracle.from_medium_desc(s.medium, s.density, s.albedo)
    iv, r2v = cvr.default_camera(W, H)
    L = orc.launch(iv, r2v, (W, H), (W, H), (0, 0), 2, 0)
    return orc, L


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        orc, L = _scene_and_launch()
        stats = {}

        def render_range(first, count):
            img, st = orc.render(L, first, count, nthreads=2)
            stats.update(st.as_dict())
            return torch.from_numpy(img)

        acc = render_sharded(render_range, W * H * ITERS, rank, world, lambda t: dist.all_reduce(t))
        counts = torch.tensor([stats["steps"], stats["escaped"], stats["paths"]], dtype=torch.int64)
        dist.all_reduce(counts)
        if rank == 0:
            np.save(os.path.join(outdir, "img.npy"), acc.numpy())
            np.save(os.path.join(outdir, "counts.npy"), counts.numpy())
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_render_equals_single(tmp_path):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    assert os.path.join(root, "oracle") in sys.path
    mp.start_processes(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True, start_method="fork")
    img = np.load(tmp_path / "img.npy")
    counts = np.load(tmp_path / "counts.npy")
    orc, L = _scene_and_launch()
    ref, st = orc.render(L, 0, W * H * ITERS, nthreads=2)
    assert tuple(counts) == (st.steps, st.escaped, st.paths)
    bound = 2 * ITERS * 2.0 ** -24 * np.maximum(np.abs(img), np.abs(ref)) + 1e-30
    assert (np.abs(img[..., :3] - ref[..., :3]) <= bound[..., :3]).all()


@pytest.mark.parametrize("n,world", [(8, 8), (8, 3), (9, 2), (1, 4), (0, 2)])
def test_tile_shards_cover_each_tile_once(n, world):
    tiles = sorted(t for r in range(world) for t in tiles_of(n, r, world))
    assert tiles == list(range(n))
    if n == world:  # tile k -> GPU k (C4)
        assert all(tiles_of(n, r, world) == [r] for r in range(world))


TW, TH, TILES = 32, 24, (4, 2)  # 8 tiles of 8x12


def _tile_image(orc, iv, r2v, kernel, first, stride):
    """The rank's tiles of the reference tile loop restated with the oracle,
    each with its sequential-loop seed (RenderKernelLauncher.cu:359,573)."""
    tw, th = TW // TILES[0], TH // TILES[1]
    n_paths = tw * th * ITERS
    img = np.zeros((TH, TW, 4), np.float32)
    steps = 0
    for k in range(first, TILES[0] * TILES[1], stride):
        ox, oy = tw * (k % TILES[0]), th * (k // TILES[0])
        sb = {2: k * n_paths, 4: k}.get(kernel, 0)
        L = orc.launch(iv, r2v, (TW, TH), (tw, th), (ox, oy), kernel, sb)
        tile, st = orc.render(L, 0, n_paths, nthreads=2)
        img[oy:oy + th, ox:ox + tw] = tile / np.float32(ITERS)
        steps += st.steps
    return img, steps


def _tile_worker(rank, world, port, outdir, kernel):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import cudavolumerenderer_amd as cvr
        import oracle
        s = cvr.Scene.synthetic("bucky")
        orc = oracle.Oracle.from_medium_desc(s.medium, s.density, s.albedo)
        iv, r2v = cvr.default_camera(TW, TH)
        steps = [0]

        def render_tiles(first, stride):
            img, steps[0] = _tile_image(orc, iv, r2v, kernel, first, stride)
            return torch.from_numpy(img)

        img = render_tiles_sharded(render_tiles, TILES[0] * TILES[1], rank, world, lambda t: dist.all_reduce(t))
        st = torch.tensor([steps[0]], dtype=torch.int64)
        dist.all_reduce(st)
        if rank == 0:
            np.save(os.path.join(outdir, "img.npy"), img.numpy())
            np.save(os.path.join(outdir, "steps.npy"), st.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kernel", [2, 4])  # regenerationSK (seed += n_paths), streamingSK (seed += 1)
def test_two_rank_gloo_tile_sharding_equals_tile_loop(tmp_path, kernel):
    mp.start_processes(_tile_worker, args=(2, _free_port(), str(tmp_path), kernel), nprocs=2, join=True,
                       start_method="fork")
    img = np.load(tmp_path / "img.npy")
    steps = int(np.load(tmp_path / "steps.npy")[0])
    import cudavolumerenderer_amd as cvr
    import oracle
    s = cvr.Scene.synthetic("bucky")
    orc = oracle.Oracle.from_medium_desc(s.medium, s.density, s.albedo)
    iv, r2v = cvr.default_camera(TW, TH)
    ref, ref_steps = _tile_image(orc, iv, r2v, kernel, 0, 1)
    assert steps == ref_steps
    # disjoint tiles: the sum with zeros is exact
    assert np.array_equal(np.nan_to_num(img), np.nan_to_num(ref))


def _tile_paths_image(orc, iv, r2v, kernel, first, count):
    """Every tile of the reference tile loop, paths [first, first+count) of
    each, with the tile's sequential-loop seed, restated with the oracle."""
    tw, th = TW // TILES[0], TH // TILES[1]
    n_paths = tw * th * ITERS
    img = np.zeros((TH, TW, 4), np.float32)
    steps = 0
    for k in range(TILES[0] * TILES[1]):
        ox, oy = tw * (k % TILES[0]), th * (k // TILES[0])
        sb = {2: k * n_paths, 4: k}.get(kernel, 0)
        L = orc.launch(iv, r2v, (TW, TH), (tw, th), (ox, oy), kernel, sb)
        tile, st = orc.render(L, first, count, nthreads=2)
        img[oy:oy + th, ox:ox + tw] = tile / np.float32(ITERS)
        steps += st.steps
    return img, steps


def _tile_paths_worker(rank, world, port, outdir, kernel):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import cudavolumerenderer_amd as cvr
        import oracle
        s = cvr.Scene.synthetic("bucky")
        orc = oracle.Oracle.from_medium_desc(s.medium, s.density, s.albedo)
        iv, r2v = cvr.default_camera(TW, TH)
        steps = [0]

        def render_tiles_range(first, count):
            img, steps[0] = _tile_paths_image(orc, iv, r2v, kernel, first, count)
            return torch.from_numpy(img)

        n_tile = (TW // TILES[0]) * (TH // TILES[1]) * ITERS
        img = render_tile_paths_sharded(render_tiles_range, n_tile, rank, world, lambda t: dist.all_reduce(t))
        st = torch.tensor([steps[0]], dtype=torch.int64)
        dist.all_reduce(st)
        if rank == 0:
            np.save(os.path.join(outdir, "img.npy"), img.numpy())
            np.save(os.path.join(outdir, "steps.npy"), st.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kernel", [2, 4])
def test_three_rank_gloo_tile_path_sharding_equals_tile_loop(tmp_path, kernel):
    """--shard tilepaths: every rank takes a path shard of every tile; the
    sum over ranks is the sequential tile loop up to fp32 summation order."""
    mp.start_processes(_tile_paths_worker, args=(3, _free_port(), str(tmp_path), kernel), nprocs=3, join=True,
                       start_method="fork")
    img = np.load(tmp_path / "img.npy")
    steps = int(np.load(tmp_path / "steps.npy")[0])
    import cudavolumerenderer_amd as cvr
    import oracle
    s = cvr.Scene.synthetic("bucky")
    orc = oracle.Oracle.from_medium_desc(s.medium, s.density, s.albedo)
    iv, r2v = cvr.default_camera(TW, TH)
    ref, ref_steps = _tile_image(orc, iv, r2v, kernel, 0, 1)
    assert steps == ref_steps
    # rgb only: w is a plain store of 1 per render (not an output), so it adds up over ranks
    img, ref = np.nan_to_num(img[..., :3]), np.nan_to_num(ref[..., :3])
    bound = 2 * 3 * ITERS * 2.0 ** -24 * np.maximum(np.abs(img), np.abs(ref)) + 1e-30
    assert (np.abs(img - ref) <= bound).all()


# ------------------------------------------------------------ block shards ----
@pytest.mark.parametrize("tw,th,samples,world", [(24, 16, 3, 2), (24, 16, 3, 3), (64, 8, 2, 8), (8, 8, 1, 4)])
def test_block_shards_partition_path_ids(tw, th, samples, world):
    """cvr_set_block_shard's shards (blocks r, r+world, ..., every sample)
    partition the launch's path ids, and no shard exceeds another by more
    than one block of every sample."""
    from cudavolumerenderer_amd.distributed import block_shard_path_ids
    ids = [block_shard_path_ids(tw, th, samples, r, world) for r in range(world)]
    allids = np.sort(np.concatenate(ids))
    assert np.array_equal(allids, np.arange(tw * th * samples))
    sizes = [len(i) for i in ids]
    assert max(sizes) - min(sizes) <= 64 * samples
    with pytest.raises(ValueError):
        block_shard_path_ids(12, 8, 1, 0, 2)


def _block_worker(rank, world, port, outdir, mode):
    from cudavolumerenderer_amd.distributed import (HostImage, block_shard_path_ids, blocks_to_host,
                                                    init_process_group, reduce_to_host)
    # bench.py's process-group init (env rendezvous, as under torch.distributed.run)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    init_process_group(dist, "gloo")
    try:
        orc, L = _scene_and_launch()
        n = W * H * 4
        host = HostImage(torch, dist, n, rank, world, tag=f"test_{port}", pin=False)
        acc_flat = torch.zeros(host.chunk * world, dtype=torch.float32)
        acc = acc_flat[:n].view(-1, 4).numpy()
        ids = block_shard_path_ids(W, H, ITERS, rank, world)
        steps = 0
        for start in ids[::8]:  # one 8-pixel row of a block: 8 consecutive path ids
            rec = orc.trace_paths(L, int(start), 8)
            steps += int(rec["n_steps"].sum())
            esc = rec[(rec["flags"] & 1) != 0]
            np.add.at(acc[:, :3], esc["image_id"], esc["T"])
            acc[esc["image_id"], 3] = 1.0
        if mode == "blocks":  # bench.py's end of a block-sharded render: own blocks, no reduction
            blocks_to_host(acc_flat, host, W, H, float(ITERS))
        else:  # the reduce-scatter form (weak / tile modes)
            part = torch.empty(host.chunk, dtype=torch.float32)
            reduce_to_host(acc_flat, part, host, float(ITERS), dist)
        counts = torch.tensor([steps, len(ids)], dtype=torch.int64)
        dist.all_reduce(counts)
        dist.barrier()
        if rank == 0:
            np.save(os.path.join(outdir, "img.npy"), host.flat[:n].numpy().reshape(H, W, 4).copy())
            np.save(os.path.join(outdir, "counts.npy"), counts.numpy())
        host.close(dist)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,mode", [(2, "blocks"), (3, "blocks"), (2, "reduce"), (3, "reduce")])
def test_block_shard_gloo_render_equals_single(tmp_path, world, mode):
    """bench.py's default multi-GPU step on CPU: every rank renders its block
    shard (the oracle stands in for k_wpool) and writes its own blocks,
    normalised, into the shared host image (blocks); or one reduce-scatter sums
    the framebuffers and every rank writes its slice (reduce).  The image
    equals the 1-rank render /iterations."""
    mp.start_processes(_block_worker, args=(world, _free_port(), str(tmp_path), mode), nprocs=world, join=True,
                       start_method="fork")
    img = np.load(tmp_path / "img.npy")
    counts = np.load(tmp_path / "counts.npy")
    orc, L = _scene_and_launch()
    ref, st = orc.render(L, 0, W * H * ITERS, nthreads=2)
    ref = ref / np.float32(ITERS)
    assert tuple(counts) == (st.steps, st.paths)
    bound = 2 * ITERS * 2.0 ** -24 * np.maximum(np.abs(img), np.abs(ref)) + 1e-30
    assert (np.abs(img[..., :3] - ref[..., :3]) <= bound[..., :3]).all()
    assert img[..., :3].max() > 0
