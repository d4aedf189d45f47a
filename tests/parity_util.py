"""Shared parity helpers for the -m gpu tests (HIP path vs the CPU oracle).

Contract:
  * per pixel: the only difference between a HIP render and the oracle's
    render of the same path ids is the order of the fp32 additions into the
    pixel, so |gpu - cpu| <= 2 (n - 1) 2^-24 max(|gpu|, |cpu|) for a pixel
    that receives n contributions (plus 1e-30 for zeros); NaN pixels (quirk
    Q22) must coincide;
  * counters (paths, segments, Woodcock steps, density / albedo evaluations,
    escapes, truncations): equal.
"""
import os

import numpy as np

NTHREADS = min(16, os.cpu_count() or 1)
COUNTERS = ("paths", "segments", "steps", "density", "albedo", "escaped", "truncated")

# per-tile seed advance of each launcher's reset() (RenderKernelLauncher.cu:359,480,573,664):
# kernel id -> seed of tile k given the tile's path count
TILE_SEED = {
    0: lambda seed, k, n: seed,                               # naiveSK
    1: lambda seed, k, n: seed,                               # naiveMK
    2: lambda seed, k, n: (seed + k * n) & 0xFFFFFFFF,        # regenerationSK
    3: lambda seed, k, n: (seed + k * n) & 0xFFFFFFFF,        # streamingMK
    4: lambda seed, k, n: (seed + k) & 0xFFFFFFFF,            # streamingSK
    5: lambda seed, k, n: (seed + k) & 0xFFFFFFFF,            # sortingSK
}


def assert_pixels_close(gpu, cpu, n_contrib, what=""):
    ng, nc = np.isnan(gpu), np.isnan(cpu)
    assert (ng == nc).all(), f"{what}: NaN pattern differs: gpu {ng.sum()} cpu {nc.sum()}"
    gpu = np.where(ng, 0, gpu)
    cpu = np.where(nc, 0, cpu)
    bound = 2.0 * max(n_contrib - 1, 1) * 2.0 ** -24 * np.maximum(np.abs(gpu), np.abs(cpu)) + 1e-30
    diff = np.abs(gpu.astype(np.float64) - cpu.astype(np.float64))
    bad = diff > bound
    assert not bad.any(), (f"{what}: {bad.sum()} pixels out of tolerance; worst diff {diff.max()} "
                           f"at {np.unravel_index(np.argmax(diff - bound), diff.shape)}")


def oracle_for_scene(oracle_mod, scene):
    """The oracle over a loaded or synthetic scene (dense or leaf storage)."""
    if scene.is_sparse:
        table, dens, alb, bg = scene.leaves()
        d = scene.sparse_medium
        return oracle_mod.Oracle.from_leaves(scene.dims, table, dens.reshape(-1, 512),
                                             None if alb is None else alb.reshape(-1, 512, 4), bg,
                                             tuple(d.box_min), tuple(d.box_max), d.scale, d.max_density,
                                             d.g, tuple(d.roughness), d.eta)
    return oracle_mod.Oracle.from_medium_desc(scene.medium, scene.density, scene.albedo)


def oracle_image(orc, iv, r2v, W, H, tiles, iters, kernel, seed=0):
    """The reference's tile loop (CudaVolPath.cpp:249-347) restated with the
    oracle: every tile's paths with that tile's seed, normalised by iters."""
    tw, th = W // tiles[0], H // tiles[1]
    n_paths = tw * th * iters
    img = np.zeros((H, W, 4), np.float32)
    stats = dict.fromkeys(COUNTERS, 0)
    for k in range(tiles[0] * tiles[1]):
        ox, oy = tw * (k % tiles[0]), th * int(np.float32(k) / np.float32(tiles[0]))
        L = orc.launch(iv, r2v, (W, H), (tw, th), (ox, oy), kernel, TILE_SEED[kernel](seed, k, n_paths))
        tile, st = orc.render(L, 0, n_paths, nthreads=NTHREADS)
        img[oy:oy + th, ox:ox + tw] = tile / np.float32(iters)
        for key, v in st.as_dict().items():
            stats[key] += v
    return img, stats


def gpu_range_render(ctx, tile, offset, iterations, seed, first, count):
    """One launch of the production scheduler over path ids [first, first +
    count) of a tile (cvr_set_path_range + cvr_launch_render): the
    unnormalised tile accumulator and the launch's counters."""
    tw, th = tile
    ctx.set_resolution(tw, th)
    ctx.set_iterations(iterations)
    ctx.set_offset(*offset)
    ctx.set_seed(seed)
    ctx.set_path_range(first, count)
    ctx.clear_output()
    ctx.launch_render()
    st = ctx.stats()
    return ctx.copy_output(tw, th), st


def assert_counters_equal(gpu_stats, cpu_stats, what=""):
    cpu = cpu_stats if isinstance(cpu_stats, dict) else cpu_stats.as_dict()
    for k in COUNTERS:
        assert getattr(gpu_stats, k) == cpu[k], f"{what}: counter {k}: gpu {getattr(gpu_stats, k)} cpu {cpu[k]}"
