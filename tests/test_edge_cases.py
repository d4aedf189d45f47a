"""Edge cases at the launcher boundary (the reference's own runs
cover only full renders): ragged resolutions and tile remainders (quirk Q1),
tiles that are not multiples of the 8x8 pixel blocks, a single pixel, grids
one voxel thick, an all-zero medium (max_density 0: the Woodcock majorant is
infinite), and launches with no work.  Every render is compared with the CPU
oracle under the per-pixel contract of DESIGN.md §4.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NTHREADS = min(16, os.cpu_count() or 1)
SEED_ADVANCE = {2: "n_paths", 3: "n_paths", 4: 1, 5: 1}  # per-tile reset() of each launcher


def _oracle_image(orc, iv, r2v, W, H, tiles, iters, kernel):
    """The reference's tile loop restated with the oracle (CudaVolPath.cpp:249-347)."""
    tw, th = W // tiles[0], H // tiles[1]
    n_paths = tw * th * iters
    img = np.zeros((H, W, 4), np.float32)
    steps = 0
    for k in range(tiles[0] * tiles[1]):
        ox, oy = tw * (k % tiles[0]), th * (k // tiles[0])
        adv = SEED_ADVANCE.get(kernel, 0)
        sb = (k * n_paths if adv == "n_paths" else k * adv) & 0xFFFFFFFF
        L = orc.launch(iv, r2v, (W, H), (tw, th), (ox, oy), kernel, sb)
        tile, st = orc.render(L, 0, n_paths, nthreads=NTHREADS)
        img[oy:oy + th, ox:ox + tw] = tile / np.float32(iters)
        steps += st.steps
    return img, steps


def _close(gpu, cpu, iters):
    ng, nc = np.isnan(gpu), np.isnan(cpu)
    assert (ng == nc).all()
    gpu, cpu = np.where(ng, 0, gpu), np.where(nc, 0, cpu)
    bound = 2.0 * max(iters - 1, 1) * 2.0 ** -24 * np.maximum(np.abs(gpu), np.abs(cpu)) + 1e-30
    assert (np.abs(gpu - cpu) <= bound).all()


def _render(cvr, medium, W, H, tiles, iters, kernel):
    ctx = cvr.Context(0, kernel)
    ctx.set_medium(medium)
    iv, r2v = cvr.default_camera(W, H)
    ctx.set_camera(iv, r2v, (W, H))
    ctx.init()
    img, st = ctx.render_image(W, H, tiles, iters)
    return img, st, iv, r2v


KERNELS = ["naiveSK", "regenerationSK", "streamingSK", "sortingSK", "streamingMK", "naiveMK"]


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("W,H,tiles", [(37, 23, (3, 2)), (1, 1, (1, 1)), (70, 9, (4, 1)), (64, 40, (1, 3))])
def test_ragged_and_tiny_renders_match_oracle(cvr, oracle_mod, kernel, W, H, tiles):
    """Remainder pixels of an uneven tiling are never rendered (Q1: they stay
    0); tiles of any size run through the schedulers' path-id order."""
    s = cvr.Scene.synthetic("manix", 0, (64, 58, 64))
    iters = 3
    img, st, iv, r2v = _render(cvr, s.medium, W, H, tiles, iters, kernel)
    orc = oracle_mod.Oracle.from_medium_desc(s.medium, s.density, s.albedo)
    ref, steps = _oracle_image(orc, iv, r2v, W, H, tiles, iters, cvr.KERNELS.index(kernel))
    _close(img, ref, iters)
    assert st.steps == steps
    tw, th = W // tiles[0], H // tiles[1]
    assert st.paths == tw * th * iters * tiles[0] * tiles[1]
    assert not img[th * tiles[1]:, :, :3].any() and not img[:, tw * tiles[0]:, :3].any()


@pytest.mark.parametrize("dims", [(1, 5, 7), (9, 1, 4), (6, 8, 1), (1, 1, 1)])
@pytest.mark.parametrize("kernel", ["naiveSK", "regenerationSK"])
def test_one_voxel_thick_grids_match_oracle(cvr, oracle_mod, dims, kernel):
    """res - 1 = 0 on an axis: the grid coordinate is 0 there and every tap
    clamps to the single layer (Volume.h:47-69)."""
    rng = np.random.default_rng(sum(dims))
    nx, ny, nz = dims
    D = rng.random((nz, ny, nx), dtype=np.float32)
    A = np.concatenate([rng.random((nz, ny, nx, 3), dtype=np.float32), np.ones((nz, ny, nx, 1), np.float32)], -1)
    desc, keep = cvr.medium_from_arrays(D, A)
    W = H = 32
    iters = 2
    img, st, iv, r2v = _render(cvr, desc, W, H, (1, 1), iters, kernel)
    orc = oracle_mod.Oracle(D, A)
    ref, steps = _oracle_image(orc, iv, r2v, W, H, (1, 1), iters, cvr.KERNELS.index(kernel))
    _close(img, ref, iters)
    assert st.steps == steps and st.density > 0


@pytest.mark.parametrize("kernel", ["naiveSK", "regenerationSK", "streamingMK"])
def test_all_zero_medium(cvr, oracle_mod, kernel):
    """max_density 0 (an empty VDB): inv_sigma = 1/(scale * 0) = inf, so
    every Woodcock step lands past the box and only the GGX boundary acts;
    no density is ever evaluated and no brick bounds are built."""
    D = np.zeros((8, 8, 8), np.float32)
    A = np.ones((8, 8, 8, 4), np.float32)
    desc, keep = cvr.medium_from_arrays(D, A, max_density=0.0)
    W = H = 48
    iters = 2
    img, st, iv, r2v = _render(cvr, desc, W, H, (1, 1), iters, kernel)
    orc = oracle_mod.Oracle(D, A, max_density=0.0)
    ref, steps = _oracle_image(orc, iv, r2v, W, H, (1, 1), iters, cvr.KERNELS.index(kernel))
    _close(img, ref, iters)
    assert st.steps == steps and st.density == 0 and st.albedo == 0 and st.escaped > 0


def test_launches_without_work(cvr):
    """Zero iterations and an empty path range launch nothing and report zero
    counters; the zero-iteration image is 0/0 as the reference's
    UtilityFunctors::Scale would give (NaN), not a crash."""
    s = cvr.Scene.synthetic("bucky")
    ctx = cvr.Context(0, "regenerationSK")
    ctx.set_medium(s.medium)
    iv, r2v = cvr.default_camera(16, 16)
    ctx.set_camera(iv, r2v, (16, 16))
    ctx.init()
    img, st = ctx.render_image(16, 16, (1, 1), 0)
    assert st.paths == 0 and st.steps == 0
    assert np.isnan(img[..., :3]).all()
    ctx.set_resolution(16, 16)
    ctx.set_iterations(4)
    ctx.set_path_range(100, 0)
    ctx.clear_output()
    ctx.launch_render()
    assert ctx.stats().paths == 0
    assert not ctx.copy_output(16, 16)[..., :3].any()
