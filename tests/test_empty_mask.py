"""The sparse wave pool's empty-region mask (CVR_OPT_EMPTY_MASK, round 5): each
wave stages one bit per super-brick of whole leaves in LDS and loads a Woodcock
point's brick word only when its super-brick holds a cell leaf; every word it
skips is known (0: bound code 0, the zero cell leaf; off the grid the
sentinel's).  Against the same launch loading every word: equal counters
(fetches included: the skipped words are the loaded ones), pixels within the
summation-order bound; the production launch's per-path records against the
oracle (Utilities.cuh:129-155 through the brick bounds of DESIGN.md §3)."""
import numpy as np
import pytest

from parity_util import COUNTERS, assert_pixels_close, oracle_for_scene
from test_gpu_records import _compare, _ctx

EMASK_BITS = 32 * 64  # kEmaskWords words (cvr_walk.h CVR_WPOOL_EMASK_WORDS)


def mask_bits(scene):
    """cvr_set_medium_sparse's mask: (super-brick shift in cells, set bits, total bits)."""
    table, _, _, _ = scene.leaves()
    occ = table != 0xFFFFFFFF
    lz, ly, lx = occ.shape
    cell = occ.copy()  # a leaf has a cell leaf iff it or a forward neighbour exists
    for dz in (0, 1):
        for dy in (0, 1):
            for dx in (0, 1):
                cell[:lz - dz, :ly - dy, :lx - dx] |= occ[dz:, dy:, dx:]
    # each axis of the super-brick grid padded to a power of two (the kernel's
    # index is sz << eshz | sy << eshy | sx)
    k = 0
    while sum((-(-n >> k) - 1).bit_length() for n in (lz, ly, lx)) > EMASK_BITS.bit_length() - 1:
        k += 1
    ez, ey, ex = (-(-n // (1 << k)) for n in (lz, ly, lx))
    pad = np.zeros((ez << k, ey << k, ex << k), bool)
    pad[:lz, :ly, :lx] = cell
    sb = pad.reshape(ez, 1 << k, ey, 1 << k, ex, 1 << k).any(axis=(1, 3, 5))
    return 3 + k, int(sb.sum()), sb.size


@pytest.mark.parametrize("dims", [(96, 48, 104), (512, 256, 512)])
def test_mask_has_clear_super_bricks(cvr, dims):
    """The test scenes exercise the skip: clear super-bricks at leaf (es 3) and
    coarser (es 5: 32^3 cells) granularity."""
    es, on, n = mask_bits(cvr.Scene.synthetic("cloud", 0, dims))
    assert es == (3 if dims[0] < 128 else 5)
    assert 0 < on < n


@pytest.mark.gpu
@pytest.mark.parametrize("dims", [(96, 48, 104), (512, 256, 512)])
@pytest.mark.parametrize("kernel", ["regenerationSK", "naiveSK", "naiveMK"])
def test_empty_mask_changes_nothing(cvr, dims, kernel):
    scene = cvr.Scene.synthetic("cloud", 0, dims)
    W, H, iters = 160, 120, 4
    out = []
    for em in (1, 0):
        c, _, _ = _ctx(cvr, scene, W, H, kernel)
        c.set_option(cvr.OPT_EMPTY_MASK, em)
        out.append(c.render_image(W, H, (2, 1), iters))
        c.close()
    (i1, s1), (i0, s0) = out
    for k in COUNTERS + ("fetches",):
        assert getattr(s1, k) == getattr(s0, k), k
    assert s1.paths == W * H * iters and s1.steps > 0
    assert_pixels_close(i1, i0, iters, f"{dims} {kernel}: mask vs every word loaded")


@pytest.mark.gpu
def test_empty_mask_records_bit_exact(cvr, oracle_mod):
    """The production launch (mask on, the default) at es 5, every path's final
    record against the oracle's trace of the same path id."""
    scene = cvr.Scene.synthetic("cloud", 0, (512, 256, 512))
    W = H = 96
    iters = 4
    ctx, iv, r2v = _ctx(cvr, scene, W, H)
    ctx.set_resolution(W, H)
    ctx.set_offset(0, 0)
    ctx.set_iterations(iters)
    ctx.set_seed(0)
    n = W * H * iters
    ctx.set_path_range(0, n)
    g = ctx.trace_launch(n)
    orc = oracle_for_scene(oracle_mod, scene)
    c = orc.trace_paths(orc.launch(iv, r2v, (W, H), (W, H), (0, 0), 2, 0), 0, n)
    _compare(g, c, "emask es 5 records", mixed=False)
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("bounds,cells", [(0, 1), (1, 1), (2, 0), (3, 0)])
def test_empty_mask_brick_and_cell_layouts(cvr, bounds, cells):
    """Brick sizes 2^3..8^3 (CVR_OPT_BOUNDS 1-3; 0: unbounded, so no mask: the
    words of empty bricks are then 255 << 24) and the 8-tap gather instead of
    cells: the mask only skips loads whose word it knows."""
    scene = cvr.Scene.synthetic("cloud", 0, (96, 48, 104))
    W, H, iters = 128, 96, 3
    out = []
    for em in (1, 0):
        c = cvr.Context(0, "regenerationSK")
        c.set_option(cvr.OPT_BOUNDS, bounds)
        c.set_option(cvr.OPT_CELLS, cells)
        c.set_medium_sparse(scene.sparse_medium)
        iv, r2v = cvr.default_camera(W, H)
        c.set_camera(iv, r2v, (W, H))
        c.init()
        c.set_option(cvr.OPT_EMPTY_MASK, em)
        out.append(c.render_image(W, H, (1, 1), iters))
        c.close()
    (i1, s1), (i0, s0) = out
    for k in COUNTERS + ("fetches",):
        assert getattr(s1, k) == getattr(s0, k), k
    assert_pixels_close(i1, i0, iters, f"bounds {bounds} cells {cells}: mask vs every word loaded")
