"""The sparse wave pool's four-pool workgroups (round 6, cvr_wpool.hip kWpgSparse): each
wave of a workgroup keeps its own pool, lists and queue cursor, and the workgroup shares
one LDS copy of the launch parameters and the empty-region mask.  A wave-pool grid counts
waves in whole workgroups (cvr_api.cpp wpool_launch_grid), so any grid option renders the
same paths: equal counters and pixels up to the summation order against the default grid,
and per-path records equal to the oracle's with a one-workgroup grid
(RegenerationVolPTsk_kernel.cuh:146-232 through Utilities.cuh:129-155)."""
import pytest

from parity_util import COUNTERS, assert_pixels_close, oracle_for_scene
from test_gpu_records import _compare, _ctx

CLOUD_SMALL = (512, 256, 512)


@pytest.mark.gpu
@pytest.mark.parametrize("grid", [1, 6, 9, 250])
def test_sparse_grid_in_whole_workgroups(cvr, grid):
    scene = cvr.Scene.synthetic("cloud", 0, CLOUD_SMALL)
    W, H, iters = 96, 64, 3
    out = []
    for g in (0, grid):
        c, _, _ = _ctx(cvr, scene, W, H)
        c.set_option(cvr.OPT_GRID, g)
        out.append(c.render_image(W, H, (1, 1), iters))
        c.close()
    (i0, s0), (i1, s1) = out
    for k in COUNTERS + ("fetches",):
        assert getattr(s1, k) == getattr(s0, k), k
    assert s1.paths == W * H * iters
    assert_pixels_close(i1, i0, iters, f"grid {grid} vs the occupancy grid")


@pytest.mark.gpu
def test_sparse_one_workgroup_records_bit_exact(cvr, oracle_mod):
    """Four waves (one workgroup) carry a whole launch: every path's final record
    equals the oracle's."""
    scene = cvr.Scene.synthetic("cloud", 0, CLOUD_SMALL)
    W = H = 48
    iters = 2
    ctx, iv, r2v = _ctx(cvr, scene, W, H)
    ctx.set_option(cvr.OPT_GRID, 4)
    ctx.set_resolution(W, H)
    ctx.set_offset(0, 0)
    ctx.set_iterations(iters)
    ctx.set_seed(0)
    n = W * H * iters
    ctx.set_path_range(0, n)
    g = ctx.trace_launch(n)
    orc = oracle_for_scene(oracle_mod, scene)
    c = orc.trace_paths(orc.launch(iv, r2v, (W, H), (W, H), (0, 0), 2, 0), 0, n)
    _compare(g, c, "one sparse workgroup, records", mixed=False)
    ctx.close()
