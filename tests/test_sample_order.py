"""CVR_OPT_SAMPLE_ORDER (round 5): the pixel-block work order with each pixel's
samples innermost, and the event batch's per-pixel combining of escapes
before the framebuffer atomics (splat_wave).  Scheduling and summation order
only: against the sample-major order (0) and the oracle the counters must be
equal, every production path's record bit-exact, and the pixels within the
summation-order bound.  Order 0 is the default (order 1 ran
sparse media by default until the empty-region mask made order 0 faster there
too)."""
import numpy as np
import pytest

from parity_util import COUNTERS, assert_pixels_close, oracle_for_scene
from test_gpu_records import _compare, _ctx

pytestmark = pytest.mark.gpu


def _scene(cvr, name):
    if name == "cloud":
        from test_sparse import CLOUD_SMALL
        return cvr.Scene.synthetic("cloud", 0, CLOUD_SMALL)
    return cvr.Scene.synthetic(name)


@pytest.mark.parametrize("name", ["manix", "hetvol", "bucky", "cloud"])
@pytest.mark.parametrize("kernel", ["regenerationSK", "streamingSK"])
def test_sample_orders_agree(cvr, name, kernel):
    scene = _scene(cvr, name)
    W, H, iters = 256, 192, 5
    out = []
    for order in (0, 1, -1):
        c, _, _ = _ctx(cvr, scene, W, H, kernel)
        c.set_option(cvr.OPT_SAMPLE_ORDER, order)
        img, st = c.render_image(W, H, (1, 1), iters)
        out.append((img, st))
        c.close()
    (i0, s0), (i1, s1), (id_, sd) = out
    for k in COUNTERS + ("fetches",):
        assert getattr(s0, k) == getattr(s1, k) == getattr(sd, k), k
    assert np.array_equal(i0[..., 3], i1[..., 3])
    assert_pixels_close(i1[..., :3], i0[..., :3], iters, f"{name} {kernel}: samples innermost vs sample-major")
    assert_pixels_close(id_[..., :3], i0[..., :3], iters, f"{name} {kernel}: default order")


@pytest.mark.parametrize("name", ["manix", "cloud"])
def test_sample_inner_records_bit_exact(cvr, oracle_mod, name):
    """The production launch in order 1 (combining splats), every path's final
    record against the oracle's trace of the same path id."""
    scene = _scene(cvr, name)
    W = H = 128
    iters = 6
    ctx, iv, r2v = _ctx(cvr, scene, W, H)
    ctx.set_option(cvr.OPT_SAMPLE_ORDER, 1)
    ctx.set_resolution(W, H)
    ctx.set_offset(0, 0)
    ctx.set_iterations(iters)
    ctx.set_seed(0)
    n = W * H * iters
    ctx.set_path_range(0, n)
    g = ctx.trace_launch(n)
    orc = oracle_for_scene(oracle_mod, scene)
    c = orc.trace_paths(orc.launch(iv, r2v, (W, H), (W, H), (0, 0), 2, 0), 0, n)
    _compare(g, c, f"{name} order 1 records", mixed=name != "cloud")  # (albedo 1: roulette never ends a path)
    ctx.close()
