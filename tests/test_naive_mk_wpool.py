"""naiveMK on the wave pool (round 5, k_wpool's kMedMK instances): d_init (camera
ray on the (iteration, pixel, 0) stream, AABB, the GGX sample at the box) and
every bounce re-seeded from (iteration, pixel, depth) with three unused draws
(NaiveVolPTmk_kernel.cuh:20-151, quirk Q12), scheduled by the wave pool
instead of one work-item per path.  Against the one-path-per-work-item kernel
(CVR_OPT_SCHEDULER 4, k_naive_mk) and the oracle's naiveMK tile loop: equal
counters, pixels within the summation-order bound, on dense, uniform-albedo
and sparse media, with tiles and a segment cap."""
import numpy as np
import pytest

from parity_util import COUNTERS, assert_pixels_close, oracle_for_scene, oracle_image

pytestmark = pytest.mark.gpu


def _scene(cvr, name):
    if name == "cloud":
        from test_sparse import CLOUD_SMALL
        return cvr.Scene.synthetic("cloud", 0, CLOUD_SMALL)
    return cvr.Scene.synthetic(name)


def _render(cvr, scene, W, H, tiles, iters, sched=None, max_seg=None):
    c = cvr.Context(0, "naiveMK")
    if scene.is_sparse:
        c.set_medium_sparse(scene.sparse_medium)
    else:
        c.set_medium(scene.medium)
    iv, r2v = cvr.default_camera(W, H)
    c.set_camera(iv, r2v, (W, H))
    if sched is not None:
        c.set_option(cvr.OPT_SCHEDULER, sched)
    if max_seg is not None:
        c.set_option(cvr.OPT_MAX_SEGMENTS, max_seg)
    c.init()
    img, st = c.render_image(W, H, tiles, iters)
    c.close()
    return img, st, iv, r2v


@pytest.mark.parametrize("name", ["manix", "hetvol", "bucky", "cloud"])
@pytest.mark.parametrize("tiles", [(1, 1), (2, 2)])
def test_mk_wave_pool_equals_per_item_and_oracle(cvr, oracle_mod, name, tiles):
    scene = _scene(cvr, name)
    W, H, iters = 128, 96, 3
    img, st, iv, r2v = _render(cvr, scene, W, H, tiles, iters)
    ref, rst, _, _ = _render(cvr, scene, W, H, tiles, iters, sched=4)
    for k in COUNTERS + ("fetches",):
        assert getattr(st, k) == getattr(rst, k), k
    assert np.array_equal(np.isnan(img), np.isnan(ref))
    assert_pixels_close(img[..., :3], ref[..., :3], iters, f"{name} {tiles}: wave pool vs per item")
    if W * H * iters <= 128 * 96 * 3 and name != "cloud":
        orc = oracle_for_scene(oracle_mod, scene)
        oimg, ost = oracle_image(orc, iv, r2v, W, H, tiles, iters, 1)
        for k in COUNTERS:
            assert getattr(st, k) == ost[k], k
        assert_pixels_close(img[..., :3], oimg[..., :3], iters, f"{name} {tiles}: wave pool vs oracle")


def test_mk_wave_pool_segment_cap(cvr):
    """CVR_OPT_MAX_SEGMENTS: d_init is segment 1, every d_extend one more; a
    path at the cap ends truncated, as walk_mk counts it."""
    scene = _scene(cvr, "hetvol")
    for cap in (1, 2, 4):
        a = _render(cvr, scene, 64, 64, (1, 1), 2, max_seg=cap)[1]
        b = _render(cvr, scene, 64, 64, (1, 1), 2, sched=4, max_seg=cap)[1]
        for k in COUNTERS:
            assert getattr(a, k) == getattr(b, k), (cap, k)
        assert a.truncated > 0
