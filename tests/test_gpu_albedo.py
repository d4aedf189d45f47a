"""Uniform albedo read as a constant (CVR_OPT_UNIFORM_ALBEDO): a dense medium
whose albedo voxels all hold the same rgb renders the same image and counters
with the option on (no albedo loads) as with it off (the 8 taps loaded), and
as the oracle; a medium with half of its albedo changed is not treated as
uniform."""
import numpy as np
import pytest

from parity_util import COUNTERS, assert_pixels_close, oracle_for_scene, oracle_image

pytestmark = pytest.mark.gpu

W, H, ITERS = 128, 96, 3


def _render(cvr, medium, uniform):
    c = cvr.Context(0, "regenerationSK")
    c.set_option(cvr.OPT_UNIFORM_ALBEDO, uniform)
    c.set_medium(medium)
    iv, r2v = cvr.default_camera(W, H)
    c.set_camera(iv, r2v, (W, H))
    c.init()
    img, st = c.render_image(W, H, (1, 1), ITERS)
    c.close()
    return img, st


def test_uniform_albedo_constant_equals_loads_and_oracle(cvr, oracle_mod):
    scene = cvr.Scene.synthetic("hetvol")
    alb = np.asarray(scene.albedo).reshape(-1, 4)
    assert (alb[:, :3] == alb[0, :3]).all(), "the hetvol proxy's albedo is uniform"
    on, st_on = _render(cvr, scene.medium, 1)
    off, st_off = _render(cvr, scene.medium, 0)
    for k in COUNTERS:
        assert getattr(st_on, k) == getattr(st_off, k), k
    assert st_on.albedo > 0
    assert np.array_equal(on[..., 3], off[..., 3])
    assert_pixels_close(on[..., :3], off[..., :3], ITERS, "uniform albedo on vs off")
    iv, r2v = cvr.default_camera(W, H)
    ref, rst = oracle_image(oracle_for_scene(oracle_mod, scene), iv, r2v, W, H, (1, 1), ITERS, 2)
    for k in COUNTERS:
        assert getattr(st_on, k) == rst[k], k
    assert_pixels_close(on[..., :3], ref[..., :3], ITERS, "uniform albedo vs oracle")


def test_almost_uniform_albedo_is_loaded(cvr, oracle_mod):
    """Half of the albedo grid changed (x < nx / 2): the grid is not uniform, the
    lookups load it, and the image follows the oracle of the changed grid (it
    differs from the uniform render)."""
    scene = cvr.Scene.synthetic("hetvol")
    nx, ny, nz = scene.dims
    m = scene.medium
    D = np.asarray(scene.density, np.float32).reshape(nz, ny, nx).copy()
    A = np.asarray(scene.albedo, np.float32).reshape(nz, ny, nx, 4).copy()
    A[:, :, : nx // 2, :3] = (0.2, 0.5, 0.7)
    desc, keep = cvr.medium_from_arrays(D, A, tuple(m.box_min), tuple(m.box_max), m.scale, m.max_density, m.g,
                                        tuple(m.roughness), m.eta)
    img, st = _render(cvr, desc, 1)
    orc = oracle_mod.Oracle.from_medium_desc(desc, D, A)
    iv, r2v = cvr.default_camera(W, H)
    ref, rst = oracle_image(orc, iv, r2v, W, H, (1, 1), ITERS, 2)
    for key in COUNTERS:
        assert getattr(st, key) == rst[key], key
    assert_pixels_close(img[..., :3], ref[..., :3], ITERS, "changed voxel vs oracle")
    uni, _ = _render(cvr, scene.medium, 1)
    assert not np.array_equal(uni[..., :3], img[..., :3]), "the changed voxel should change the image"
