"""Workgroup-shared event lists (CVR_OPT_WAVE_PAIR 1, k_wpair): two waves per
workgroup file their boundary and collision events into shared LDS rings and
either wave runs a batch from them.  Scheduling only,
so against the one-wave pool (k_wpool) and the oracle the counters must be
equal and the pixels within the summation-order bound, with full grids,
tiny grids (one or two workgroups: the two waves contend for every list entry)
and block shards.

k_wpair lost 4.1x and is not in the product libcvr.so (round 6): these tests run
against the experiment build only,
  make variant-pair && CVR_LIB=build/variants/pair/libcvr.so pytest tests/test_wave_pair.py -m gpu
and skip otherwise."""
import os

import numpy as np
import pytest

from parity_util import COUNTERS, assert_pixels_close, oracle_for_scene, oracle_image

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif("pair" not in os.environ.get("CVR_LIB", ""),
                                 reason="k_wpair is built only into `make variant-pair` (CVR_LIB)")]


def _ctx(cvr, scene, W, H, kernel, pair, grid=0):
    c = cvr.Context(0, kernel)
    c.set_medium(scene.medium)
    iv, r2v = cvr.default_camera(W, H)
    c.set_camera(iv, r2v, (W, H))
    c.set_option(cvr.OPT_WAVE_PAIR, pair)
    if grid:
        c.set_option(cvr.OPT_GRID, grid)
    c.init()
    return c, iv, r2v


@pytest.mark.parametrize("name", ["manix", "hetvol"])
@pytest.mark.parametrize("kernel", ["regenerationSK", "streamingSK"])
@pytest.mark.parametrize("grid", [0, 2, 6])
def test_pair_equals_single_wave_pool(cvr, name, kernel, grid):
    scene = cvr.Scene.synthetic(name)
    W, H, iters = 256, 256, 4
    out = []
    for pair in (0, 1):
        c, _, _ = _ctx(cvr, scene, W, H, kernel, pair, grid)
        img, st = c.render_image(W, H, (1, 1), iters)
        out.append((img, st))
        c.close()
    (i0, s0), (i1, s1) = out
    for k in COUNTERS + ("fetches",):
        assert getattr(s0, k) == getattr(s1, k), k
    assert np.array_equal(i0[..., 3], i1[..., 3])
    assert_pixels_close(i1[..., :3], i0[..., :3], iters, f"{name} {kernel} grid {grid}: pair vs one wave")


def test_pair_vs_oracle_and_block_shards(cvr, oracle_mod):
    """The pair instance against the oracle's image of the same paths, and its
    block shards (strong multi-GPU split) summing to the whole."""
    scene = cvr.Scene.synthetic("manix")
    W, H, iters = 128, 128, 3
    c, iv, r2v = _ctx(cvr, scene, W, H, "regenerationSK", 1)
    c.set_seed(0)
    img, st = c.render_image(W, H, (1, 1), iters)
    orc = oracle_for_scene(oracle_mod, scene)
    ref, rst = oracle_image(orc, iv, r2v, W, H, (1, 1), iters, 2)
    for k in COUNTERS:
        assert getattr(st, k) == rst[k], k
    assert_pixels_close(img[..., :3], ref[..., :3], iters, "pair vs oracle")
    acc = np.zeros_like(img)
    for r in range(3):
        c.set_block_shard(r, 3)
        c.set_seed(0)  # render_image advances the seed as reset() does
        part, _ = c.render_image(W, H, (1, 1), iters)
        acc += np.where(np.isnan(part), 0, part)
    c.close()
    fin = ~np.isnan(img)
    assert_pixels_close(acc[..., :3][fin[..., :3]], img[..., :3][fin[..., :3]], iters, "pair shards")
