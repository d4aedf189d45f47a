"""Committed fixtures (tests/golden/, made by tools/make_golden.py).

CPU: the oracle still reproduces them bit for bit (drift guard), the
synthetic scenes are byte-identical, the RNG streams are unchanged.
GPU: the HIP path reproduces the per-path records without running the
oracle at all (bit-exact).
"""
import hashlib
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = {"bucky": ("bucky", None), "manix_small": ("manix", (64, 58, 64)), "hetvol": ("hetvol", None)}


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def scene_for(cvr, key):
    scene, dims = CASES[key]
    return cvr.Scene.synthetic(scene, 0, dims)


def digest(s):
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(s.density).tobytes())
    h.update(np.ascontiguousarray(s.albedo).tobytes())
    return h.digest()


def same_records(a, b):
    for f in ("image_id", "flags", "n_segments", "n_steps", "n_density", "n_albedo"):
        assert np.array_equal(a[f], b[f]), f
    assert np.array_equal(a["T"].view(np.uint32), b["T"].view(np.uint32))


@pytest.mark.parametrize("key", list(CASES))
def test_oracle_reproduces_golden(cvr, oracle_mod, key):
    g = load(f"oracle_{key}.npz")
    s = scene_for(cvr, key)
    assert digest(s) == g["scene_sha256"].tobytes(), "synthetic scene changed"
    W, H, iters, seed = (int(v) for v in g["meta"])
    orc = oracle_mod.Oracle.from_medium_desc(s.medium, s.density, s.albedo)
    iv, r2v = cvr.default_camera(W, H)
    for kid in (0, 2):
        L = orc.launch(iv, r2v, (W, H), (W, H), (0, 0), kid, seed)
        same_records(orc.trace_paths(L, 0, W * H * iters), g[f"paths_k{kid}"])
        img, _ = orc.render(L, 0, W * H * iters)
        assert np.array_equal(img.view(np.uint32), g[f"image_k{kid}"].view(np.uint32))


def test_rng_streams_golden(oracle_mod):
    g = load("rng_xorwow.npz")
    for i, sd in enumerate(g["seeds"]):
        u, f = oracle_mod.rng_stream(int(sd), g["u32"].shape[1])
        assert np.array_equal(u, g["u32"][i]) and np.array_equal(f.view(np.uint32), g["f32"][i].view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("key", list(CASES))
@pytest.mark.parametrize("kernel", ["naiveSK", "naiveMK", "regenerationSK"])
def test_gpu_reproduces_golden(cvr, key, kernel):
    g = load(f"oracle_{key}.npz")
    W, H, iters, seed = (int(v) for v in g["meta"])
    s = scene_for(cvr, key)
    ctx = cvr.Context(0, kernel)
    ctx.set_medium(s.medium)
    iv, r2v = cvr.default_camera(W, H)
    ctx.set_camera(iv, r2v, (W, H))
    ctx.set_seed(seed)
    ctx.init()
    ctx.set_resolution(W, H)
    ctx.set_iterations(iters)
    kid = cvr.KERNELS.index(kernel)
    same_records(ctx.trace_paths(0, W * H * iters), g[f"paths_k{kid}"])
    # the production launch accumulates the same image (fp32 atomics: order only)
    ctx.clear_output()
    ctx.launch_render()
    img = ctx.copy_output(W, H)
    ref = g[f"image_k{kid}"]
    nan = np.isnan(ref)
    assert np.array_equal(np.isnan(img), nan)
    bound = 2 * iters * 2.0 ** -24 * np.abs(np.where(nan, 0, ref)) + 1e-30
    assert (np.abs(np.where(nan, 0, img) - np.where(nan, 0, ref)) <= bound).all()
