"""Quirk flags of SURVEY.md Appendix A that switch between the reference's
behaviour and its fix:

  Q4  worldToAABB precedence (Utilities.cuh:129-132): p - min/extent by
      default, (p - min)/extent with CVR_OPT_WORLD_TO_AABB 1.
  Q11 naiveMK compaction count end - begin - 1 (RenderKernelLauncher.cu:271):
      fixed by default, the reference's drop-one-per-bounce (and its underflow,
      reported as an error) with CVR_OPT_MK_COMPACTION 1.
  Q17 VDB files without an albedo grid (VDBAdapter.cpp:32-37): refused by
      default, loaded with a default albedo through cvr_scene_load_ex.

CPU tests pin the oracle's restatements (the Q11 reference compaction is
re-derived in Python from the fixed walk's per-path records) and the loader;
-m gpu tests compare the HIP path with the oracle.
"""
import os

import numpy as np
import pytest

from parity_util import NTHREADS, assert_counters_equal, assert_pixels_close, oracle_for_scene, oracle_image
from vdb_writer import write_vdb

NAIVE_MK = 1


# ------------------------------------------------------------------ Q11 ----
def _mk_reference_from_records(rec, tile_px, iterations):
    """The reference's naiveMK host loop (RenderKernelLauncher.cu:183-272),
    re-derived from the fixed walk's per-path records: naiveMK re-seeds its
    RNG from (iteration, pixel, depth) at every bounce, so under the
    reference's compaction a path evolves exactly as in the fixed walk until
    it is dropped.  A path with n_segments = 1 + E runs E extends and ends in
    bounce E - 1.  Returns (per-pixel contribution sums (tile_px, 3), error
    (iteration, bounce) or None)."""
    out = np.zeros((tile_px, 3), np.float64)
    for it in range(iterations):
        r = rec[it * tile_px:(it + 1) * tile_px]
        E = r["n_segments"].astype(np.int64) - 1
        missed = (r["flags"] & 4) != 0
        out[missed] += 1.0
        live = set(np.nonzero(E >= 1)[0].tolist())
        b = 0
        n_processed = tile_px
        while n_processed != 0:
            ended = [p for p in live if E[p] == b + 1]
            for p in ended:
                if r["flags"][p] & 1:
                    out[p] += r["T"][p]
            surv = [p for p in live if E[p] > b + 1]
            if not surv:
                return out, (it, b)
            n_processed = len(surv) - 1
            live = set(surv) - {max(surv)}
            b += 1
    return out, None


def _bucky_oracle(cvr, oracle_mod):
    scene = cvr.Scene.synthetic("bucky")
    return scene, oracle_mod.Oracle.from_medium_desc(scene.medium, scene.density, scene.albedo)


@pytest.mark.parametrize("W,H,off", [(8, 8, (124, 124)), (16, 4, (120, 126)), (3, 5, (126, 125)),
                                     (32, 32, (112, 112))])
def test_mk_reference_oracle_matches_python_restatement(cvr, oracle_mod, W, H, off):
    scene, orc = _bucky_oracle(cvr, oracle_mod)
    iters = 3
    iv, r2v = cvr.default_camera(256, 256)
    L = orc.launch(iv, r2v, (256, 256), (W, H), off, NAIVE_MK, 0)
    rec = orc.trace_paths(L, 0, W * H * iters)
    want, werr = _mk_reference_from_records(rec, W * H, iters)
    img, st, err = orc.render_mk_reference(L, iters)
    assert err == werr
    np.testing.assert_allclose(img.reshape(-1, 4)[:, :3], want, rtol=1e-6, atol=0)


def test_mk_reference_drops_paths(cvr, oracle_mod):
    """Where the reference's loop completes, it renders strictly less than the
    fixed walk (one dropped path per bounce)."""
    scene, orc = _bucky_oracle(cvr, oracle_mod)
    iv, r2v = cvr.default_camera(256, 256)
    done = 0
    for oy in range(96, 160, 4):
        L = orc.launch(iv, r2v, (256, 256), (8, 8), (124, oy), NAIVE_MK, 0)
        ref, _, err = orc.render_mk_reference(L, 1)
        if err is not None:
            continue
        fixed, _ = orc.render(L, 0, 64)
        assert ref[..., :3].sum() < fixed[..., :3].sum()
        done += 1
    assert done > 0, "no tile completed without the underflow"


# ------------------------------------------------------------------- Q4 ----
def test_world_to_aabb_fix_is_identity_on_unit_box(cvr, oracle_mod):
    """VDB/Raw/MHD scenes live in the unit box [-0.5, 0.5]^3: there
    p - min/extent == (p - min)/extent, and the fixed coordinate (p - min) *
    ((res - 1)/1) rounds the same, so every path is bit-identical."""
    scene, orc = _bucky_oracle(cvr, oracle_mod)
    iv, r2v = cvr.default_camera(64, 64)
    a = orc.trace_paths(orc.launch(iv, r2v, (64, 64), (64, 64), (0, 0), 2, 0, world_to_aabb=0), 0, 8192)
    b = orc.trace_paths(orc.launch(iv, r2v, (64, 64), (64, 64), (0, 0), 2, 0, world_to_aabb=1), 0, 8192)
    assert (a["T"].view(np.uint32) == b["T"].view(np.uint32)).all()
    assert (a["n_steps"] == b["n_steps"]).all()


def test_world_to_aabb_fix_changes_nonunit_box(oracle_mod):
    """On a non-unit box the two coordinates differ (the reference samples the
    density grid at a shifted point)."""
    rng = np.random.default_rng(4)
    d = rng.uniform(0, 1, (12, 10, 14)).astype(np.float32)
    a = np.ones(d.shape + (4,), np.float32)
    orc = oracle_mod.Oracle(d, a, box_min=(-0.3, -0.2, -0.4), box_max=(0.5, 0.4, 0.8), scale=40.0)
    p_ref = (0.1, 0.1, 0.2)
    # the density coordinate of the reference vs the fix at one point
    ref = orc.density_at(np.subtract(p_ref, np.divide((-0.3, -0.2, -0.4), (0.8, 0.6, 1.2))))
    fix = orc.density_at(np.divide(np.subtract(p_ref, (-0.3, -0.2, -0.4)), (0.8, 0.6, 1.2)))
    assert ref != fix
    iv = np.array([1, 0, 0, 0, 0, -1, 0, 0, 0, 0, -1, 3], np.float32)
    r2v = np.array([0.3, 0.3], np.float32)
    L0 = orc.launch(iv, r2v, (32, 32), (32, 32), (0, 0), 0, 0, world_to_aabb=0)
    L1 = orc.launch(iv, r2v, (32, 32), (32, 32), (0, 0), 0, 0, world_to_aabb=1)
    s0 = orc.trace_paths(L0, 0, 1024)
    s1 = orc.trace_paths(L1, 0, 1024)
    assert s0["n_steps"].sum() > 0
    assert (s0["n_steps"] != s1["n_steps"]).any()


# ------------------------------------------------------------------ Q17 ----
def _density_only_vdb(path, mode="raw"):
    rng = np.random.default_rng(17)
    leaves = []
    for o in [(0, 0, 0), (8, 0, 0), (16, 8, 24), (40, 16, 8), (56, 0, 0), (24, 24, 16)]:
        m = rng.uniform(size=512) < 0.6
        v = np.where(m, rng.uniform(0.05, 1.0, 512), 0.0).astype(np.float32)
        leaves.append((o, m, v))
    write_vdb(str(path), {"density": ({"leaves": leaves, "tiles16": [], "tiles32": []}, 1)}, mode)


def test_density_only_vdb_needs_the_flag(cvr, tmp_path):
    p = tmp_path / "cloud.vdb"
    _density_only_vdb(p)
    with pytest.raises(cvr.CvrError) as e:  # VDBAdapter.cpp:32-37
        cvr.Scene.load(str(p))
    assert "albedo" in str(e.value)


@pytest.mark.parametrize("mode", ["raw", "zip"])
def test_density_only_vdb_default_albedo_dense_and_sparse(cvr, tmp_path, mode):
    p = tmp_path / f"cloud_{mode}.vdb"
    _density_only_vdb(p, mode)
    alb = (0.9, 0.8, 0.7)
    dense = cvr.Scene.load(str(p), "Vdb", default_albedo=alb)
    sparse = cvr.Scene.load(str(p), "VdbSparse", default_albedo=alb)
    assert not dense.is_sparse and sparse.is_sparse
    a = dense.albedo
    assert np.array_equal(a[..., :3], np.broadcast_to(np.float32(alb), a[..., :3].shape))
    assert (a[..., 3] == 1).all()
    table, dens, lalb, bg = sparse.leaves()
    assert lalb is None and tuple(bg) == pytest.approx(alb + (1.0,))
    # the sparse leaves densify to the dense grid
    nx, ny, nz = dense.dims
    assert sparse.dims == dense.dims
    full = np.zeros((table.shape[0] * 8, table.shape[1] * 8, table.shape[2] * 8), np.float32)
    for (lz, ly, lx), s in np.ndenumerate(table):
        if s != 0xFFFFFFFF:
            full[lz * 8:lz * 8 + 8, ly * 8:ly * 8 + 8, lx * 8:lx * 8 + 8] = dens[s]
    assert np.array_equal(full[:nz, :ny, :nx], dense.density)
    assert dense.medium.max_density == sparse.max_density == dense.density.max()


# ----------------------------------------------------------- GPU parity ----
@pytest.mark.gpu
@pytest.mark.parametrize("W,H,off,iters", [(8, 8, (124, 124), 2), (16, 4, (120, 126), 2), (3, 5, (126, 125), 3),
                                           (32, 32, (112, 112), 1), (8, 8, (124, 100), 1)])
def test_gpu_mk_reference_compaction_vs_oracle(cvr, oracle_mod, W, H, off, iters):
    """naiveMK with the reference's compaction (CVR_OPT_MK_COMPACTION 1): the
    HIP per-bounce launches drop the same paths as the oracle, and report the
    underflow at the same iteration and bounce."""
    scene, orc = _bucky_oracle(cvr, oracle_mod)
    iv, r2v = cvr.default_camera(256, 256)
    ctx = cvr.Context(0, "naiveMK")
    ctx.set_medium(scene.medium)
    ctx.set_camera(iv, r2v, (256, 256))
    ctx.set_option(cvr.OPT_MK_COMPACTION, 1)
    ctx.init()
    ctx.set_resolution(W, H)
    ctx.set_iterations(iters)
    ctx.set_offset(*off)
    ctx.clear_output()
    L = orc.launch(iv, r2v, (256, 256), (W, H), off, NAIVE_MK, 0)
    ref, rst, err = orc.render_mk_reference(L, iters)
    if err is not None:
        with pytest.raises(cvr.CvrError) as e:
            ctx.launch_render()
        assert f"iteration {err[0]} bounce {err[1]}" in str(e.value)
        return
    ctx.launch_render()
    st = ctx.stats()
    img = ctx.copy_output(W, H)
    assert_counters_equal(st, rst, "naiveMK reference compaction")
    assert_pixels_close(img, ref, iters, "naiveMK reference compaction")


@pytest.mark.gpu
def test_gpu_mk_reference_compaction_completes_somewhere(cvr, oracle_mod):
    """At least one tile runs the reference's loop to its end, and the GPU
    image then matches the oracle."""
    scene, orc = _bucky_oracle(cvr, oracle_mod)
    iv, r2v = cvr.default_camera(256, 256)
    for oy in range(96, 160, 4):
        L = orc.launch(iv, r2v, (256, 256), (8, 8), (124, oy), NAIVE_MK, 0)
        ref, rst, err = orc.render_mk_reference(L, 1)
        if err is None:
            break
    assert err is None
    ctx = cvr.Context(0, "naiveMK")
    ctx.set_medium(scene.medium)
    ctx.set_camera(iv, r2v, (256, 256))
    ctx.set_option(cvr.OPT_MK_COMPACTION, 1)
    ctx.set_resolution(8, 8)
    ctx.set_iterations(1)
    ctx.set_offset(124, oy)
    ctx.clear_output()
    ctx.launch_render()
    st = ctx.stats()
    assert_counters_equal(st, rst, "naiveMK reference compaction")
    assert_pixels_close(ctx.copy_output(8, 8), ref, 1, "naiveMK reference compaction")


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", ["regenerationSK", "naiveSK", "streamingMK"])
def test_gpu_world_to_aabb_fix_nonunit_box(cvr, oracle_mod, tmp_path, kernel):
    """The Q4 fix on the Mitsuba smoke scene re-pointed at non-unit .vol boxes
    (test_gpu_production.make_xml_scene): the HIP render with
    CVR_OPT_WORLD_TO_AABB 1 equals the oracle's fixed walk, and differs from
    the reference's."""
    from test_gpu_production import make_xml_scene
    scene = make_xml_scene(cvr, tmp_path)
    W = H = 128
    iters = 4
    kid = cvr.KERNELS.index(kernel)
    iv, r2v = scene.camera(W, H)
    ctx = cvr.Context(0, kernel)
    ctx.set_medium(scene.medium)
    ctx.set_camera(iv, r2v, (W, H))
    ctx.set_option(cvr.OPT_WORLD_TO_AABB, 1)
    ctx.init()
    out, st = ctx.render_image(W, H, (1, 1), iters)
    orc = oracle_for_scene(oracle_mod, scene)
    L = orc.launch(iv, r2v, (W, H), (W, H), (0, 0), kid, 0, world_to_aabb=1)
    ref, rst = orc.render(L, 0, W * H * iters, nthreads=NTHREADS)
    assert_counters_equal(st, rst, f"Q4 fix {kernel}")
    assert_pixels_close(out, ref / np.float32(iters), iters, f"Q4 fix {kernel}")
    reproduced, _ = oracle_image(orc, iv, r2v, W, H, (1, 1), iters, kid)
    assert not np.array_equal(np.nan_to_num(reproduced), np.nan_to_num(out))


@pytest.mark.gpu
@pytest.mark.parametrize("scene_type", ["Vdb", "VdbSparse"])
def test_gpu_density_only_vdb_default_albedo_vs_oracle(cvr, oracle_mod, tmp_path, scene_type):
    """A wdas_cloud-style density-only VDB loaded with a default albedo
    (Q17 flag), rendered by the production scheduler (dense or sparse
    instance) vs the oracle."""
    p = tmp_path / "cloud.vdb"
    _density_only_vdb(p, "zip")
    scene = cvr.Scene.load(str(p), scene_type, default_albedo=(0.95, 0.9, 0.85))
    W = H = 128
    iters = 4
    ctx = cvr.Context(0, "regenerationSK")
    if scene.is_sparse:
        ctx.set_medium_sparse(scene.sparse_medium)
    else:
        ctx.set_medium(scene.medium)
    iv, r2v = scene.camera(W, H)
    ctx.set_camera(iv, r2v, (W, H))
    ctx.init()
    out, st = ctx.render_image(W, H, (1, 1), iters)
    ref, rst = oracle_image(oracle_for_scene(oracle_mod, scene), iv, r2v, W, H, (1, 1), iters, 2)
    assert_counters_equal(st, rst, f"density-only {scene_type}")
    assert_pixels_close(out, ref, iters, f"density-only {scene_type}")
    assert st.albedo > 0
