"""Per-path bit-exact parity of the production kernel itself.

cvr_trace_launch runs the benchmark's launch (regenerationSK / sortingSK on
the wave-pool scheduler, k_wpool's dense and sparse instances, pixel-block
work order, every scheduling knob at its default) and has each path write its
final record when it ends.  Every path's image id, end flags (escaped /
truncated / roulette), throughput T bits and segment count must equal the
oracle's trace of the same path id (oracle/cvr_oracle.c: the reference's
RegenerationVolPTsk / NaiveVolPTsk walk, RegenerationVolPTsk_kernel.cuh:146-232,
NaiveVolPTsk_kernel.cuh:17-87)."""
import os

import numpy as np
import pytest

from parity_util import TILE_SEED, oracle_for_scene

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _ctx(cvr, scene, W, H, kernel="regenerationSK", iv=None, r2v=None):
    ctx = cvr.Context(0, kernel)
    if scene.is_sparse:
        ctx.set_medium_sparse(scene.sparse_medium)
    else:
        ctx.set_medium(scene.medium)
    if iv is None:
        iv, r2v = cvr.default_camera(W, H)
    ctx.set_camera(iv, r2v, (W, H))
    ctx.init()
    return ctx, iv, r2v


def _compare(g, c, what, mixed=True):
    assert len(g) == len(c)
    for f in ("image_id", "flags", "n_segments"):
        mism = np.nonzero(g[f] != c[f])[0]
        assert mism.size == 0, f"{what}: {f} differs for {mism.size} paths, first {mism[:5]}"
    tb, cb = g["T"].view(np.uint32), c["T"].view(np.uint32)
    both_nan = np.isnan(g["T"]) & np.isnan(c["T"])
    mism = np.nonzero(((tb != cb) & ~both_nan).any(axis=1))[0]
    assert mism.size == 0, f"{what}: T bits differ for {mism.size} paths, first {mism[:5]}"
    if mixed:
        assert (c["flags"] & 1).any() and (c["flags"] == 0).any(), what  # escapes and roulette deaths


def _launch_vs_oracle(ctx, orc, iv, r2v, full, tile, offset, iters, seed, first, count, kid, what, mixed=True):
    ctx.set_resolution(*tile)
    ctx.set_offset(*offset)
    ctx.set_iterations(iters)
    ctx.set_seed(seed)
    ctx.set_path_range(first, count)
    g = ctx.trace_launch(count)
    L = orc.launch(iv, r2v, full, tile, offset, kid, seed)
    c = orc.trace_paths(L, first, count)
    _compare(g, c, what, mixed)
    return g


@pytest.mark.parametrize("kernel", ["regenerationSK", "sortingSK"])
@pytest.mark.parametrize("name", ["manix", "hetvol", "bucky"])
def test_production_launch_per_path_bit_exact(cvr, oracle_mod, name, kernel):
    scene = cvr.Scene.synthetic(name)
    W = H = 256
    iters = 4
    ctx, iv, r2v = _ctx(cvr, scene, W, H, kernel)
    orc = oracle_for_scene(oracle_mod, scene)
    kid = cvr.KERNELS.index(kernel)
    _launch_vs_oracle(ctx, orc, iv, r2v, (W, H), (W, H), (0, 0), iters, 0, 0, W * H * iters, kid, f"{name} {kernel}")


def test_production_launch_records_c2_sample_and_shard(cvr, oracle_mod):
    """C2 (1024^2, 20 it): two whole samples in the benchmark's work order,
    then block shard 5 of 8 of all 20 samples (the per-rank launch of an
    8-GPU render): every launched path bit-exact, the others untouched."""
    from cudavolumerenderer_amd.distributed import block_shard_path_ids
    scene = cvr.Scene.synthetic("manix")
    W = H = 1024
    P = W * H
    ctx, iv, r2v = _ctx(cvr, scene, W, H)
    orc = oracle_for_scene(oracle_mod, scene)
    _launch_vs_oracle(ctx, orc, iv, r2v, (W, H), (W, H), (0, 0), 20, 0, 7 * P, 2 * P, 2, "C2 samples 7-8")
    ctx.set_iterations(20)
    ctx.set_path_range(0, 20 * P)
    ctx.set_block_shard(5, 8)
    g = ctx.trace_launch(20 * P)
    ids = block_shard_path_ids(W, H, 20, 5, 8)
    mask = np.zeros(20 * P, bool)
    mask[ids] = True
    assert (g["n_segments"][~mask] == 0).all()
    sel = ids[::97]  # a spread sample of the shard's paths, traced one by one by the oracle
    L = orc.launch(iv, r2v, (W, H), (W, H), (0, 0), 2, 0)
    c = np.concatenate([orc.trace_paths(L, int(p), 1) for p in sel])
    _compare(g[sel], c, "C2 shard 5/8")


def test_production_launch_records_c4_tiles(cvr, oracle_mod):
    """C4 (2048^2, 256 it, 4x2 tiles): a 2-sample range of every tile with
    that tile's regenerationSK seed (+n_paths per tile)."""
    scene = cvr.Scene.synthetic("manix")
    W = H = 2048
    tw, th = W // 4, H // 2
    P = tw * th
    iters = 256
    ctx, iv, r2v = _ctx(cvr, scene, W, H)
    orc = oracle_for_scene(oracle_mod, scene)
    for k in range(8):
        off = (tw * (k % 4), th * (k // 4))
        s0 = (53 * k + 5) % (iters - 2)
        _launch_vs_oracle(ctx, orc, iv, r2v, (W, H), (tw, th), off, iters, TILE_SEED[2](0, k, P * iters),
                          s0 * P, 2 * P, 2, f"C4 tile {k}")


def test_production_launch_records_c5_sparse(cvr, oracle_mod):
    """C5 (sparse cloud, 4096^2, 20 it): 2 M path ids of sample 11 through
    k_wpool's sparse instance (an unaligned range: path-id work order)."""
    scene = cvr.Scene.synthetic("cloud")
    W = H = 4096
    ctx, iv, r2v = _ctx(cvr, scene, W, H)
    orc = oracle_for_scene(oracle_mod, scene)
    _launch_vs_oracle(ctx, orc, iv, r2v, (W, H), (W, H), (0, 0), 20, 0, 11 * W * H + 123457, 2 << 20, 2,
                      "C5 sample 11")


def test_production_launch_records_bonsai_vdb(cvr, oracle_mod):
    """The reference's bonsai_small.vdb (real data) with its scene camera."""
    scene = cvr.Scene.load(os.path.join(GOLDEN, "bonsai_small.vdb"))
    W = H = 512
    iv, r2v = scene.camera(W, H)
    ctx, _, _ = _ctx(cvr, scene, W, H, "regenerationSK", iv, r2v)
    orc = oracle_for_scene(oracle_mod, scene)
    _launch_vs_oracle(ctx, orc, iv, r2v, (W, H), (W, H), (0, 0), 4, 0, 0, W * H * 4, 2, "bonsai")


def test_production_launch_records_mhd_and_xml(cvr, oracle_mod, tmp_path):
    """Scenes through the MHD loader (convert-mhd semantics) and the Mitsuba
    XML loader with non-unit .vol boxes (quirks Q4 and Q15 change the walk),
    per path through the production launch."""
    import test_gpu_production as tp
    rng = np.random.default_rng(11)
    nz, ny, nx = 56, 40, 48
    z, y, x = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    r = np.sqrt(((x - 23) / 20.0) ** 2 + ((y - 19) / 16.0) ** 2 + ((z - 27) / 24.0) ** 2)
    img = np.clip(1500 * (1.1 - r) + rng.normal(0, 80, r.shape), -1000, 3000).round()
    tp._write_mhd(str(tmp_path / "ct.mhd"), img)
    mhd = cvr.Scene.load(str(tmp_path / "ct.mhd"))
    (tmp_path / "xml").mkdir()
    xml = tp.make_xml_scene(cvr, tmp_path / "xml")
    assert not np.allclose(np.array(xml.medium.box_max) - np.array(xml.medium.box_min), 1.0)
    for name, scene in (("mhd", mhd), ("xml", xml)):
        W = H = 256
        iv, r2v = scene.camera(W, H)
        ctx, _, _ = _ctx(cvr, scene, W, H, "regenerationSK", iv, r2v)
        orc = oracle_for_scene(oracle_mod, scene)
        _launch_vs_oracle(ctx, orc, iv, r2v, (W, H), (W, H), (0, 0), 4, 3, 0, W * H * 4, 2, name)


def test_production_launch_records_ragged_and_tiny(cvr, oracle_mod):
    """Edge shapes of the launch: image sides that are not multiples of the
    8x8 pixel block (the work order falls back to path-id order), a ragged
    tile at an offset, a contiguous shard of a ragged image, a shard whose
    rank owns no block, a 1x1 image and an empty range."""
    scene = cvr.Scene.synthetic("manix")
    orc = oracle_for_scene(oracle_mod, scene)
    kid = 2
    # 100x60: 3 whole samples
    W, H = 100, 60
    ctx, iv, r2v = _ctx(cvr, scene, W, H)
    _launch_vs_oracle(ctx, orc, iv, r2v, (W, H), (W, H), (0, 0), 3, 0, 0, W * H * 3, kid, "100x60")
    # an unaligned range of the same image (starts and ends mid-sample)
    _launch_vs_oracle(ctx, orc, iv, r2v, (W, H), (W, H), (0, 0), 3, 5, 4321, 7777, kid, "100x60 mid-sample")
    # contiguous shard 1 of 3 of the ragged image: its third of the ids, the rest untouched
    n = W * H * 3
    ctx.set_resolution(W, H)
    ctx.set_offset(0, 0)
    ctx.set_seed(0)
    ctx.set_path_range(0, n)
    ctx.set_block_shard(1, 3)
    g = ctx.trace_launch(n)
    ctx.set_block_shard(0, 1)
    lo, hi = n // 3, 2 * n // 3
    assert (g["n_segments"][:lo] == 0).all() and (g["n_segments"][hi:] == 0).all()
    L = orc.launch(iv, r2v, (W, H), (W, H), (0, 0), kid, 0)
    _compare(g[lo:hi], orc.trace_paths(L, lo, hi - lo), "100x60 shard 1/3")
    # a ragged 37x23 tile at (50, 30) of a 131x77 image
    W2, H2 = 131, 77
    ctx2, iv2, r2v2 = _ctx(cvr, scene, W2, H2)
    _launch_vs_oracle(ctx2, orc, iv2, r2v2, (W2, H2), (37, 23), (50, 30), 4, 9, 0, 37 * 23 * 4, kid, "tile 37x23")
    # 8x8 image = one pixel block: shard 1 of 3 owns no block and launches nothing
    ctx3, iv3, r2v3 = _ctx(cvr, scene, 8, 8)
    ctx3.set_resolution(8, 8)
    ctx3.set_iterations(2)
    ctx3.set_seed(0)
    ctx3.set_path_range(0, 128)
    ctx3.set_block_shard(1, 3)
    g = ctx3.trace_launch(128)
    assert (g["n_segments"] == 0).all()
    ctx3.set_block_shard(0, 3)
    g = ctx3.trace_launch(128)
    L3 = orc.launch(iv3, r2v3, (8, 8), (8, 8), (0, 0), kid, 0)
    _compare(g, orc.trace_paths(L3, 0, 128), "8x8 shard 0/3", mixed=False)
    # 1x1 image, 64 samples, then an empty range
    ctx4, iv4, r2v4 = _ctx(cvr, scene, 1, 1)
    g = _launch_vs_oracle(ctx4, orc, iv4, r2v4, (1, 1), (1, 1), (0, 0), 64, 0, 0, 64, kid, "1x1", mixed=False)
    assert (g["image_id"] == 0).all()
    ctx4.set_path_range(0, 0)
    assert ctx4.trace_launch(0).size == 0
