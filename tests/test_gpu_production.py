"""The production scheduler (k_wpool, dense and sparse instances) against the
CPU oracle on BASELINE configs C4 / C5 and on real scene data.

Every test here launches the kernel the benchmark times (regenerationSK ->
scheduler 3, k_wpool; a sparse medium selects its sparse instance) through
cvr_launch_render over a path-id range, and compares the unnormalised tile
accumulator and every counter with the oracle's render of the same path ids
(tests/parity_util.py: summation-order bound per pixel, counters equal).
Path ranges that cover whole samples of the tile (first and count multiples of
tile_w*tile_h) run in the benchmark's pixel-block work order.

Real data: data/vdb/bonsai_small.vdb (the reference's only real volume, read
by VDBAdapter.cpp:15-131 / VDBSceneBuilder.h:40-80), an MHD volume through the
convert-mhd semantics (mhd_to_vdb.py:36-76), and the reference's Mitsuba smoke
scene (data/mitsubaxml/smoke/hetvol.xml, XmlSceneBuilder.h:39-266) re-pointed
at generated .vol files whose boxes are not the unit cube, so that quirk Q4
(worldToAABB precedence, Utilities.cuh:129-132) and Q15 (AABB of the last
.vol read, majorant capped at 1, XmlSceneBuilder.h:108-113) change the walk.
"""
import os
import struct
import zlib

import numpy as np
import pytest

from parity_util import (NTHREADS, TILE_SEED, assert_counters_equal, assert_pixels_close, gpu_range_render,
                         oracle_for_scene, oracle_image)

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
REGEN = 2


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


def _range_vs_oracle(ctx, orc, iv, r2v, W, H, tile, offset, iters, seed, first, count, what):
    img, st = gpu_range_render(ctx, tile, offset, iters, seed, first, count)
    L = orc.launch(iv, r2v, (W, H), tile, offset, REGEN, seed)
    ref, rst = orc.render(L, first, count, nthreads=NTHREADS)
    tile_px = tile[0] * tile[1]
    n_contrib = -(-count // tile_px) + 1
    assert st.paths == count, what
    assert_counters_equal(st, rst, what)
    assert_pixels_close(img, ref, n_contrib, what)
    assert st.density > 0 and st.albedo > 0 and st.escaped > 0, what
    return st


def test_c4_wpool_tile_ranges_vs_oracle(cvr, oracle_mod):
    """BASELINE C4 (manix proxy, 2048^2, 256 it, --number-of-tiles 4 2): in
    every tile, with that tile's regenerationSK seed (+n_paths per tile), a
    3-sample range in the benchmark's work order, plus one unaligned range."""
    scene = cvr.Scene.synthetic("manix")
    W = H = 2048
    iters, tiles = 256, (4, 2)
    tw, th = W // tiles[0], H // tiles[1]
    P = tw * th
    n_paths = P * iters
    ctx, iv, r2v = _ctx(cvr, scene, W, H)
    orc = oracle_for_scene(oracle_mod, scene)
    for k in range(tiles[0] * tiles[1]):
        off = (tw * (k % tiles[0]), th * (k // tiles[0]))
        seed = TILE_SEED[REGEN](0, k, n_paths)
        s0 = (37 * k + 11) % (iters - 3)
        _range_vs_oracle(ctx, orc, iv, r2v, W, H, (tw, th), off, iters, seed, s0 * P, 3 * P, f"tile {k}")
    _range_vs_oracle(ctx, orc, iv, r2v, W, H, (tw, th), (tw, th), iters, TILE_SEED[REGEN](0, 5, n_paths),
                     n_paths // 2 + 12345, 1 << 20, "tile 5 unaligned")


def test_c5_wpool_sparse_sample_vs_oracle(cvr, oracle_mod):
    """BASELINE C5 (2048x1024x2048 sparse cloud proxy, 4096^2, 20 it): one
    whole sample of the frame (16.8 M paths) through k_wpool's sparse
    instance, pixels and counters against the oracle reading the same
    leaves."""
    scene = cvr.Scene.synthetic("cloud")
    assert scene.is_sparse and scene.dims == (2048, 1024, 2048)
    W = H = 4096
    iters = 20
    ctx, iv, r2v = _ctx(cvr, scene, W, H)
    orc = oracle_for_scene(oracle_mod, scene)
    st = _range_vs_oracle(ctx, orc, iv, r2v, W, H, (W, H), (0, 0), iters, 0, 13 * W * H, W * H, "C5 sample 13")
    assert st.fetches < st.density


# ------------------------------------------------------------ real data ----
BONSAI = os.path.join(GOLDEN, "bonsai_small.vdb")


@pytest.fixture(scope="module")
def bonsai(cvr):
    return cvr.Scene.load(BONSAI)


@pytest.mark.parametrize("kernel", ["regenerationSK", "naiveSK"])
def test_bonsai_vdb_render_vs_oracle(cvr, oracle_mod, bonsai, kernel):
    """The reference's bonsai_small.vdb (91x197x256, OpenVDB v224 blosc) at
    1024^2, 20 iterations with the VDB scene camera, through the HIP path
    (cvr_render_image) vs the oracle's tile loop."""
    W = H = 1024
    iters = 20
    iv, r2v = bonsai.camera(W, H)
    ctx, _, _ = _ctx(cvr, bonsai, W, H, kernel, iv, r2v)
    img, st = ctx.render_image(W, H, (1, 1), iters)
    kid = cvr.KERNELS.index(kernel)
    ref, rst = oracle_image(oracle_for_scene(oracle_mod, bonsai), iv, r2v, W, H, (1, 1), iters, kid)
    assert_counters_equal(st, rst, f"bonsai {kernel}")
    assert_pixels_close(img, ref, iters, f"bonsai {kernel}")
    assert st.albedo > 0 and st.density > 0


def test_bonsai_vdb_sparse_read_renders_like_dense(cvr, bonsai):
    """VdbSparse (leaves straight from the file) through k_wpool's sparse
    instance renders the dense read's image with the same counters."""
    W = H = 256
    sp = cvr.Scene.load(BONSAI, "VdbSparse")
    iv, r2v = bonsai.camera(W, H)
    a, _, _ = _ctx(cvr, bonsai, W, H, "regenerationSK", iv, r2v)
    b, _, _ = _ctx(cvr, sp, W, H, "regenerationSK", iv, r2v)
    ia, sa = a.render_image(W, H, (2, 2), 8)
    ib, sb = b.render_image(W, H, (2, 2), 8)
    for k in ("paths", "segments", "steps", "density", "albedo", "escaped"):
        assert getattr(sa, k) == getattr(sb, k), k
    assert_pixels_close(ia, ib, 8, "bonsai sparse vs dense")


def _write_mhd(path, img_zyx):
    nz, ny, nx = img_zyx.shape
    raw = zlib.compress(img_zyx.astype("<i2").tobytes())
    head = ("ObjectType = Image\nNDims = 3\nBinaryData = True\nBinaryDataByteOrderMSB = False\n"
            f"CompressedData = True\nCompressedDataSize = {len(raw)}\nDimSize = {nx} {ny} {nz}\n"
            f"ElementType = MET_SHORT\nElementDataFile = {os.path.basename(path)}.raw\n")
    open(path, "w").write(head)
    open(str(path) + ".raw", "wb").write(raw)


@pytest.mark.parametrize("kernel", ["regenerationSK", "streamingSK"])
def test_mhd_scene_render_vs_oracle(cvr, oracle_mod, tmp_path, kernel):
    """A CT-like MET_SHORT volume through the MHD loader (normalise,
    smoothstep, copyFromArray axis swap, active-box densification), rendered
    through the HIP path with 2x2 tiles vs the oracle."""
    rng = np.random.default_rng(11)
    nz, ny, nx = 56, 40, 48
    z, y, x = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    r = np.sqrt(((x - 23) / 20.0) ** 2 + ((y - 19) / 16.0) ** 2 + ((z - 27) / 24.0) ** 2)
    img = np.clip(1500 * (1.1 - r) + rng.normal(0, 80, r.shape), -1000, 3000).round()
    p = tmp_path / "ct.mhd"
    _write_mhd(str(p), img)
    scene = cvr.Scene.load(str(p))
    assert scene.medium.scale == 100.0
    W = H = 256
    iters = 8
    iv, r2v = scene.camera(W, H)
    ctx, _, _ = _ctx(cvr, scene, W, H, kernel, iv, r2v)
    out, st = ctx.render_image(W, H, (2, 2), iters)
    ref, rst = oracle_image(oracle_for_scene(oracle_mod, scene), iv, r2v, W, H, (2, 2), iters,
                            cvr.KERNELS.index(kernel))
    assert_counters_equal(st, rst, f"mhd {kernel}")
    assert_pixels_close(out, ref, iters, f"mhd {kernel}")
    assert st.albedo > 0


def _write_vol(path, data_zyxc, bbox):
    nz, ny, nx, ch = data_zyxc.shape
    head = b"VOL" + bytes([3]) + struct.pack("<iiiii", 1, nx, ny, nz, ch) + struct.pack("<6f", *bbox)
    open(path, "wb").write(head + data_zyxc.astype("<f4").tobytes())


@pytest.fixture(scope="module")
def xml_scene(cvr, tmp_path_factory):
    return make_xml_scene(cvr, tmp_path_factory.mktemp("xml"))


def make_xml_scene(cvr, d):
    """hetvol.xml (the reference's smoke scene) re-pointed at generated .vol
    files in directory `d`: density box (-1,-2,-3)-(1,2,3), albedo box
    (-0.3,-0.2,-0.4)-(0.5,0.4,0.8); the scene AABB is the albedo's (Q15) and
    densities reach 1.6 > the capped majorant 1."""
    rng = np.random.default_rng(23)
    nz, ny, nx = 24, 20, 28
    z, y, x = np.meshgrid(np.linspace(-1, 1, nz), np.linspace(-1, 1, ny), np.linspace(-1, 1, nx), indexing="ij")
    blob = np.clip(1.6 * (1.0 - np.sqrt(x * x + y * y + z * z)) + rng.normal(0, 0.1, x.shape), 0, 1.6)
    dens = blob.astype(np.float32)[..., None]
    alb = rng.uniform(0.3, 1.0, (nz, ny, nx, 3)).astype(np.float32)
    _write_vol(d / "d.vol", dens, (-1, -2, -3, 1, 2, 3))
    _write_vol(d / "a.vol", alb, (-0.3, -0.2, -0.4, 0.5, 0.4, 0.8))
    xml = open(os.path.join(GOLDEN, "hetvol.xml")).read()
    xml = xml.replace("smoke.vol", "d.vol").replace("albedo.vol", "a.vol").replace('value="800"', 'value="40"')
    (d / "scene.xml").write_text(xml)
    return cvr.Scene.load(str(d / "scene.xml"))


@pytest.mark.parametrize("kernel", ["regenerationSK", "naiveSK", "streamingSK", "naiveMK"])
def test_xml_scene_nonunit_box_render_vs_oracle(cvr, oracle_mod, xml_scene, kernel):
    m = xml_scene.medium
    ext = np.array(m.box_max) - np.array(m.box_min)
    assert tuple(m.box_min) == pytest.approx((-0.3, -0.2, -0.4)) and not np.allclose(ext, 1.0)
    assert m.max_density == 1.0 and xml_scene.density.max() > 1.0  # Q15
    W = H = 256
    iters = 8
    iv, r2v = xml_scene.camera(W, H)
    ctx, _, _ = _ctx(cvr, xml_scene, W, H, kernel, iv, r2v)
    out, st = ctx.render_image(W, H, (1, 1), iters)
    ref, rst = oracle_image(oracle_for_scene(oracle_mod, xml_scene), iv, r2v, W, H, (1, 1), iters,
                            cvr.KERNELS.index(kernel))
    assert_counters_equal(st, rst, f"xml {kernel}")
    assert_pixels_close(out, ref, iters, f"xml {kernel}")
    assert st.albedo > 0


@pytest.mark.parametrize("kernel", ["regenerationSK", "naiveSK"])
def test_xml_scene_per_path_bit_exact(cvr, oracle_mod, xml_scene, kernel):
    """Per-path records on the non-unit box: image id, flags, segment / step /
    density / albedo counts and the throughput bits equal the oracle's."""
    W = H = 64
    iters = 3
    kid = cvr.KERNELS.index(kernel)
    iv, r2v = xml_scene.camera(W, H)
    orc = oracle_for_scene(oracle_mod, xml_scene)
    c = orc.trace_paths(orc.launch(iv, r2v, (W, H), (W, H), (0, 0), kid, 9), 0, W * H * iters)
    ctx, _, _ = _ctx(cvr, xml_scene, W, H, kernel, iv, r2v)
    ctx.set_seed(9)
    ctx.set_resolution(W, H)
    ctx.set_iterations(iters)
    g = ctx.trace_paths(0, W * H * iters)
    for f in ("image_id", "flags", "n_segments", "n_steps", "n_density", "n_albedo"):
        assert (g[f] == c[f]).all(), f
    assert (g["T"].view(np.uint32) == c["T"].view(np.uint32)).all()
    assert c["n_albedo"].sum() > 0
