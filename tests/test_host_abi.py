"""Host-side checks that need no GPU: the C-ABI library loads and exports
every function include/cvr.h declares, the host-only entry points (tiling,
camera, kernel names, scene loaders, HDR writer) behave like the reference,
and every GPU entry point fails with a status code (never exits) when no
device is present.  The CLI is exercised for argument handling.
"""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "cvr.h")
CLI = os.path.join(ROOT, "cudavolumerenderer_amd", "cvr")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^[A-Za-z_][\w\s\*]*?\b(cvr_\w+)\s*\(", src, flags=re.M)))


def test_library_exports_every_declared_function(cvr):
    lib = cvr.load()
    names = declared_functions()
    assert len(names) >= 39, names
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    nm = subprocess.check_output(["nm", "-D", "--defined-only", cvr.LIB_PATH], text=True)
    exported = set(re.findall(r"\bT (cvr_\w+)", nm))
    assert set(names) <= exported
    # the C ABI carries no C++ or torch types: every exported cvr_* is unmangled
    assert not re.search(r"\bT _Z\w*cvr_(create|launch)", nm)


def test_abi_version_and_kernel_names(cvr):
    lib = cvr.load()
    assert lib.cvr_abi_version() >= 1
    lib.cvr_kernel_name.restype = C.c_char_p
    # Config.h kernel order (naiveSK, naiveMK, regenerationSK, streamingMK, streamingSK, sortingSK)
    for i, k in enumerate(cvr.KERNELS):
        assert lib.cvr_kernel_from_name(k.encode()) == i
        assert lib.cvr_kernel_name(i).decode() == k
    assert lib.cvr_kernel_from_name(b"warpSK") == 6  # CVR_KERNEL_UNKNOWN


def test_gpu_entry_points_fail_cleanly_without_device(cvr):
    if subprocess.run(["bash", "-c", "test -e /dev/kfd"]).returncode == 0:
        pytest.skip("a GPU is present")
    with pytest.raises(cvr.CvrError) as e:
        cvr.Context(0, "regenerationSK")
    assert "CVR_ERR_HIP" in str(e.value)
    lib = cvr.load()
    lib.cvr_last_error.restype = C.c_char_p
    assert lib.cvr_launch_render(None) < 0
    assert lib.cvr_last_error(None) is not None


def test_default_camera_matches_reference_constants(cvr):
    """CudaVolPath.cpp:67-85 + Camera.h:25-71: eye (0,0,100), looking -z,
    up -y (MITSUBA_COMPARABLE), fov_x 0.7 degrees, fov_y = fov_x*H/W."""
    iv, r2v = cvr.default_camera(1024, 768)
    assert list(iv) == [1, 0, 0, 0, 0, -1, 0, 0, 0, 0, -1, 100]
    assert r2v[0] == np.float32(np.tan(np.float32(0.7) * np.float32(np.pi) / np.float32(360)))
    assert r2v[1] == pytest.approx(np.tan(0.7 * 768 / 1024 * np.pi / 360), rel=1e-6)


# ------------------------------------------------------------- scenes ----
def raw_transfer_np(density):
    """RawSceneBuilder::getAlbedoFromDensity (RawSceneBuilder.h:95-140)."""
    f = np.float32
    tf = []
    for (a, b, n) in [((0.02, 0.2, 0.02), (1.0, 0.02, 0.02), 20), ((1.0, 0.02, 0.02), (0.0, 0.02, 1.0), 80)]:
        a, b = np.array(a, f), np.array(b, f)
        for i in range(n):
            tf.append(np.append(a + (f(i) * (b - a) / f(100)), f(1)))
    tf = np.array(tf, f)
    return tf[np.ceil(density * f(len(tf) - 1)).astype(np.int64)]


def test_raw_loader_semantics(cvr, tmp_path):
    """RawSceneBuilder.h:35-90: 32^3 uchar, x fastest, normalised by max;
    scale 40, max_density 1, AABB [-0.5, 0.5]^3, transfer-function albedo."""
    rng = np.random.default_rng(2)
    raw = rng.integers(0, 200, 32 ** 3, dtype=np.uint8)
    p = tmp_path / "vol.raw"
    p.write_bytes(raw.tobytes())
    s = cvr.Scene.load(str(p), "Raw")
    d = s.density
    assert d.shape == (32, 32, 32)
    np.testing.assert_array_equal(d.reshape(-1), raw.astype(np.float32) / np.float32(raw.max()))
    np.testing.assert_array_equal(s.albedo.reshape(-1, 4), raw_transfer_np(d.reshape(-1)))
    m = s.medium
    assert (m.scale, m.max_density) == (40.0, 1.0)
    assert tuple(m.box_min) == (-0.5,) * 3 and tuple(m.box_max) == (0.5,) * 3


def test_raw_loader_rejects_short_file_q16(cvr, tmp_path):
    p = tmp_path / "short.raw"
    p.write_bytes(b"\x01" * 100)
    with pytest.raises(cvr.CvrError):
        cvr.Scene.load(str(p), "Raw")
    with pytest.raises(cvr.CvrError):
        cvr.Scene.load(str(tmp_path / "missing.raw"), "Raw")


def test_synthetic_scenes(cvr):
    """SURVEY.md §8(d) proxies: shapes, value ranges, loader constants."""
    b = cvr.Scene.synthetic("bucky")
    assert b.dims == (32, 32, 32) and b.density.max() == 1.0 and len(b.raw_bytes) == 32 ** 3
    assert b.medium.scale == 40.0
    m = cvr.Scene.synthetic("manix", 0, (64, 58, 64))
    d, a = m.density, m.albedo
    assert d.shape == (64, 58, 64)  # (z, y, x) view of an x-fastest grid
    assert 0 <= d.min() and d.max() <= 1 and (d == 0).mean() > 0.2
    # mhd_to_vdb.py:62-64: albedo = (d, 0, 0), w = 1
    np.testing.assert_array_equal(a[..., 0], d)
    assert (a[..., 1] == 0).all() and (a[..., 2] == 0).all() and (a[..., 3] == 1).all()
    assert m.medium.scale == 100.0 and m.medium.max_density == d.max()
    h = cvr.Scene.synthetic("hetvol")
    assert h.dims == (128, 128, 50)
    assert np.allclose(h.albedo[..., :3], 0.9)
    # deterministic
    m2 = cvr.Scene.synthetic("manix", 0, (64, 58, 64))
    assert np.array_equal(m2.density, d)
    with pytest.raises(cvr.CvrError):
        cvr.Scene.synthetic("nope")


def test_write_hdr_roundtrip(cvr, tmp_path):
    """Image::saveHDR (Image.cpp:58-62, stb Radiance RGBE): decode and compare
    within RGBE precision; NaN pixels (quirk Q22) are written black."""
    rng = np.random.default_rng(4)
    H, W = 5, 7
    img = rng.uniform(0, 3, (H, W, 4)).astype(np.float32)
    img[0, 0, :3] = 0
    img[1, 1, 1] = np.nan
    p = tmp_path / "x.hdr"
    cvr.write_hdr(str(p), img)
    data = p.read_bytes()
    head, _, body = data.partition(b"\n\n")
    assert head.startswith(b"#?RADIANCE") and b"FORMAT=32-bit_rle_rgbe" in head
    res, _, pix = body.partition(b"\n")
    assert res == b"-Y %d +X %d" % (H, W)
    e = np.frombuffer(pix, np.uint8).reshape(H, W, 4).astype(np.float64)
    dec = np.where(e[..., 3:4] > 0, (e[..., :3] + 0.5) * np.ldexp(1.0, (e[..., 3:4] - 136).astype(int)), 0)
    ok = np.ones((H, W), bool)
    ok[1, 1] = False
    # RGBE keeps 8 bits relative to the pixel's largest component
    err = np.abs(dec - img[..., :3]).max(axis=-1)
    assert (err[ok] <= img[..., :3].max(axis=-1)[ok] * 2.0 ** -7).all()
    assert (e[1, 1] == 0).all() and (e[0, 0] == 0).all()


# ---------------------------------------------------------------- CLI ----
@pytest.fixture(scope="module")
def cli():
    if not os.path.exists(CLI):
        subprocess.check_call(["make", "-s", "-C", ROOT, "all"])
    return CLI


def test_cli_help_lists_reference_flags(cli):
    out = subprocess.run([cli, "--help"], capture_output=True, text=True)
    assert out.returncode == 0
    for flag in ("--scene-file", "--scene-type", "--algorithm", "--kernel", "--iterations", "--resolution",
                 "--number-of-tiles", "--trials", "--output"):
        assert flag in out.stdout


def test_cli_argument_errors(cli):
    r = subprocess.run([cli, "--iterations"], capture_output=True, text=True)
    assert r.returncode != 0 and "missing" in r.stderr
    r = subprocess.run([cli, "--synthetic", "bucky", "--kernel", "bogusSK", "--interactive", "0"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0


def test_cli_without_gpu_reports_error(cli):
    if subprocess.run(["bash", "-c", "test -e /dev/kfd"]).returncode == 0:
        pytest.skip("a GPU is present")
    r = subprocess.run([cli, "--synthetic", "bucky", "-r", "64", "64", "-i", "1", "--interactive", "0"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "HIP" in (r.stderr + r.stdout)
