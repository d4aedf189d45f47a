"""Sparse (8^3-leaf) medium storage, SURVEY.md §8(d) C5.

cvr_set_medium_sparse stores the grid as leaves and builds the cell-leaf pool
and brick words on the device; rendering must be identical to the dense
upload of the densified grid (only the storage differs).  CPU tests check the
leaf builders and the oracle's leaf storage; -m gpu tests check the HIP path
per path (bit-exact) against the dense upload and the oracle, and C5 at full
size (2048x1024x2048 cloud proxy, 4096^2).
"""
import os

import numpy as np
import pytest

NTHREADS = min(16, os.cpu_count() or 1)
CLOUD_SMALL = (96, 48, 104)  # partial leaves on every axis


def densify(scene):
    """(density (z,y,x), albedo (z,y,x,4)) of a sparse view."""
    table, dens, alb, bg = scene.leaves()
    nx, ny, nz = scene.dims
    lz, ly, lx = table.shape
    D = np.zeros((lz * 8, ly * 8, lx * 8), np.float32)
    A = np.empty((lz * 8, ly * 8, lx * 8, 4), np.float32)
    A[:] = np.asarray(bg, np.float32)
    zz, yy, xx = np.nonzero(table != 0xFFFFFFFF)
    for z, y, x in zip(zz, yy, xx):
        s = table[z, y, x]
        D[z * 8:z * 8 + 8, y * 8:y * 8 + 8, x * 8:x * 8 + 8] = dens[s]
        if alb is not None:
            A[z * 8:z * 8 + 8, y * 8:y * 8 + 8, x * 8:x * 8 + 8] = alb[s]
    return np.ascontiguousarray(D[:nz, :ny, :nx]), np.ascontiguousarray(A[:nz, :ny, :nx])


def sparse_oracle(oracle_mod, scene):
    table, dens, alb, bg = scene.leaves()
    d = scene.sparse_medium
    return oracle_mod.Oracle.from_leaves(scene.dims, table, dens.reshape(-1, 512),
                                         None if alb is None else alb.reshape(-1, 512, 4), bg,
                                         tuple(d.box_min), tuple(d.box_max), d.scale, d.max_density)


# ------------------------------------------------------------------ CPU -----
@pytest.mark.parametrize("name,dims", [("bucky", None), ("manix", (64, 58, 64)), ("hetvol", None)])
def test_dense_to_leaves_roundtrip(cvr, name, dims):
    s = cvr.Scene.synthetic(name, 0, dims)
    table, dens, alb, bg = s.leaves()
    assert not s.is_sparse
    D, A = densify(s)
    assert np.array_equal(D.view(np.uint32), s.density.view(np.uint32))
    assert np.array_equal(A.view(np.uint32), s.albedo.view(np.uint32))
    used = table[table != 0xFFFFFFFF]
    assert np.array_equal(np.sort(used), np.arange(dens.shape[0]))  # slots 0..n-1, each once
    assert dens.shape[0] < table.size or name == "bucky"


def test_cloud_proxy_is_sparse_and_deterministic(cvr):
    a = cvr.Scene.synthetic("cloud", 0, CLOUD_SMALL)
    b = cvr.Scene.synthetic("cloud", 0, CLOUD_SMALL)
    c = cvr.Scene.synthetic("cloud", 9, CLOUD_SMALL)
    assert a.is_sparse and a.medium is None
    with pytest.raises(cvr.CvrError):
        a.density  # noqa: B018  (no dense view)
    ta, da, aa, bga = a.leaves()
    tb, db, _, _ = b.leaves()
    assert np.array_equal(ta, tb) and np.array_equal(da, db)
    assert not np.array_equal(ta, c.leaves()[0])
    assert aa is None and bga == (1.0, 1.0, 1.0, 1.0)
    used = ta != 0xFFFFFFFF
    assert np.array_equal(ta[used], np.arange(used.sum()))  # slots follow the leaf order
    assert (da.reshape(len(da), -1) != 0).any(axis=1).all()  # every stored leaf holds density
    assert 0.05 < used.mean() < 0.4 and a.max_density == float(da.max()) == 1.0
    assert (da >= 0).all() and (da <= 1).all()


def test_oracle_leaf_storage_equals_dense(cvr, oracle_mod):
    s = cvr.Scene.synthetic("cloud", 0, CLOUD_SMALL)
    D, A = densify(s)
    dense = oracle_mod.Oracle(D, A, scale=100.0, max_density=s.max_density)
    sparse = sparse_oracle(oracle_mod, s)
    iv, r2v = cvr.default_camera(64, 64)
    for kernel in (0, 2):
        L = dense.launch(iv, r2v, (64, 64), (64, 64), (0, 0), kernel, 3)
        a = dense.trace_paths(L, 0, 64 * 64 * 2)
        b = sparse.trace_paths(L, 0, 64 * 64 * 2)
        assert a.tobytes() == b.tobytes()
        assert a["n_density"].sum() > 0 and a["n_albedo"].sum() > 0


# ------------------------------------------------------------------ GPU -----
def _ctx(cvr, W, H, kernel, seed=0, bounds=None, cells=1):
    ctx = cvr.Context(0, kernel)
    ctx.set_option(cvr.OPT_CELLS, cells)
    if bounds is not None:
        ctx.set_option(cvr.OPT_BOUNDS, bounds)
    iv, r2v = cvr.default_camera(W, H)
    ctx.set_camera(iv, r2v, (W, H))
    ctx.set_seed(seed)
    return ctx, iv, r2v


def _trace(ctx, W, H, iters):
    ctx.init()
    ctx.set_resolution(W, H)
    ctx.set_iterations(iters)
    return ctx.trace_paths(0, W * H * iters)


@pytest.mark.gpu
@pytest.mark.parametrize("name,dims", [("bucky", None), ("manix", (64, 58, 64)), ("hetvol", None),
                                       ("cloud", CLOUD_SMALL)])
@pytest.mark.parametrize("kernel", ["naiveSK", "regenerationSK", "naiveMK"])
@pytest.mark.parametrize("bounds,cells", [(None, 1), (0, 1), (2, 1), (None, 0)])
def test_sparse_upload_per_path_equals_dense(cvr, oracle_mod, name, dims, kernel, bounds, cells):
    s = cvr.Scene.synthetic(name, 0, dims)
    W = H = 48
    iters = 2
    sp, iv, r2v = _ctx(cvr, W, H, kernel, 5, bounds, cells)
    sp.set_medium_sparse(s.sparse_medium)
    g = _trace(sp, W, H, iters)
    if s.is_sparse:
        D, A = densify(s)
        orc = oracle_mod.Oracle(D, A, scale=100.0, max_density=s.max_density)
    else:
        orc = oracle_mod.Oracle.from_medium_desc(s.medium, s.density, s.albedo)
    c = orc.trace_paths(orc.launch(iv, r2v, (W, H), (W, H), (0, 0), cvr.KERNELS.index(kernel), 5), 0,
                        W * H * iters)
    for f in ("image_id", "flags", "n_segments", "n_steps", "n_density", "n_albedo"):
        assert (g[f] == c[f]).all(), f
    assert (g["T"].view(np.uint32) == c["T"].view(np.uint32)).all()
    assert c["n_density"].sum() > 0


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", ["naiveSK", "regenerationSK", "streamingSK", "sortingSK", "streamingMK",
                                    "naiveMK"])
def test_sparse_render_image_equals_dense_render(cvr, kernel):
    """Every scheduler (the wave pool's sparse instance for regenerationSK)
    renders a sparse cloud exactly as the dense upload of the same grid."""
    s = cvr.Scene.synthetic("cloud", 0, CLOUD_SMALL)
    D, A = densify(s)
    W, H, iters = 96, 64, 3
    sp, _, _ = _ctx(cvr, W, H, kernel)
    sp.set_medium_sparse(s.sparse_medium)
    sp.init()
    img, st = sp.render_image(W, H, (2, 2), iters)
    dn, _, _ = _ctx(cvr, W, H, kernel)
    desc, keep = cvr.medium_from_arrays(D, A, max_density=s.max_density)
    dn.set_medium(desc)
    dn.init()
    ref, rst = dn.render_image(W, H, (2, 2), iters)
    for k in ("paths", "segments", "steps", "density", "albedo", "escaped"):
        assert getattr(st, k) == getattr(rst, k), k
    ng, nr = np.isnan(img), np.isnan(ref)
    assert (ng == nr).all()
    img, ref = np.where(ng, 0, img), np.where(nr, 0, ref)
    bound = 2.0 * iters * 2.0 ** -24 * np.maximum(np.abs(img), np.abs(ref)) + 1e-30
    assert (np.abs(img - ref) <= bound).all()
    assert st.albedo > 0 and st.fetches < st.density


@pytest.mark.gpu
def test_c5_cloud_4096_full_size(cvr, oracle_mod):
    """BASELINE config C5 at full size on one GPU: the 2048x1024x2048 sparse
    cloud proxy (~10 % active), 4096^2, 20 iterations, regenerationSK.
    Size-independent checks: two path-id shards sum to the whole render with
    identical counters, and sampled path ranges are bit-exact against the
    oracle reading the same leaves."""
    s = cvr.Scene.synthetic("cloud")
    assert s.dims == (2048, 1024, 2048)
    W = H = 4096
    iters = 20
    n = W * H * iters
    ctx, iv, r2v = _ctx(cvr, W, H, "regenerationSK")
    ctx.set_medium_sparse(s.sparse_medium)
    ctx.init()
    ctx.set_resolution(W, H)
    ctx.set_iterations(iters)
    ctx.clear_output()
    ctx.launch_render()
    full = ctx.copy_output(W, H)
    st = ctx.stats()
    assert st.paths == n and st.truncated == 0 and st.albedo > 0
    parts = np.zeros_like(full)
    steps = 0
    for first, count in ((0, n // 2), (n // 2, n - n // 2)):
        ctx.set_path_range(first, count)
        ctx.clear_output()
        ctx.launch_render()
        parts += ctx.copy_output(W, H)
        steps += ctx.stats().steps
    assert steps == st.steps
    full, parts = full[..., :3], parts[..., :3]  # w is a plain store of 1 per render
    ok = ~np.isnan(full)
    assert (np.isnan(parts) == ~ok).all()
    bound = 2.0 * iters * 2.0 ** -24 * np.maximum(np.abs(full), np.abs(parts)) + 1e-30
    assert (np.abs(full - parts)[ok] <= bound[ok]).all()
    orc = sparse_oracle(oracle_mod, s)
    L = orc.launch(iv, r2v, (W, H), (W, H), (0, 0), 2, 0)
    ctx.set_path_range(0, n)
    for first in (0, W * (H // 2) + W // 2 - 1024, n // 2 + 7777, n - 4096):
        g = ctx.trace_paths(first, 4096)
        c = orc.trace_paths(L, first, 4096)
        for f in ("image_id", "flags", "n_segments", "n_steps", "n_density", "n_albedo"):
            assert (g[f] == c[f]).all(), (first, f)
        assert (g["T"].view(np.uint32) == c["T"].view(np.uint32)).all(), first


def _read_hdr(path):
    """Flat RGBE scanlines as cvr_write_hdr writes them -> (H, W, 3) float."""
    data = open(path, "rb").read()
    head, _, rest = data.partition(b"\n\n")
    dims, _, px = rest.partition(b"\n")
    _, h, _, w = dims.split()
    e = np.frombuffer(px, np.uint8).reshape(int(h), int(w), 4).astype(np.float64)
    scale = np.where(e[..., 3] > 0, np.ldexp(1.0, (e[..., 3] - 136).astype(int)), 0.0)
    return e[..., :3] * scale[..., None]


@pytest.mark.gpu
def test_cli_sparse_upload_matches_dense(tmp_path):
    """--use-unified-memory 1 (the reference's choice for scenes that do not
    fit) uploads the grid as leaves; the image matches the dense upload.  A
    sparse-only scene (the C5 cloud proxy) renders through the CLI."""
    import subprocess
    cli = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cudavolumerenderer_amd", "cvr")
    imgs = []
    for unified in ("0", "1"):
        out = str(tmp_path / f"m{unified}")
        r = subprocess.run([cli, "--synthetic", "manix", "-r", "96", "96", "-i", "4", "--interactive", "0",
                            "--use-unified-memory", unified, "-o", out], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        imgs.append(_read_hdr(out + ".hdr"))
    assert imgs[0].max() > 0
    # RGBE keeps 8 mantissa bits of the pixel's largest channel: compare to that
    tol = np.maximum(imgs[0].max(-1), imgs[1].max(-1))[..., None] / 64 + 1e-6
    assert (np.abs(imgs[0] - imgs[1]) <= tol).all()
    out = str(tmp_path / "cloud")
    r = subprocess.run([cli, "--synthetic", "cloud", "-r", "64", "64", "-i", "1", "--interactive", "0", "-o", out],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert _read_hdr(out + ".hdr").max() > 0
