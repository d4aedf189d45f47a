"""Scene loaders: the OpenVDB reader on the
reference's own data file and on generated files, and the MHD loader against
a numpy restatement of the reference's MHD->VDB converter.
"""
import hashlib
import os
import struct
import zlib

import numpy as np
import pytest

from vdb_writer import write_vdb

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
BONSAI = os.path.join(GOLDEN, "bonsai_small.vdb")


# ------------------------------------------------------------ OpenVDB ----
def vdb_grid_metadata(path):
    """Per-grid metadata of a VDB file (name -> {key: raw bytes})."""
    b = open(path, "rb").read()
    p = [0]

    def rd(fmt):
        v = struct.unpack_from(fmt, b, p[0])
        p[0] += struct.calcsize(fmt)
        return v

    def rs():
        (n,) = rd("<I")
        s = b[p[0]:p[0] + n]
        p[0] += n
        return s.decode()

    rd("<qIIIB")
    p[0] += 36
    (n,) = rd("<i")
    assert n == 0
    (ng,) = rd("<i")
    out = {}
    for _ in range(ng):
        name, _typ, _par = rs(), rs(), rs()
        gp, _bp, ep = rd("<qqq")
        p[0] = gp + 4
        (nm,) = rd("<i")
        meta = {}
        for _ in range(nm):
            k, _t = rs(), rs()
            (sz,) = rd("<I")
            meta[k] = b[p[0]:p[0] + sz]
            p[0] += sz
        out[name] = meta
        p[0] = ep
    return out


def test_bonsai_vdb_matches_file_metadata(cvr):
    """data/vdb/bonsai_small.vdb (the reference's real file; OpenVDB 8.1, file
    v224, blosc-LZ4 + active-mask compression).  The reader's active set
    matches the file's own bookkeeping (file_bbox_*, file_voxel_count), and the
    converter invariants hold (mhd_to_vdb.py:53,62-64): density in [0, 1],
    albedo = (density, 0, 0)."""
    meta = vdb_grid_metadata(BONSAI)
    s = cvr.Scene.load(BONSAI)
    for g in ("density", "albedo"):
        lo = np.frombuffer(meta[g]["file_bbox_min"], np.int32)
        hi = np.frombuffer(meta[g]["file_bbox_max"], np.int32)
        assert tuple(hi - lo + 1) == s.dims == (91, 197, 256)
    d, a = s.density, s.albedo
    count = struct.unpack("<q", meta["density"]["file_voxel_count"])[0]
    assert int((d != 0).sum()) == count == 87684
    assert int((a[..., 0] != 0).sum()) == struct.unpack("<q", meta["albedo"]["file_voxel_count"])[0]
    assert d.min() == 0.0 and d.max() == 1.0
    assert np.array_equal(a[..., 0], d) and not a[..., 1:3].any() and (a[..., 3] == 1).all()
    m = s.medium
    assert (m.scale, m.max_density) == (100.0, 1.0)  # VDBSceneBuilder.h:54-77
    assert tuple(m.box_min) == (-0.5,) * 3 and tuple(m.box_max) == (0.5,) * 3
    # frozen: any change in the decoded voxels shows up here
    h = hashlib.sha256(np.ascontiguousarray(d).tobytes()).hexdigest()
    assert h == BONSAI_DENSITY_SHA256, h


BONSAI_DENSITY_SHA256 = "106d542b2fcc4aad30732ccb5058e2e20368aa0b39e98e86fcc2754ceaf16ab1"


def _sparse_scene(rng, tiles=True):
    leaves = []
    for o in [(0, 0, 0), (8, 0, 0), (16, 8, 24), (120, 64, 8), (136, 0, 0)]:
        m = rng.uniform(size=512) < 0.4
        v = np.where(m, rng.uniform(0.05, 1.0, 512), 0.0).astype(np.float32)
        leaves.append((o, m, v))
    nodes = {"leaves": leaves, "tiles16": [((32, 16, 0), 0.5)] if tiles else [], "tiles32": []}
    return nodes


def _expected_dense(nodes):
    pts = []
    for (o, m, v) in nodes["leaves"]:
        for i in np.nonzero(m)[0]:
            pts.append(((o[0] + (i >> 6), o[1] + ((i >> 3) & 7), o[2] + (i & 7)), 1, v[i]))
    for (o, val) in nodes["tiles16"]:
        pts.append((o, 8, val))
    lo = np.min([p[0] for p in pts], axis=0)
    hi = np.max([np.asarray(p[0]) + p[1] - 1 for p in pts], axis=0)
    dim = hi - lo + 1
    dense = np.zeros((dim[2], dim[1], dim[0]), np.float32)
    for (c, _ext, val) in pts:  # a tile fills only its origin voxel (ValueOn iterator)
        dense[c[2] - lo[2], c[1] - lo[1], c[0] - lo[0]] = val
    return dense


@pytest.mark.parametrize("mode", ["raw", "zip", "mask1", "blosc_memcpy"])
def test_vdb_reader_on_generated_files(cvr, tmp_path, mode):
    rng = np.random.default_rng(7)
    nodes = _sparse_scene(rng)
    nodes3 = {"leaves": [(o, m, np.stack([v, v * 0.5, v * 0.25], -1)) for (o, m, v) in nodes["leaves"]],
              "tiles16": [(o, (val, val * 0.5, val * 0.25)) for (o, val) in nodes["tiles16"]], "tiles32": []}
    p = tmp_path / f"gen_{mode}.vdb"
    write_vdb(str(p), {"density": (nodes, 1), "albedo": (nodes3, 3)}, mode)
    s = cvr.Scene.load(str(p))
    want = _expected_dense(nodes)
    assert s.dims == (want.shape[2], want.shape[1], want.shape[0])
    assert np.array_equal(s.density, want)
    a = s.albedo
    assert np.array_equal(a[..., 0], want) and np.array_equal(a[..., 1], want * np.float32(0.5))
    assert s.medium.max_density == want.max()


def test_vdb_reader_errors(cvr, tmp_path):
    p = tmp_path / "bad.vdb"
    p.write_bytes(b"not a vdb file at all")
    with pytest.raises(cvr.CvrError) as e:
        cvr.Scene.load(str(p))
    assert "VDB" in str(e.value)
    rng = np.random.default_rng(1)
    q = tmp_path / "noalbedo.vdb"
    write_vdb(str(q), {"density": (_sparse_scene(rng), 1)}, "raw")
    with pytest.raises(cvr.CvrError) as e:  # VDBAdapter.cpp:32-37 requires an albedo grid (Q17)
        cvr.Scene.load(str(q))
    assert "albedo" in str(e.value)


# ---------------------------------------------------------------- MHD ----
def converter_restated(img_zyx):
    """scripts/convert-mhd/mhd_to_vdb.py:39-71 in numpy float32, followed by
    the VDB reader's densification over the active bounding box."""
    image = img_zyx.astype(np.float32)
    mn, mx = image.min(), image.max()
    normalized = (image - mn) / (mx - mn)
    t = np.clip((normalized - 0.2) / (0.6 - 0.2), 0.0, 1.0)
    dens = t * t * (3.0 - 2.0 * t)
    assert dens.dtype == np.float32
    vdb = dens  # copyFromArray: array[i][j][k] -> VDB (x=i, y=j, z=k)
    nz = np.argwhere(vdb != 0)
    lo, hi = nz.min(0), nz.max(0)
    crop = vdb[lo[0]:hi[0] + 1, lo[1]:hi[1] + 1, lo[2]:hi[2] + 1]  # indexed (x, y, z)
    return np.ascontiguousarray(crop.transpose(2, 1, 0))  # -> (z, y, x) view of an x-fastest array


def _write_mhd(path, img_zyx, etype, compressed, local=False, msb=False):
    dt = {"MET_SHORT": "<i2", "MET_UCHAR": "u1", "MET_FLOAT": "<f4", "MET_USHORT": "<u2"}[etype]
    if msb:
        dt = dt.replace("<", ">")
    raw = img_zyx.astype(dt).tobytes()
    if compressed:
        raw = zlib.compress(raw)
    nz, ny, nx = img_zyx.shape
    head = (f"ObjectType = Image\nNDims = 3\nBinaryData = True\nBinaryDataByteOrderMSB = {msb}\n"
            f"CompressedData = {compressed}\nDimSize = {nx} {ny} {nz}\nElementType = {etype}\n")
    if local:
        open(path, "wb").write((head + "ElementDataFile = LOCAL\n").encode() + raw)
    else:
        open(path, "w").write(head + f"ElementDataFile = {os.path.basename(path)}.raw\n")
        open(str(path) + ".raw", "wb").write(raw)


@pytest.mark.parametrize("etype,compressed,local,msb", [("MET_SHORT", True, False, False),
                                                        ("MET_UCHAR", False, True, False),
                                                        ("MET_USHORT", True, True, True),
                                                        ("MET_FLOAT", False, False, False)])
def test_mhd_loader_matches_converter(cvr, tmp_path, etype, compressed, local, msb):
    rng = np.random.default_rng(3)
    nz, ny, nx = 13, 17, 21
    z, y, x = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    r = np.sqrt(((x - 9) / 7.0) ** 2 + ((y - 8) / 6.0) ** 2 + ((z - 6) / 5.0) ** 2)
    img = np.clip(200 * (1.2 - r) + rng.normal(0, 10, r.shape), 0, 250)
    if etype in ("MET_SHORT", "MET_USHORT", "MET_UCHAR"):
        img = np.round(img)
    img = img.astype(np.float32)
    p = tmp_path / "vol.mhd"
    _write_mhd(str(p), img, etype, compressed, local, msb)
    s = cvr.Scene.load(str(p))
    want = converter_restated(img)
    assert s.dims == (want.shape[2], want.shape[1], want.shape[0])
    assert np.array_equal(s.density, want)
    assert np.array_equal(s.albedo[..., 0], want) and not s.albedo[..., 1:3].any()
    assert s.medium.scale == 100.0 and s.medium.max_density == want.max()


def test_reference_mhd_headers_parse_but_payloads_are_absent(cvr, tmp_path):
    """data/mhd/*.mhd are real headers whose .raw payloads are git-LFS
    pointers: the loader reports an I/O error instead of crashing."""
    hdr = ("ObjectType = Image\nNDims = 3\nBinaryData = True\nBinaryDataByteOrderMSB = False\n"
           "CompressedData = True\nCompressedDataSize = 6193601\nDimSize = 256 230 256\n"
           "ElementType = MET_SHORT\nElementDataFile = manix_small.raw\n")
    (tmp_path / "manix_small.mhd").write_text(hdr)
    (tmp_path / "manix_small.raw").write_text("version https://git-lfs.github.com/spec/v1\n")
    with pytest.raises(cvr.CvrError):
        cvr.Scene.load(str(tmp_path / "manix_small.mhd"))


# ---------------------------------------------------------- Mitsuba XML --
def _write_vol(path, data_zyxc, bbox):
    nz, ny, nx, ch = data_zyxc.shape
    head = b"VOL" + bytes([3]) + struct.pack("<iiiii", 1, nx, ny, nz, ch) + struct.pack("<6f", *bbox)
    open(path, "wb").write(head + data_zyxc.astype("<f4").tobytes())


def test_xml_scene_semantics(cvr, tmp_path):
    """XmlSceneBuilder.h:39-266: density/albedo gridvolumes named in the XML,
    scale from the XML, majorant max(min(1, v)) (Q15), AABB of the last file
    read, i.e. the albedo (Q15), camera fov from the perspective sensor."""
    rng = np.random.default_rng(5)
    nz, ny, nx = 6, 7, 9
    dens = rng.uniform(0, 1.6, (nz, ny, nx, 1)).astype(np.float32)
    alb = rng.uniform(0, 1, (nz, ny, nx, 3)).astype(np.float32)
    _write_vol(tmp_path / "d.vol", dens, (-1, -2, -3, 1, 2, 3))
    _write_vol(tmp_path / "a.vol", alb, (-0.5, -0.25, 0, 0.5, 0.75, 2))
    xml = open(os.path.join(GOLDEN, "hetvol.xml")).read()  # the reference's smoke scene, re-pointed
    xml = xml.replace("smoke.vol", "d.vol").replace("albedo.vol", "a.vol").replace('value="800"', 'value="123.5"')
    (tmp_path / "scene.xml").write_text(xml)
    s = cvr.Scene.load(str(tmp_path / "scene.xml"))
    assert s.dims == (nx, ny, nz)
    assert np.array_equal(s.density, dens[..., 0])
    assert np.array_equal(s.albedo[..., :3], alb) and (s.albedo[..., 3] == 1).all()
    m = s.medium
    assert m.scale == np.float32(123.5)
    assert m.max_density == 1.0  # capped (Q15) although the grid goes to 1.6
    assert tuple(m.box_min) == (-0.5, -0.25, 0.0) and tuple(m.box_max) == (0.5, 0.75, 2.0)
    iv, r2v = s.camera(400, 200)
    assert r2v[0] == pytest.approx(np.tan(0.33 * np.pi / 360), rel=1e-6)  # <float name="fov" value="0.33"/>
    assert r2v[1] == pytest.approx(np.tan(0.33 * 0.5 * np.pi / 360), rel=1e-6)
    assert list(iv) == list(cvr.default_camera(400, 200)[0])


def test_xml_scene_errors(cvr, tmp_path):
    # the reference's smoke scene: its .vol payloads are git-LFS pointers
    (tmp_path / "hetvol.xml").write_text(open(os.path.join(GOLDEN, "hetvol.xml")).read())
    (tmp_path / "smoke.vol").write_text("version https://git-lfs.github.com/spec/v1\n")
    with pytest.raises(cvr.CvrError) as e:
        cvr.Scene.load(str(tmp_path / "hetvol.xml"))
    assert "smoke.vol" in str(e.value)
    (tmp_path / "bad.xml").write_text("<scene><medium type='homogeneous'/></scene>")
    with pytest.raises(cvr.CvrError) as e:
        cvr.Scene.load(str(tmp_path / "bad.xml"))
    assert "gridvolume" in str(e.value)


# ------------------------------------------------------ sparse VDB read ----
def _densify_leaves(s):
    table, dens, alb, bg = s.leaves()
    nx, ny, nz = s.dims
    lz, ly, lx = table.shape
    D = np.zeros((lz * 8, ly * 8, lx * 8), np.float32)
    A = np.empty((lz * 8, ly * 8, lx * 8, 4), np.float32)
    A[:] = np.asarray(bg, np.float32)
    for z, y, x in zip(*np.nonzero(table != 0xFFFFFFFF)):
        k = table[z, y, x]
        D[z * 8:z * 8 + 8, y * 8:y * 8 + 8, x * 8:x * 8 + 8] = dens[k]
        if alb is not None:
            A[z * 8:z * 8 + 8, y * 8:y * 8 + 8, x * 8:x * 8 + 8] = alb[k]
    return D[:nz, :ny, :nx], A[:nz, :ny, :nx]


@pytest.mark.parametrize("which", ["bonsai", "generated"])
def test_vdb_sparse_read_equals_dense_read(cvr, tmp_path, which):
    """VdbSparse reads the active values straight into 8^3 leaves; densified,
    they are bit-identical to the dense read (density, albedo, majorant)."""
    path = BONSAI
    if which == "generated":
        rng = np.random.default_rng(3)
        nodes = _sparse_scene(rng)
        nodes3 = {"leaves": [(o, m, np.stack([v, v * 0.5, v * 0.25], -1)) for (o, m, v) in nodes["leaves"]],
                  "tiles16": [(o, (val, val * 0.5, val * 0.25)) for (o, val) in nodes["tiles16"]], "tiles32": []}
        path = str(tmp_path / "gen.vdb")
        write_vdb(path, {"density": (nodes, 1), "albedo": (nodes3, 3)}, "zip")
    dense = cvr.Scene.load(path, "Vdb")
    sparse = cvr.Scene.load(path, "VdbSparse")
    assert sparse.is_sparse and sparse.dims == dense.dims
    D, A = _densify_leaves(sparse)
    assert np.array_equal(D.view(np.uint32), dense.density.view(np.uint32))
    assert np.array_equal(A.view(np.uint32), dense.albedo.view(np.uint32))
    assert sparse.max_density == dense.max_density
    table, dens, _, _ = sparse.leaves()
    assert (dens.reshape(len(dens), -1) != 0).any(axis=1).all() or which == "generated"


def test_vdb_reader_goes_sparse_above_2pow30_voxels(cvr, tmp_path):
    """A VDB whose active box exceeds 2^30 voxels (20 GB of dense host arrays)
    is read into leaves by the plain Vdb/Auto types (C5-sized files)."""
    rng = np.random.default_rng(5)
    m = rng.uniform(size=512) < 0.5
    v = np.where(m, rng.uniform(0.1, 1.0, 512), 0.0).astype(np.float32)
    nodes = {"leaves": [((0, 0, 0), m, v), ((4088, 2040, 2040), m, v * 0.5)], "tiles16": [], "tiles32": []}
    nodes3 = {"leaves": [(o, mm, np.stack([vv, vv, vv], -1)) for (o, mm, vv) in nodes["leaves"]],
              "tiles16": [], "tiles32": []}
    p = str(tmp_path / "huge.vdb")
    write_vdb(p, {"density": (nodes, 1), "albedo": (nodes3, 3)}, "raw")
    s = cvr.Scene.load(p)
    assert s.is_sparse and s.dims == (4096, 2048, 2048)
    table, dens, alb, bg = s.leaves()
    assert table.shape == (256, 256, 512) and len(dens) == 2 and bg == (0.0, 0.0, 0.0, 1.0)
    vx = v.reshape(8, 8, 8)  # VDB leaf index (x << 6) | (y << 3) | z -> [x, y, z]
    assert np.array_equal(dens[table[0, 0, 0]], vx.transpose(2, 1, 0))
    assert np.array_equal(dens[table[255, 255, 511]], (vx * np.float32(0.5)).transpose(2, 1, 0))
    assert s.max_density == float(v.max())
