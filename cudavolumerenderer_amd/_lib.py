"""ctypes binding of libcvr.so (include/cvr.h).

This is the only way Python reaches the renderer: every call goes through the
C ABI that a C/C++/Go/Java host would bind.  There is no
Python or CPU fallback: if libcvr.so is missing or a HIP call fails, the call
raises.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_DEFAULT_LIB = os.path.abspath(os.path.join(_HERE, "libcvr.so"))
# CVR_LIB: an experiment build instead of the in-tree library (e.g. `make variant-pair`'s,
# for tests/test_wave_pair.py); unset, the in-tree libcvr.so
LIB_PATH = os.environ.get("CVR_LIB") or _DEFAULT_LIB

CVR_OK = 0
ERRORS = {-1: "CVR_ERR_INVALID", -2: "CVR_ERR_HIP", -3: "CVR_ERR_STATE", -4: "CVR_ERR_IO",
          -5: "CVR_ERR_UNSUPPORTED", -6: "CVR_ERR_NOMEM"}

# Config::Kernel order (Config.h:87-95)
KERNELS = ["naiveSK", "naiveMK", "regenerationSK", "streamingMK", "streamingSK", "sortingSK"]
NAIVE_SK, NAIVE_MK, REGENERATION_SK, STREAMING_MK, STREAMING_SK, SORTING_SK = range(6)
SCENE_TYPES = {"Auto": 0, "MitsubaXml": 1, "Vdb": 2, "Raw": 3, "Mhd": 4, "VdbSparse": 5}

OPT_MAX_SEGMENTS, OPT_CHUNK, OPT_EVENT_THRESHOLD, OPT_GRID, OPT_SCATTER_EPS = 1, 2, 3, 4, 5
OPT_SCHEDULER, OPT_POOL, OPT_TIMING, OPT_CELLS, OPT_WAVES, OPT_ORDER, OPT_QUEUES = 6, 7, 8, 9, 10, 11, 12
OPT_BOUNDS, OPT_TAIL, OPT_BATCH, OPT_RNG_BINDING, OPT_MORTON = 13, 14, 15, 16, 17
OPT_WORLD_TO_AABB, OPT_MK_COMPACTION, OPT_SUBQUEUES, OPT_DRAIN, OPT_INFLIGHT, OPT_FRAME_FLUSH = 18, 19, 20, 22, 23, 24
OPT_UNIFORM_ALBEDO, OPT_WAVE_PAIR, OPT_SAMPLE_ORDER, OPT_EMPTY_MASK, OPT_COUNT_WORDS = 25, 26, 27, 28, 29


class CvrError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


class MediumDesc(C.Structure):
    _fields_ = [("res", C.c_uint32 * 3), ("density", C.POINTER(C.c_float)),
                ("albedo", C.POINTER(C.c_float)), ("box_min", C.c_float * 3),
                ("box_max", C.c_float * 3), ("scale", C.c_float), ("max_density", C.c_float),
                ("g", C.c_float), ("roughness", C.c_float * 2), ("eta", C.c_float)]


NO_LEAF = 0xFFFFFFFF


class SparseMediumDesc(C.Structure):
    _fields_ = [("res", C.c_uint32 * 3), ("leaf_dims", C.c_uint32 * 3),
                ("leaf_table", C.POINTER(C.c_uint32)), ("n_leaves", C.c_uint32),
                ("leaf_density", C.POINTER(C.c_float)), ("leaf_albedo", C.POINTER(C.c_float)),
                ("albedo_background", C.c_float * 4), ("box_min", C.c_float * 3),
                ("box_max", C.c_float * 3), ("scale", C.c_float), ("max_density", C.c_float),
                ("g", C.c_float), ("roughness", C.c_float * 2), ("eta", C.c_float)]


class Stats(C.Structure):
    _fields_ = [("paths", C.c_uint64), ("segments", C.c_uint64), ("steps", C.c_uint64),
                ("density", C.c_uint64), ("albedo", C.c_uint64), ("escaped", C.c_uint64),
                ("truncated", C.c_uint64), ("kernel_ms", C.c_double), ("iterations", C.c_uint64),
                ("track_ms", C.c_double), ("events_ms", C.c_double), ("fetches", C.c_uint64),
                ("words", C.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class PathRecord(C.Structure):
    _fields_ = [("image_id", C.c_uint32), ("flags", C.c_uint32), ("T", C.c_float * 3),
                ("n_segments", C.c_uint32), ("n_steps", C.c_uint32), ("n_density", C.c_uint32),
                ("n_albedo", C.c_uint32)]


PATH_RECORD_DTYPE = np.dtype([("image_id", "<u4"), ("flags", "<u4"), ("T", "<f4", (3,)),
                              ("n_segments", "<u4"), ("n_steps", "<u4"), ("n_density", "<u4"),
                              ("n_albedo", "<u4")])
assert PATH_RECORD_DTYPE.itemsize == C.sizeof(PathRecord)


class LoadOptions(C.Structure):
    _fields_ = [("flags", C.c_uint32), ("default_albedo", C.c_float * 3)]


LOAD_DEFAULT_ALBEDO = 1


class RenderDesc(C.Structure):
    _fields_ = [("resolution", C.c_uint32 * 2), ("n_tiles", C.c_uint32 * 2), ("iterations", C.c_uint32)]


_lib = None


def load() -> C.CDLL:
    """Load libcvr.so (built by `make` / __graft_entry__.build()); raise if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise FileNotFoundError(f"{LIB_PATH} not built: run `make` (or __graft_entry__.build())")
    lib = C.CDLL(LIB_PATH)
    P, U32, U64, I32, I64, F = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int, C.c_int64, C.c_float
    FP = C.POINTER(C.c_float)
    sig = {
        "cvr_abi_version": (I32, []),
        "cvr_create": (I32, [I32, I32, C.POINTER(P)]),
        "cvr_destroy": (I32, [P]),
        "cvr_last_error": (C.c_char_p, [P]),
        "cvr_set_medium": (I32, [P, C.POINTER(MediumDesc)]),
        "cvr_set_medium_sparse": (I32, [P, C.POINTER(SparseMediumDesc)]),
        "cvr_scene_sparse_medium": (I32, [P, C.POINTER(SparseMediumDesc)]),
        "cvr_scene_is_sparse": (I32, [P]),
        "cvr_set_camera": (I32, [P, FP, FP, FP]),
        "cvr_set_resolution": (I32, [P, U32, U32]),
        "cvr_get_resolution": (I32, [P, C.POINTER(U32), C.POINTER(U32)]),
        "cvr_set_offset": (I32, [P, U32, U32]),
        "cvr_set_iterations": (I32, [P, U32]),
        "cvr_set_path_range": (I32, [P, U64, U64]),
        "cvr_set_block_shard": (I32, [P, U32, U32]),
        "cvr_set_block_order": (I32, [P, P, U32]),
        "cvr_share_medium": (I32, [P, P]),
        "cvr_trace_launch": (I32, [P, P, U64]),
        "cvr_image_to_host": (I32, [P, P, C.c_size_t, C.c_float, P]),
        "cvr_render_frame": (I32, [P, P, C.c_size_t, U32, C.POINTER(Stats)]),
        "cvr_frame_flush_info": (I32, [P, C.POINTER(U32), C.POINTER(U32)]),
        "cvr_blocks_to_host": (I32, [P, P, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_float, P]),
        "cvr_launch_blocks": (I32, [P, P, P, P]),
        "cvr_set_seed": (I32, [P, U32]),
        "cvr_get_seed": (I32, [P, C.POINTER(U32)]),
        "cvr_set_output": (I32, [P, P]),
        "cvr_output_ptr": (P, [P]),
        "cvr_set_stream": (I32, [P, P]),
        "cvr_own_stream": (P, [P]),
        "cvr_set_option": (I32, [P, I32, I64]),
        "cvr_init": (I32, [P]),
        "cvr_launch_render": (I32, [P]),
        "cvr_reset": (I32, [P]),
        "cvr_synchronize": (I32, [P]),
        "cvr_clear_output": (I32, [P]),
        "cvr_get_stats": (I32, [P, C.POINTER(Stats)]),
        "cvr_copy_output": (I32, [P, FP, F]),
        "cvr_trace_paths": (I32, [P, U32, U32, C.POINTER(PathRecord)]),
        "cvr_device_info": (I32, [P, C.POINTER(I32), C.POINTER(I32)]),
        "cvr_render_image": (I32, [P, C.POINTER(RenderDesc), P, FP, C.POINTER(Stats)]),
        "cvr_render_tiles": (I32, [P, C.POINTER(RenderDesc), U32, U32, P, FP, C.POINTER(Stats)]),
        "cvr_render_share_to_host": (I32, [P, C.POINTER(RenderDesc), U32, U32, P, C.c_size_t, C.POINTER(Stats)]),
        "cvr_host_alloc": (I32, [C.c_size_t, C.POINTER(C.c_void_p)]),
        "cvr_host_free": (I32, [P]),
        "cvr_default_camera": (I32, [U32, U32, FP, FP]),
        "cvr_tiling": (I32, [U32, U32, U32, U32, C.POINTER(U32)]),
        "cvr_tile_origin": (I32, [U32, U32, C.POINTER(U32), C.POINTER(U32)]),
        "cvr_scene_load": (I32, [C.c_char_p, I32, C.POINTER(P)]),
        "cvr_scene_load_ex": (I32, [C.c_char_p, I32, C.POINTER(LoadOptions), C.POINTER(P)]),
        "cvr_scene_synthetic": (I32, [C.c_char_p, U32, C.POINTER(U32), C.POINTER(P)]),
        "cvr_scene_medium": (I32, [P, C.POINTER(MediumDesc)]),
        "cvr_scene_camera": (I32, [P, U32, U32, P, P]),
        "cvr_scene_raw_bytes": (I32, [P, C.POINTER(C.POINTER(C.c_uint8)), C.POINTER(C.c_size_t)]),
        "cvr_scene_destroy": (None, [P]),
        "cvr_write_hdr": (I32, [C.c_char_p, FP, U32, U32]),
        "cvr_kernel_from_name": (I32, [C.c_char_p]),
        "cvr_kernel_name": (C.c_char_p, [I32]),
    }
    # an older experiment build (tools' --lib, A/B against a previous commit) may lack newer entry
    # points; the in-tree library must export every one (tests/test_host_abi.py)
    older_ok = os.path.abspath(LIB_PATH) != _DEFAULT_LIB
    for name, (res, args) in sig.items():
        if older_ok and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _fp(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _check(code: int, ctx=None):
    if code != CVR_OK:
        msg = load().cvr_last_error(ctx)
        raise CvrError(code, msg.decode() if msg else "")


# ------------------------------------------------------------------ helpers --
def default_camera(width: int, height: int):
    """Camera.h:25-71 + CudaVolPath.cpp:67-85 -> (inv_view[12], raster_to_view[2])."""
    lib = load()
    iv = np.zeros(12, np.float32)
    r2v = np.zeros(2, np.float32)
    _check(lib.cvr_default_camera(width, height, _fp(iv), _fp(r2v)))
    return iv, r2v


def tiling(width: int, height: int, ntx: int, nty: int):
    lib = load()
    td = (C.c_uint32 * 2)()
    _check(lib.cvr_tiling(width, height, ntx, nty, td))
    return int(td[0]), int(td[1])


def tile_origin(tile_id: int, ntx: int, tile_dim: Sequence[int]):
    lib = load()
    td = (C.c_uint32 * 2)(*tile_dim)
    org = (C.c_uint32 * 2)()
    _check(lib.cvr_tile_origin(tile_id, ntx, td, org))
    return int(org[0]), int(org[1])


def image_to_host(device_ptr: int, host_ptr: int, n_floats: int, scale: float, stream_ptr: Optional[int]):
    """host[i] = device[i] / scale, written by a kernel on `stream_ptr` into
    pinned or registered host memory (cvr_image_to_host; asynchronous)."""
    _check(load().cvr_image_to_host(C.c_void_p(device_ptr), C.c_void_p(host_ptr), n_floats, scale,
                                    C.c_void_p(stream_ptr) if stream_ptr else None))


def blocks_to_host(device_ptr: int, host_ptr: int, width: int, height: int, rank: int, world: int, scale: float,
                   stream_ptr: Optional[int]):
    """The pixels of block shard (rank, world) of a width x height float4
    image, divided by scale, stored by a kernel on `stream_ptr` at their places
    in the full pinned/registered host image (cvr_blocks_to_host; asynchronous)."""
    _check(load().cvr_blocks_to_host(C.c_void_p(device_ptr), C.c_void_p(host_ptr), width, height, rank, world,
                                     scale, C.c_void_p(stream_ptr) if stream_ptr else None))


def write_hdr(path: str, rgba: np.ndarray):
    rgba = np.ascontiguousarray(rgba, dtype=np.float32)
    h, w = rgba.shape[:2]
    _check(load().cvr_write_hdr(path.encode(), _fp(rgba), w, h))


# ------------------------------------------------------------------- scenes --
class Scene:
    """A loaded or synthetic scene (SceneBuilder + Scene, Scene.h:56-81)."""

    def __init__(self, handle):
        self._h = handle
        self.is_sparse = bool(load().cvr_scene_is_sparse(self._h))
        self._sparse = None
        self.medium = None
        if not self.is_sparse:
            self.medium = MediumDesc()
            _check(load().cvr_scene_medium(self._h, C.byref(self.medium)))

    @property
    def sparse_medium(self) -> SparseMediumDesc:
        """8^3-leaf view (cvr_scene_sparse_medium; built once for dense scenes)."""
        if self._sparse is None:
            d = SparseMediumDesc()
            _check(load().cvr_scene_sparse_medium(self._h, C.byref(d)))
            self._sparse = d
        return self._sparse

    @classmethod
    def synthetic(cls, name: str, seed: int = 0, dims: Optional[Sequence[int]] = None) -> "Scene":
        lib = load()
        h = C.c_void_p()
        d = (C.c_uint32 * 3)(*dims) if dims is not None else None
        _check(lib.cvr_scene_synthetic(name.encode(), seed, d, C.byref(h)))
        return cls(h)

    @classmethod
    def load(cls, path: str, scene_type: str = "Auto", default_albedo: Optional[Sequence[float]] = None) -> "Scene":
        """Load a scene file (cvr_scene_load_ex).  default_albedo (r, g, b): a VDB
        file without an albedo grid loads with that albedo everywhere (quirk
        Q17's flag; the reference refuses such files, VDBAdapter.cpp:32-37)."""
        lib = load()
        h = C.c_void_p()
        opts = None
        if default_albedo is not None:
            opts = LoadOptions()
            opts.flags = LOAD_DEFAULT_ALBEDO
            opts.default_albedo[:] = [float(v) for v in default_albedo]
        _check(lib.cvr_scene_load_ex(path.encode(), SCENE_TYPES[scene_type],
                                     C.byref(opts) if opts is not None else None, C.byref(h)))
        return cls(h)

    def camera(self, width: int, height: int):
        """(inv_view[12], raster_to_view[2]) of this scene's camera (cvr_scene_camera)."""
        iv = np.zeros(12, np.float32)
        r2v = np.zeros(2, np.float32)
        _check(load().cvr_scene_camera(self._h, width, height, _fp(iv), _fp(r2v)))
        return iv, r2v

    @property
    def dims(self):
        return tuple(int(v) for v in (self.sparse_medium if self.is_sparse else self.medium).res)

    def _dense_only(self):
        if self.is_sparse:
            raise CvrError(-5, "scene is stored sparse only (use leaves() / sparse_medium)")

    @property
    def max_density(self) -> float:
        return float((self.sparse_medium if self.is_sparse else self.medium).max_density)

    @property
    def has_albedo(self) -> bool:
        """Whether the medium stores albedo voxels (a sparse scene may use albedo_bg everywhere)."""
        return (not self.is_sparse) or bool(self.sparse_medium.leaf_albedo)

    def leaves(self):
        """(leaf_table (lz, ly, lx) u32, leaf_density (n, 8, 8, 8), leaf_albedo (n, 8, 8, 8, 4) or
        None, albedo_background) as numpy views owned by the scene."""
        d = self.sparse_medium
        lx, ly, lz = (int(v) for v in d.leaf_dims)
        table = np.ctypeslib.as_array(d.leaf_table, shape=(lz, ly, lx))
        n = int(d.n_leaves)
        dens = np.ctypeslib.as_array(d.leaf_density, shape=(n, 8, 8, 8)) if n else np.zeros((0, 8, 8, 8), np.float32)
        alb = np.ctypeslib.as_array(d.leaf_albedo, shape=(n, 8, 8, 8, 4)) if (n and d.leaf_albedo) else None
        return table, dens, alb, tuple(d.albedo_background)

    @property
    def density(self) -> np.ndarray:
        """(z, y, x) view of the fp32 density grid (owned by the scene)."""
        self._dense_only()
        nx, ny, nz = self.dims
        return np.ctypeslib.as_array(self.medium.density, shape=(nz, ny, nx))

    @property
    def albedo(self) -> np.ndarray:
        self._dense_only()
        nx, ny, nz = self.dims
        return np.ctypeslib.as_array(self.medium.albedo, shape=(nz, ny, nx, 4))

    @property
    def raw_bytes(self) -> bytes:
        p = C.POINTER(C.c_uint8)()
        n = C.c_size_t()
        _check(load().cvr_scene_raw_bytes(self._h, C.byref(p), C.byref(n)))
        return bytes(np.ctypeslib.as_array(p, shape=(n.value,))) if n.value else b""

    def close(self):
        if self._h:
            load().cvr_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def medium_from_arrays(density: np.ndarray, albedo: np.ndarray, box_min=(-0.5,) * 3, box_max=(0.5,) * 3,
                       scale=100.0, max_density=None, g=0.0, roughness=(0.1, 0.1), eta=None):
    """Build a MediumDesc over caller arrays (kept alive by the returned tuple)."""
    density = np.ascontiguousarray(density, dtype=np.float32)
    albedo = np.ascontiguousarray(albedo, dtype=np.float32)
    nz, ny, nx = density.shape
    assert albedo.shape == (nz, ny, nx, 4)
    m = MediumDesc()
    m.res[:] = (nx, ny, nz)
    m.density = _fp(density)
    m.albedo = _fp(albedo)
    m.box_min[:] = box_min
    m.box_max[:] = box_max
    m.scale = scale
    m.max_density = float(density.max()) if max_density is None else max_density
    m.g = g
    m.roughness[:] = roughness
    m.eta = np.float32(np.float32(1.05) / np.float32(1.01)) if eta is None else eta
    return m, (density, albedo)


# ------------------------------------------------------------------ context --
class Context:
    """One kernel launcher bound to one GPU (VolPTKernelLauncher, RenderKernelLauncher.h:54-73)."""

    def __init__(self, device: int = 0, kernel="regenerationSK"):
        lib = load()
        kid = KERNELS.index(kernel) if isinstance(kernel, str) else int(kernel)
        h = C.c_void_p()
        _check(lib.cvr_create(device, kid, C.byref(h)))
        self._h = h
        self.kernel = kid

    def _c(self, code):
        _check(code, self._h)

    def set_medium(self, medium: MediumDesc):
        self._c(load().cvr_set_medium(self._h, C.byref(medium)))

    def set_medium_sparse(self, desc: SparseMediumDesc):
        self._c(load().cvr_set_medium_sparse(self._h, C.byref(desc)))

    def set_camera(self, inv_view, raster_to_view, full_res):
        iv = np.ascontiguousarray(inv_view, np.float32)
        r = np.ascontiguousarray(raster_to_view, np.float32)
        fr = np.ascontiguousarray(full_res, np.float32)
        self._c(load().cvr_set_camera(self._h, _fp(iv), _fp(r), _fp(fr)))

    def set_resolution(self, w, h):
        self._c(load().cvr_set_resolution(self._h, w, h))

    @property
    def resolution(self):
        """The tile resolution the library renders now (cvr_get_resolution): render_image /
        render_tiles set it to their tile size too."""
        w, h = C.c_uint32(), C.c_uint32()
        self._c(load().cvr_get_resolution(self._h, C.byref(w), C.byref(h)))
        return w.value, h.value

    def set_offset(self, x, y):
        self._c(load().cvr_set_offset(self._h, x, y))

    def set_iterations(self, it):
        self._c(load().cvr_set_iterations(self._h, it))

    def set_path_range(self, first, count):
        self._c(load().cvr_set_path_range(self._h, first, count))

    def set_block_shard(self, rank, world):
        """Launch only shard `rank` of `world` (cvr_set_block_shard)."""
        self._c(load().cvr_set_block_shard(self._h, rank, world))

    def share_medium(self, src: "Context"):
        """Render `src`'s medium without a copy (cvr_share_medium); keep `src` alive."""
        self._c(load().cvr_share_medium(self._h, src._h))
        self._medium_src = src

    def set_block_order(self, perm: Optional[np.ndarray]):
        """Block work order of the launch (cvr_set_block_order); None = natural."""
        if perm is None:
            self._c(load().cvr_set_block_order(self._h, None, 0))
            return
        p = np.ascontiguousarray(perm, np.uint32)
        self._c(load().cvr_set_block_order(self._h, p.ctypes.data_as(C.c_void_p), len(p)))

    def launch_blocks(self):
        """(n_blocks, n_queues, qbeg) of the current launch's pixel-block work order."""
        nb, nq = C.c_uint32(), C.c_uint32()
        qb = (C.c_uint32 * 9)()
        self._c(load().cvr_launch_blocks(self._h, C.byref(nb), C.byref(nq), qb))
        return nb.value, nq.value, list(qb)[:nq.value + 1]

    def set_seed(self, seed):
        self._c(load().cvr_set_seed(self._h, seed))

    def get_seed(self) -> int:
        v = C.c_uint32()
        self._c(load().cvr_get_seed(self._h, C.byref(v)))
        return v.value

    def set_output(self, device_ptr: Optional[int]):
        self._c(load().cvr_set_output(self._h, C.c_void_p(device_ptr) if device_ptr else None))

    def output_ptr(self) -> int:
        return load().cvr_output_ptr(self._h) or 0

    def set_stream(self, stream_ptr: Optional[int]):
        """Launch on `stream_ptr` (a hipStream_t; 0/None = the null stream)."""
        self._c(load().cvr_set_stream(self._h, C.c_void_p(stream_ptr) if stream_ptr else None))

    def use_own_stream(self):
        self._c(load().cvr_set_stream(self._h, load().cvr_own_stream(self._h)))

    def set_option(self, opt: int, value: int):
        self._c(load().cvr_set_option(self._h, opt, value))

    def init(self):
        self._c(load().cvr_init(self._h))

    def launch_render(self):
        self._c(load().cvr_launch_render(self._h))

    def reset(self):
        self._c(load().cvr_reset(self._h))

    def synchronize(self):
        self._c(load().cvr_synchronize(self._h))

    def clear_output(self):
        self._c(load().cvr_clear_output(self._h))

    def stats(self) -> Stats:
        s = Stats()
        self._c(load().cvr_get_stats(self._h, C.byref(s)))
        return s

    def copy_output(self, w, h, scale=1.0) -> np.ndarray:
        out = np.zeros((h, w, 4), np.float32)
        self._c(load().cvr_copy_output(self._h, _fp(out), scale))
        return out

    def trace_paths(self, first: int, count: int) -> np.ndarray:
        out = np.zeros(count, PATH_RECORD_DTYPE)
        self._c(load().cvr_trace_paths(self._h, first, count,
                                       out.ctypes.data_as(C.POINTER(PathRecord))))
        return out

    def trace_launch(self, n: int) -> np.ndarray:
        """The production wave-pool launch of the current range (n path ids)
        with per-path final records (cvr_trace_launch)."""
        out = np.zeros(n, PATH_RECORD_DTYPE)
        self._c(load().cvr_trace_launch(self._h, out.ctypes.data_as(C.POINTER(PathRecord)), n))
        return out

    def device_info(self):
        cu, grid = C.c_int(), C.c_int()
        self._c(load().cvr_device_info(self._h, C.byref(cu), C.byref(grid)))
        return cu.value, grid.value

    def render_image(self, width, height, n_tiles=(1, 1), iterations=20, device_image: Optional[int] = None,
                     host: bool = True):
        return self.render_tiles(width, height, n_tiles, iterations, 0, 1, device_image, host)

    def render_frame(self, host_ptr=None, parts: int = 0, stats: bool = True,
                     host_floats: Optional[int] = None):
        """CudaVolPath::render for one tile (cvr_render_frame): clear, render
        the set resolution / iterations, and the normalised image in host
        memory when it returns, the launch split into `parts` bands whose
        copies overlap the later bands.  host_ptr: a PinnedImage, or the
        address of a float buffer (pinned for asynchronous copies) together
        with host_floats, the floats it holds (the library rejects a buffer
        shorter than the tile); None returns a new array.  stats=False skips
        the counters (one synchronous read per band)."""
        st = Stats() if stats else None
        img = None
        w, h = self.resolution  # the library's own tile size (what cvr_render_frame writes)
        if host_ptr is None:
            if w == 0 or h == 0:
                raise CvrError(-3, "render_frame: no resolution set")
            img = np.zeros((h, w, 4), np.float32)
            host_ptr = img.ctypes.data
            host_floats = img.size
        elif isinstance(host_ptr, PinnedImage):
            host_floats = host_ptr.floats if host_floats is None else host_floats
            host_ptr = host_ptr.ptr.value
        elif host_floats is None:
            # a bare address says nothing about its size: the caller states it, so the library's
            # size check (ABI 3) always runs
            raise CvrError(-1, "render_frame: host_floats is required with a raw host_ptr")
        self._c(load().cvr_render_frame(self._h, C.c_void_p(host_ptr), host_floats, parts,
                                        C.byref(st) if stats else None))
        return img, st

    def frame_flush_info(self):
        """(blocks the last render_frame's flusher waves stored in the launch, 0 if it
        copied after the launch; calls that fell back to the copy) (cvr_frame_flush_info)."""
        b, f = C.c_uint32(0), C.c_uint32(0)
        self._c(load().cvr_frame_flush_info(self._h, C.byref(b), C.byref(f)))
        return b.value, f.value

    def render_share_to_host(self, host_ptr: int, host_floats: int, width, height, n_tiles=(1, 1), iterations=20,
                             first_tile: int = 0, tile_stride: int = 1):
        """One device's share of a multi-device render (cvr_render_share_to_host):
        tiles first_tile, first_tile + tile_stride, ... (more than one tile), else
        this context's block shard, stored normalised into the full pinned host
        image at host_ptr (width*height*4 floats, e.g. a PinnedImage)."""
        d = RenderDesc()
        d.resolution[:] = (width, height)
        d.n_tiles[:] = n_tiles
        d.iterations = iterations
        st = Stats()
        self._c(load().cvr_render_share_to_host(self._h, C.byref(d), first_tile, tile_stride, C.c_void_p(host_ptr),
                                                host_floats, C.byref(st)))
        return st

    def render_tiles(self, width, height, n_tiles=(1, 1), iterations=20, first_tile: int = 0,
                     tile_stride: int = 1, device_image: Optional[int] = None, host: bool = True):
        """Tiles first_tile, first_tile + tile_stride, ... of render_image's
        tile loop, each with its sequential-loop seed (cvr_render_tiles)."""
        d = RenderDesc()
        d.resolution[:] = (width, height)
        d.n_tiles[:] = n_tiles
        d.iterations = iterations
        st = Stats()
        img = np.zeros((height, width, 4), np.float32) if host else None
        self._c(load().cvr_render_tiles(self._h, C.byref(d), first_tile, tile_stride,
                                        C.c_void_p(device_image) if device_image else None,
                                        _fp(img) if host else None, C.byref(st)))
        return img, st

    def close(self):
        if getattr(self, "_h", None):
            load().cvr_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class PinnedImage:
    """A width x height float4 image in pinned, device-mapped host memory
    (cvr_host_alloc), viewed as a numpy array; every device can store into it."""

    def __init__(self, width: int, height: int):
        self.ptr = C.c_void_p()
        rc = load().cvr_host_alloc(width * height * 16, C.byref(self.ptr))
        if rc != 0:
            raise CvrError(rc, load().cvr_last_error(None).decode())
        self.floats = width * height * 4
        self.array = np.ctypeslib.as_array(C.cast(self.ptr, C.POINTER(C.c_float)), shape=(height, width, 4))

    def close(self):
        if self.ptr:
            load().cvr_host_free(self.ptr)
            self.ptr = C.c_void_p()
            self.array = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 (interpreter shutdown: the library may be gone)
            pass
