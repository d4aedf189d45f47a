"""ctypes loader of the CPU oracle (liboracle.so, built from cvr_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py.  The product (cudavolumerenderer_amd) never
imports this module.  Parity status: see the header of cvr_oracle.c.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")

PATH_DTYPE = np.dtype([("image_id", "<u4"), ("flags", "<u4"), ("T", "<f4", (3,)),
                       ("n_segments", "<u4"), ("n_steps", "<u4"), ("n_density", "<u4"),
                       ("n_albedo", "<u4")])


class OracleMedium(C.Structure):
    _fields_ = [("res", C.c_uint32 * 3), ("density", C.POINTER(C.c_float)),
                ("albedo", C.POINTER(C.c_float)), ("box_min", C.c_float * 3),
                ("box_max", C.c_float * 3), ("scale", C.c_float), ("max_density", C.c_float),
                ("g", C.c_float), ("roughness", C.c_float * 2), ("eta", C.c_float),
                ("leaves", C.POINTER(C.c_uint32)), ("leaf_dims", C.c_uint32 * 3),
                ("leaf_density", C.POINTER(C.c_float)), ("leaf_albedo", C.POINTER(C.c_float)),
                ("albedo_bg", C.c_float * 4)]


class OracleLaunch(C.Structure):
    _fields_ = [("inv_view", C.c_float * 12), ("raster_to_view", C.c_float * 2),
                ("full_res", C.c_float * 2), ("tile_res", C.c_float * 2),
                ("offset", C.c_uint32 * 2), ("kernel", C.c_int32), ("seed_base", C.c_uint32),
                ("max_segments", C.c_uint32), ("world_to_aabb", C.c_int32)]


class OracleStats(C.Structure):
    _fields_ = [("segments", C.c_uint64), ("steps", C.c_uint64), ("density", C.c_uint64),
                ("albedo", C.c_uint64), ("escaped", C.c_uint64), ("paths", C.c_uint64),
                ("truncated", C.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        build()
    lib = C.CDLL(LIB_PATH)
    P = C.c_void_p
    lib.oracle_trace_paths.argtypes = [C.POINTER(OracleMedium), C.POINTER(OracleLaunch), C.c_uint32,
                                       C.c_uint32, P]
    lib.oracle_render.argtypes = [C.POINTER(OracleMedium), C.POINTER(OracleLaunch), C.c_uint64,
                                  C.c_uint64, C.c_uint64, C.POINTER(C.c_float), C.c_int,
                                  C.POINTER(OracleStats)]
    lib.oracle_render.restype = C.c_int
    lib.oracle_render_thread_bound.argtypes = [C.POINTER(OracleMedium), C.POINTER(OracleLaunch), C.c_uint32,
                                               C.c_uint32, C.c_uint32, C.POINTER(C.c_float), C.POINTER(OracleStats)]
    lib.oracle_render_thread_bound.restype = C.c_int
    lib.oracle_render_stream_thread_bound.argtypes = [C.POINTER(OracleMedium), C.POINTER(OracleLaunch), C.c_uint32,
                                                      C.c_uint32, C.c_uint32, C.c_int, C.POINTER(C.c_float),
                                                      C.POINTER(OracleStats)]
    lib.oracle_render_stream_thread_bound.restype = C.c_int
    lib.oracle_render_smk_thread_bound.argtypes = [C.POINTER(OracleMedium), C.POINTER(OracleLaunch), C.c_uint32,
                                                   C.c_uint32, C.c_uint32, C.POINTER(C.c_float),
                                                   C.POINTER(OracleStats)]
    lib.oracle_render_smk_thread_bound.restype = C.c_int
    lib.oracle_render_mk_reference.argtypes = [C.POINTER(OracleMedium), C.POINTER(OracleLaunch), C.c_uint32,
                                               C.POINTER(C.c_float), C.POINTER(OracleStats), P]
    lib.oracle_render_mk_reference.restype = C.c_int
    lib.oracle_rng_stream.argtypes = [C.c_int32, C.c_uint32, P, P]
    lib.oracle_rng_state.argtypes = [C.c_int32, P]
    lib.oracle_rng_state_consts.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, P]
    lib.oracle_density.argtypes = [C.POINTER(OracleMedium), P]
    lib.oracle_density.restype = C.c_float
    lib.oracle_aabb.argtypes = [C.POINTER(OracleMedium), P, P, P]
    lib.oracle_aabb.restype = C.c_int
    lib.oracle_hg.argtypes = [P, C.c_float, C.c_float, C.c_float, P]
    lib.oracle_fresnel.argtypes = [C.c_float, C.c_float, C.POINTER(C.c_float)]
    lib.oracle_fresnel.restype = C.c_float
    lib.oracle_camera_ray.argtypes = [C.POINTER(OracleLaunch), C.c_uint32, P]
    lib.oracle_detmath.argtypes = [C.c_int, P, P, C.c_uint32, P]
    _lib = lib
    return lib


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


class Oracle:
    """Scene + launch description for the oracle; arrays are kept alive here."""

    def __init__(self, density, albedo, box_min=(-0.5,) * 3, box_max=(0.5,) * 3, scale=100.0,
                 max_density=None, g=0.0, roughness=(0.1, 0.1), eta=None):
        self.lib = load()
        # own copies: a Scene's arrays are views of memory the scene frees
        self.density = np.array(density, np.float32, order="C", copy=True)
        self.albedo = np.array(albedo, np.float32, order="C", copy=True)
        nz, ny, nx = self.density.shape
        m = OracleMedium()
        m.res[:] = (nx, ny, nz)
        m.density = self.density.ctypes.data_as(C.POINTER(C.c_float))
        m.albedo = self.albedo.ctypes.data_as(C.POINTER(C.c_float))
        m.box_min[:] = box_min
        m.box_max[:] = box_max
        m.scale = scale
        m.max_density = float(self.density.max()) if max_density is None else max_density
        m.g = g
        m.roughness[:] = roughness
        m.eta = np.float32(np.float32(1.05) / np.float32(1.01)) if eta is None else eta
        self.m = m

    @classmethod
    def from_leaves(cls, res, table, leaf_density, leaf_albedo, albedo_bg, box_min=(-0.5,) * 3,
                    box_max=(0.5,) * 3, scale=100.0, max_density=1.0, g=0.0, roughness=(0.1, 0.1), eta=None):
        """The same walk over 8^3-leaf storage (cvr_sparse_medium_desc layout):
        `table` (lz, ly, lx) u32 slots or 0xFFFFFFFF, `leaf_density` (n, 512),
        `leaf_albedo` (n, 512, 4) or None (albedo_bg everywhere)."""
        nx, ny, nz = (int(v) for v in res)
        o = cls(np.zeros((1, 1, 1), np.float32), np.zeros((1, 1, 1, 4), np.float32), box_min, box_max, scale,
                max_density, g, roughness, eta)
        o.table = np.array(table, np.uint32, order="C", copy=True)
        o.leaf_density = np.array(leaf_density, np.float32, order="C", copy=True)
        o.leaf_albedo = None if leaf_albedo is None else np.array(leaf_albedo, np.float32, order="C", copy=True)
        m = o.m
        m.res[:] = (nx, ny, nz)
        m.leaves = o.table.ctypes.data_as(C.POINTER(C.c_uint32))
        lz, ly, lx = o.table.shape
        m.leaf_dims[:] = (lx, ly, lz)
        m.leaf_density = o.leaf_density.ctypes.data_as(C.POINTER(C.c_float))
        if o.leaf_albedo is not None:
            m.leaf_albedo = o.leaf_albedo.ctypes.data_as(C.POINTER(C.c_float))
        m.albedo_bg[:] = tuple(albedo_bg)
        return o

    @classmethod
    def from_medium_desc(cls, desc, density, albedo):
        return cls(density, albedo, tuple(desc.box_min), tuple(desc.box_max), desc.scale,
                   desc.max_density, desc.g, tuple(desc.roughness), desc.eta)

    @staticmethod
    def launch(inv_view, r2v, full_res, tile_res, offset=(0, 0), kernel=0, seed_base=0,
               max_segments=1 << 20, world_to_aabb=0) -> OracleLaunch:
        """world_to_aabb: quirk Q4, 0 the reference's p - min/extent, 1 the fix
        (CVR_OPT_WORLD_TO_AABB)."""
        L = OracleLaunch()
        L.inv_view[:] = [float(v) for v in inv_view]
        L.raster_to_view[:] = [float(v) for v in r2v]
        L.full_res[:] = [float(v) for v in full_res]
        L.tile_res[:] = [float(v) for v in tile_res]
        L.offset[:] = offset
        L.kernel = kernel
        L.seed_base = seed_base
        L.max_segments = max_segments
        L.world_to_aabb = world_to_aabb
        return L

    def trace_paths(self, L: OracleLaunch, first: int, count: int) -> np.ndarray:
        out = np.zeros(count, PATH_DTYPE)
        self.lib.oracle_trace_paths(C.byref(self.m), C.byref(L), first, count, _p(out))
        return out

    def render(self, L: OracleLaunch, first: int, count: int, stride: int = 1, nthreads: int = 1,
               out: np.ndarray | None = None):
        w, h = int(L.tile_res[0]), int(L.tile_res[1])
        if out is None:
            out = np.zeros((h, w, 4), np.float32)
        st = OracleStats()
        rc = self.lib.oracle_render(C.byref(self.m), C.byref(L), first, stride, count,
                                    out.ctypes.data_as(C.POINTER(C.c_float)), nthreads, C.byref(st))
        assert rc == 0
        return out, st

    def render_thread_bound(self, L: OracleLaunch, n_threads: int, first: int, count: int):
        """regenerationSK with the RNG bound to the thread: n_threads
        lockstep threads, Rng(seed + tid) each (cvr_oracle.c
        oracle_render_thread_bound).  Returns (tile accumulator, stats)."""
        w, h = int(L.tile_res[0]), int(L.tile_res[1])
        out = np.zeros((h, w, 4), np.float32)
        st = OracleStats()
        rc = self.lib.oracle_render_thread_bound(C.byref(self.m), C.byref(L), n_threads, first, count,
                                                 out.ctypes.data_as(C.POINTER(C.c_float)), C.byref(st))
        assert rc == 0
        return out, st

    def render_stream_thread_bound(self, L: OracleLaunch, n_threads: int, first: int, count: int,
                                   sorting: bool = False):
        """streamingSK (sorting=False) / sortingSK with the RNG bound to the
        thread: one block of n_threads lockstep threads, Rng(seed +
        tid) each, Morton-sort compaction (cvr_oracle.c
        oracle_render_stream_thread_bound).  Returns (tile accumulator, stats)."""
        w, h = int(L.tile_res[0]), int(L.tile_res[1])
        out = np.zeros((h, w, 4), np.float32)
        st = OracleStats()
        rc = self.lib.oracle_render_stream_thread_bound(C.byref(self.m), C.byref(L), n_threads, first, count,
                                                        int(sorting), out.ctypes.data_as(C.POINTER(C.c_float)),
                                                        C.byref(st))
        assert rc == 0
        return out, st

    def render_smk_thread_bound(self, L: OracleLaunch, n_threads: int, first: int, count: int):
        """streamingMK with the RNG bound to the thread: one block of
        n_threads lockstep threads, a new path's RNG Rng(seed + path_id) becoming
        its thread's state, the states staying with the threads when compaction
        moves the paths (cvr_oracle.c oracle_render_smk_thread_bound).  Returns
        (tile accumulator, stats)."""
        w, h = int(L.tile_res[0]), int(L.tile_res[1])
        out = np.zeros((h, w, 4), np.float32)
        st = OracleStats()
        rc = self.lib.oracle_render_smk_thread_bound(C.byref(self.m), C.byref(L), n_threads, first, count,
                                                     out.ctypes.data_as(C.POINTER(C.c_float)), C.byref(st))
        assert rc == 0
        return out, st

    def render_mk_reference(self, L: OracleLaunch, iterations: int):
        """naiveMK with the reference's compaction count (quirk Q11 reproduced,
        cvr_oracle.c oracle_render_mk_reference).  Returns (tile accumulator,
        stats, None) or (partial accumulator, stats, (iteration, bounce)) when a
        bounce leaves no live path (the reference's count underflows)."""
        w, h = int(L.tile_res[0]), int(L.tile_res[1])
        out = np.zeros((h, w, 4), np.float32)
        st = OracleStats()
        err = np.zeros(2, np.uint32)
        rc = self.lib.oracle_render_mk_reference(C.byref(self.m), C.byref(L), iterations,
                                                 out.ctypes.data_as(C.POINTER(C.c_float)), C.byref(st), _p(err))
        assert rc in (0, -2)
        return out, st, (None if rc == 0 else (int(err[0]), int(err[1])))

    def density_at(self, p):
        p = np.asarray(p, np.float32)
        return self.lib.oracle_density(C.byref(self.m), _p(p))

    def aabb(self, o, d):
        o = np.asarray(o, np.float32)
        d = np.asarray(d, np.float32)
        out = np.zeros(5, np.float32)
        hit = self.lib.oracle_aabb(C.byref(self.m), _p(o), _p(d), _p(out))
        return bool(hit), out


def rng_stream(seed: int, n: int):
    lib = load()
    u = np.zeros(n, np.uint32)
    f = np.zeros(n, np.float32)
    lib.oracle_rng_stream(seed, n, _p(u), _p(f))
    return u, f


def rng_state(seed: int):
    lib = load()
    s = np.zeros(6, np.uint32)
    lib.oracle_rng_state(seed, _p(s))
    return s


def rng_state_consts(seed: int, x0: int, x1: int, m0: int, m1: int):
    """The oracle's seeding structure with other scramble constants (rng_init_consts)."""
    lib = load()
    s = np.zeros(6, np.uint32)
    lib.oracle_rng_state_consts(seed & 0xFFFFFFFFFFFFFFFF, x0, x1, m0, m1, _p(s))
    return s


def detmath(fn: int, x, y=None):
    lib = load()
    x = np.ascontiguousarray(x, np.float32)
    y = np.ascontiguousarray(y if y is not None else np.zeros_like(x), np.float32)
    out = np.zeros_like(x)
    lib.oracle_detmath(fn, _p(x), _p(y), x.size, _p(out))
    return out


def hg(v, g, e1, e2):
    lib = load()
    v = np.asarray(v, np.float32)
    out = np.zeros(3, np.float32)
    lib.oracle_hg(_p(v), g, e1, e2, _p(out))
    return out


def camera_ray(L: OracleLaunch, path_id: int):
    lib = load()
    out = np.zeros(6, np.float32)
    lib.oracle_camera_ray(C.byref(L), path_id, _p(out))
    return out[:3], out[3:]
