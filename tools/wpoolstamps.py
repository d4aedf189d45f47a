#!/usr/bin/env python3
"""Phase split of the wave-pool scheduler (CVR_STAMPS build): wave cycles in
EVENT batches vs TRACK iterations, lane utilisation of the TRACK loop."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import cudavolumerenderer_amd._lib as Lb  # noqa: E402

Lb.LIB_PATH = os.path.join(ROOT, "build", "stamps", "libcvr.so")
import cudavolumerenderer_amd as cvr  # noqa: E402

lib = cvr.load()
lib.cvr_debug_counters.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
scene = cvr.Scene.synthetic("manix")
W = H = 1024
iv, r2v = cvr.default_camera(W, H)
for batch in [8]:
    c = cvr.Context(0, "regenerationSK")
    c.set_option(cvr.OPT_SCHEDULER, 3)
    c.set_option(cvr.OPT_BATCH, batch)
    c.set_medium(scene.medium)
    c.set_camera(iv, r2v, (W, H))
    c.set_resolution(W, H)
    c.set_iterations(20)
    c.launch_render()
    st = c.stats()
    out = (C.c_uint64 * 16)()
    lib.cvr_debug_counters(c._h, out)
    ev, tr, n_ev, n_tr, ev_code, ev_to_regen_end, c_load, c_bnd, c_col, c_regen = list(out)[:10]
    b_only, c_only, mixed, lanes_b, lanes_c, lanes_n = list(out)[10:16]
    tot = ev + tr
    print(f"batch {batch}: kernel {st.kernel_ms:.2f} ms; event share {ev / tot:.3f}; event batches {n_ev} "
          f"({ev / max(n_ev, 1):.0f} cyc each, {(st.segments + st.paths) / max(n_ev, 1):.1f} items each); "
          f"track iterations {n_tr} ({tr / max(n_tr, 1):.0f} cyc each, {st.steps / max(n_tr, 1):.1f} lane-steps each); "
          f"per batch: load+event+roulette {ev_code / max(n_ev, 1):.0f}, regen+AABB+store "
          f"{(ev_to_regen_end - ev_code) / max(n_ev, 1):.0f}, lists {(ev - ev_to_regen_end) / max(n_ev, 1):.0f} cyc; "
          f"load {c_load / max(n_ev, 1):.0f} boundary {c_bnd / max(n_ev, 1):.0f} collision {c_col / max(n_ev, 1):.0f} "
          f"regen {c_regen / max(n_ev, 1):.0f} AABB+store {(ev_to_regen_end - c_load - c_bnd - c_col - c_regen) / max(n_ev, 1):.0f}",
          flush=True)
    nb = max(n_ev, 1)
    print(f"batches: boundary-only {b_only / nb:.3f}, collision-only {c_only / nb:.3f}, mixed {mixed / nb:.3f}, "
          f"neither {(n_ev - b_only - c_only - mixed) / nb:.3f}; lanes per batch: boundary {lanes_b / nb:.1f} "
          f"collision {lanes_c / nb:.1f} new {lanes_n / nb:.1f}", flush=True)
