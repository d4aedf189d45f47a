#!/usr/bin/env python3
"""Phase split of the pool scheduler (CVR_STAMPS build): wave cycles in EVENT,
TRACK and the barriers after each; lane utilisation of the TRACK loop."""
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
for opts in [dict(), dict(ev=32), dict(tail=48)]:
    c = cvr.Context(0, "regenerationSK")
    c.set_option(cvr.OPT_SCHEDULER, 2)
    if "ev" in opts:
        c.set_option(cvr.OPT_EVENT_THRESHOLD, opts["ev"])
    if "tail" in opts:
        c.set_option(cvr.OPT_TAIL, opts["tail"])
    c.set_medium(scene.medium)
    c.set_camera(iv, r2v, (W, H))
    c.set_resolution(W, H)
    c.set_iterations(20)
    c.launch_render()
    st = c.stats()
    out = (C.c_uint64 * 16)()
    lib.cvr_debug_counters(c._h, out)
    ev, bev, tr, btr, n_it, n_rounds = list(out)[:6]
    tot = ev + bev + tr + btr
    print(f"{opts}: kernel {st.kernel_ms:.2f} ms; share event {ev / tot:.3f} barrier-after-event {bev / tot:.3f} "
          f"track {tr / tot:.3f} barrier-after-track {btr / tot:.3f}; track iterations {n_it} "
          f"({tr / max(n_it, 1):.0f} cyc each, {st.steps / max(n_it, 1):.1f} lane-steps each); "
          f"event rounds {n_rounds} ({ev / max(n_rounds, 1):.0f} cyc each)", flush=True)
