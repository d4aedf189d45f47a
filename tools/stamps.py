#!/usr/bin/env python3
"""Phase split of the persistent kernel from the CVR_STAMPS diagnostic build
(build/stamps/libcvr.so): share of wave cycles in event phases vs Woodcock
tracking.  Shares only; the stamps themselves perturb timing."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import ctypes as C  # noqa: E402

import cudavolumerenderer_amd._lib as L  # noqa: E402

L.LIB_PATH = os.path.join(ROOT, "build", "stamps", "libcvr.so")
import cudavolumerenderer_amd as cvr  # noqa: E402

lib = cvr.load()
lib.cvr_debug_counters.argtypes = [C.c_void_p, C.POINTER(C.c_uint64)]
scene = cvr.Scene.synthetic(sys.argv[1] if len(sys.argv) > 1 else "manix")
W = H = 1024
iv, r2v = cvr.default_camera(W, H)
for ev in (56, 32, 16):
    c = cvr.Context(0, "regenerationSK")
    c.set_option(cvr.OPT_EVENT_THRESHOLD, ev)
    c.set_medium(scene.medium)
    c.set_camera(iv, r2v, (W, H))
    c.set_resolution(W, H)
    c.set_iterations(20)
    c.launch_render()
    st = c.stats()
    out = (C.c_uint64 * 16)()
    lib.cvr_debug_counters(c._h, out)
    ev_c, tr_c, n_ev, n_tr = out[0], out[1], out[2], out[3]
    tot = ev_c + tr_c
    print(f"ev={ev}: kernel {st.kernel_ms:.2f} ms; event phases {n_ev} ({ev_c / max(n_ev, 1):.0f} cyc each), "
          f"track iterations {n_tr} ({tr_c / max(n_tr, 1):.0f} cyc each); event share {ev_c / tot:.3f}, "
          f"lane-steps per track iteration {st.steps / max(n_tr, 1):.1f}")
