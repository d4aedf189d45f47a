#!/usr/bin/env python3
"""Ramp-down of one k_wpool launch, from the CVR_WPOOL_TAILSTAMP diagnostic build
(make variant NAME=tail DEFS=-DCVR_WPOOL_TAILSTAMP=1):
  CVR_LIB=build/variants/tail/libcvr.so python3 tools/tail_wpool.py [--scene manix] [--shard R N]
Per wave: start, first sight of every queue exhausted, end (s_memrealtime, 100 MHz).
Prints the launch span, when the waves saw the queues run dry, how long each then took
to drain its pool (paths live at that point, event batches after it), and how many
waves were still running over the last part of the launch."""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import cudavolumerenderer_amd as cvr  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scene", default="manix")
ap.add_argument("--res", type=int, default=1024)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--shard", type=int, nargs=2, default=None)
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
lib = cvr.load()
lib.cvr_debug_tailstamps.argtypes = [C.c_void_p, C.c_size_t]
scene = cvr.Scene.synthetic(a.scene)
W = H = a.res
iv, r2v = cvr.default_camera(W, H)
c = cvr.Context(0, "regenerationSK")
if scene.is_sparse:
    c.set_medium_sparse(scene.sparse_medium)
else:
    c.set_medium(scene.medium)
c.set_camera(iv, r2v, (W, H))
c.set_option(cvr.OPT_INFLIGHT, 1)
c.init()
c.set_resolution(W, H)
c.set_iterations(a.iters)
if a.shard:
    c.set_block_shard(*a.shard)
NW = 16384
for rep in range(a.reps):
    lib.cvr_debug_tailstamps_clear()
    c.clear_output()
    c.launch_render()
    st = c.stats()
    buf = (C.c_uint64 * (8 * NW))()
    assert lib.cvr_debug_tailstamps(buf, NW) == 0
    t = np.frombuffer(buf, dtype=np.uint64).reshape(NW, 8).astype(np.int64)
    t = t[t[:, 0] != 0]
    t0 = t[:, 0].min()
    us = lambda x: (x - t0) / 100.0  # noqa: E731  (100 MHz ticks -> us)
    start, ex, end = us(t[:, 0]), us(t[:, 1]), us(t[:, 2])
    live = t[:, 3] & 0xFFFF
    batches = (t[:, 3] >> 16) & 0xFFFFFF
    drain = end - ex
    ev_us = t[:, 4] / 100.0
    dsteps, dseg = t[:, 5], t[:, 6]
    span = end.max()
    q = lambda v: " / ".join(f"{np.percentile(v, p):.0f}" for p in (0, 10, 50, 90, 100))  # noqa: E731
    print(f"[rep {rep}] kernel {st.kernel_ms:.3f} ms (events), {len(t)} waves, span {span:.0f} us; "
          f"starts {q(start)} us")
    print(f"  queues dry seen at   (min/p10/p50/p90/max) {q(ex)} us")
    print(f"  wave ends            {q(end)} us")
    print(f"  drain per wave       {q(drain)} us; live paths at dry {q(live)}; batches after {q(batches)}")
    print(f"  event-batch time in drain {q(ev_us)} us (share of drain {ev_us.sum() / drain.sum():.3f}); "
          f"steps after dry {q(dsteps)}; segments after dry {q(dseg)}")
    last = np.argsort(end)[-20:]  # the 20 waves that end last
    print(f"  last 20 waves: drain {drain[last].mean():.0f} us, event share {ev_us[last].sum() / drain[last].sum():.3f}, "
          f"segments {dseg[last].mean():.0f}, steps {dsteps[last].mean():.0f}, batches {batches[last].mean():.0f}, "
          f"live at dry {live[last].mean():.0f}")
    for f in (0.5, 0.75, 0.9, 0.95, 0.98):
        tt = span * f
        print(f"  waves still running at {f:.2f} of span ({tt:.0f} us): {(end > tt).sum()}")
    # busy fraction of the wave slots over the launch: sum(end - start) / (waves * span)
    print(f"  wave-slot occupancy over the span {(end - start).sum() / (len(t) * span):.3f}; "
          f"lost after first dry {((span - end).clip(0)).sum() / (len(t) * span):.3f}")
c.close()
