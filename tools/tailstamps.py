#!/usr/bin/env python3
"""Ramp-up / drain profile of one wave-pool launch (CVR_TAILSTAMPS build):

  make variant NAME=tail DEFS="-DCVR_TAILSTAMPS=1"
  python tools/tailstamps.py [--scene manix] [--shard 8]

Per wave: start, first track iteration, queue exhaustion and end
(s_memrealtime, 100 MHz), track iterations and event batches before and after
exhaustion, lane-steps after exhaustion.  Prints where the launch's time goes
between the first wave's start and the last wave's end.
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import cudavolumerenderer_amd._lib as Lb  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="manix")
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--shard", type=int, default=1)
    ap.add_argument("--lib", default=os.path.join(ROOT, "build", "variants", "tail", "libcvr.so"))
    ap.add_argument("--opt", action="append", default=[], help="OPT_NAME=value")
    a = ap.parse_args()
    Lb.LIB_PATH = os.path.abspath(a.lib)
    import cudavolumerenderer_amd as cvr

    lib = cvr.load()
    lib.cvr_debug_tailstamps.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_size_t]
    scene = cvr.Scene.synthetic(a.scene)
    W = H = a.res
    iv, r2v = cvr.default_camera(W, H)
    c = cvr.Context(0, "regenerationSK")
    if scene.is_sparse:
        c.set_medium_sparse(scene.sparse_medium)
    else:
        c.set_medium(scene.medium)
    c.set_camera(iv, r2v, (W, H))
    for kv in a.opt:
        k, v = kv.split("=")
        c.set_option(getattr(cvr, k), int(v))
    c.set_resolution(W, H)
    c.set_iterations(a.iters)
    c.set_block_shard(0, a.shard)
    cu, _ = c.device_info()
    for rep in range(3):
        c.clear_output()
        c.launch_render()
        st = c.stats()
    nw = cu * 4 * 5  # the wave-pool grid (one wave per workgroup, 5 per SIMD)
    buf = (C.c_uint64 * (nw * 10))()
    lib.cvr_debug_tailstamps(c._h, buf, nw)
    s = np.frombuffer(buf, dtype=np.uint64).reshape(nw, 10).astype(np.int64)
    n = len(s)
    t0 = s[:, 0].min()
    us = lambda x: (x - t0) / 100.0  # 100 MHz -> us
    start, ex, end = us(s[:, 0]), us(s[:, 2]), us(s[:, 3])
    n_ev, n_ev_ex, sx, xcc = s[:, 5], s[:, 7], s[:, 8], s[:, 9]
    late = start > 0.5 * end.max()  # workgroups admitted only when others left (grid > residency)
    print(f"waves that started after half the span: {late.sum()}")
    q = lambda v: " ".join(f"{np.percentile(v, p):8.1f}" for p in (0, 10, 50, 90, 99, 100))
    print(f"{a.scene} {W}x{H} {a.iters} it shard 1/{a.shard}: {n} waves, kernel {st.kernel_ms:.3f} ms (events), "
          f"steps {st.steps}, paths {st.paths}")
    print("                 percentiles  0      10      50      90      99     100 (us from first wave start)")
    print(f"start          {q(start)}")
    print(f"exhausted      {q(ex)}")
    print(f"end            {q(end)}")
    print(f"end-exhausted  {q(end - ex)}")
    span = end.max()
    print(f"span {span:.1f} us; all waves exhausted at {ex.max():.1f} us; first wave ends {end.min():.1f} us")
    tot_steps = float(st.steps)
    t_ex0 = ex.min()
    print(f"lane-steps after this wave's exhaustion: {sx.sum() / tot_steps:.4f} of all; wave-time after "
          f"exhaustion {(end - ex).sum() / (end - start).sum():.4f} of all wave-time; ideal tail at the "
          f"pre-exhaustion step rate {sx.sum() / tot_steps * t_ex0:.1f} us vs actual {span - t_ex0:.1f} us")
    print(f"event batches after exhaustion {n_ev_ex.sum() / n_ev.sum():.4f} ({n_ev_ex.mean():.1f} per wave, "
          f"{n_ev.mean():.1f} total per wave)")
    # active waves over time
    grid = np.linspace(0, span, 41)
    act = [(np.sum((start <= g) & (end > g))) for g in grid]
    print("waves alive over time (us: count):")
    print("  " + "  ".join(f"{g:.0f}:{v}" for g, v in zip(grid[::2], act[::2])))
    # drain timelines of the last waves to end
    lib.cvr_debug_tailtimeline.argtypes = [C.c_void_p, C.POINTER(C.c_uint64), C.c_size_t]
    tl = (C.c_uint64 * (n * 48))()
    lib.cvr_debug_tailtimeline(c._h, tl, n)
    tl = np.frombuffer(tl, dtype=np.uint64).reshape(n, 48)
    order = np.argsort(-end)
    for w in order[:4]:
        print(f"  wave {w} (xcc {xcc[w]}): exhausted {ex[w]:.1f} end {end[w]:.1f} us, {n_ev_ex[w]} batches after:")
        row = []
        for k in range(min(int(n_ev_ex[w]), 48)):
            v = int(tl[w, k])
            row.append(f"{(v & 0xFFFFFFFF) / 100:.1f}+{((v >> 32) & 0xFFFF) / 100:.1f}us b{(v >> 48) & 255} "
                       f"r{(v >> 56) & 255}")
        print("    " + " | ".join(row))
    for x in range(8):
        m = xcc == x
        if m.any():
            print(f"  xcc {x}: {m.sum()} waves, exhausted {ex[m].min():.1f}-{ex[m].max():.1f}, "
                  f"end p50 {np.median(end[m]):.1f} max {end[m].max():.1f}")


if __name__ == "__main__":
    main()
