#!/usr/bin/env python3
"""cvr_render_frame in a process with one context (no other streams): ms per
synchronous render, repeated (C2 by default), for the variants named in
--variants: flush (one launch, in-launch output), copy (one launch, normalise +
copy after it), bands2 / bands3 (2 / 3 bands of block rows, copies overlapped),
giveup (the in-launch output instance whose flushers leave at once).

  python tools/frame_probe.py [--scene manix] [--reps 20] [--variants flush,copy]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="manix")
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="flush,copy,bands2,bands3")
    ap.add_argument("--lib", default=None, help="alternative libcvr.so (experiment builds)")
    a = ap.parse_args()
    import torch
    import cudavolumerenderer_amd as cvr
    if a.lib:
        from cudavolumerenderer_amd import _lib as lb
        lb.LIB_PATH = os.path.abspath(a.lib)
    scene = cvr.Scene.synthetic(a.scene)
    W = H = a.res
    iv, r2v = cvr.default_camera(W, H)
    c = cvr.Context(0, "regenerationSK")
    c.set_medium(scene.medium)
    c.set_camera(iv, r2v, (W, H))
    c.init()
    c.set_resolution(W, H)
    c.set_iterations(a.iters)
    host = torch.empty(W * H * 4, dtype=torch.float32, pin_memory=True)
    # giveup: the in-launch output instance with its flushers leaving at once (its block
    # counting without the stores; the host normalises and copies after the launch)
    table = {"flush": (1, 1), "copy": (1, 0), "bands2": (2, 0), "bands3": (3, 0), "giveup": (1, 2)}
    for rnd in range(a.rounds):
        for v in a.variants.split(","):
            parts, flush = table[v]
            c.set_option(cvr.OPT_FRAME_FLUSH, flush)
            for _ in range(3):
                c.render_frame(host.data_ptr(), parts, stats=False, host_floats=host.numel())
            t0 = time.perf_counter()
            for _ in range(a.reps):
                c.render_frame(host.data_ptr(), parts, stats=False, host_floats=host.numel())
            ms = (time.perf_counter() - t0) / a.reps * 1e3
            _, st = c.render_frame(host.data_ptr(), parts, host_floats=host.numel())
            print(f"round {rnd} {v:6s}: {ms:.3f} ms per render (one more with counters: clear..end "
                  f"{st.kernel_ms:.3f} ms, flushed blocks {c.frame_flush_info()}), "
                  f"{W * H * a.iters / ms / 1e3:.1f} Msamples/s", flush=True)


if __name__ == "__main__":
    main()
