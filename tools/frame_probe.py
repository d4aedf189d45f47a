#!/usr/bin/env python3
"""cvr_render_frame in a process with one context (no other streams): ms per
synchronous render for 1, 2 and 3 bands, repeated (C2 by default).

  python tools/frame_probe.py [--scene manix] [--reps 20]
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
    a = ap.parse_args()
    import torch
    import cudavolumerenderer_amd as cvr
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
    for rnd in range(a.rounds):
        for parts in (1, 2, 3):
            for _ in range(3):
                c.render_frame(host.data_ptr(), parts)
            t0 = time.perf_counter()
            ks = 0.0
            for _ in range(a.reps):
                _, st = c.render_frame(host.data_ptr(), parts)
                ks += st.kernel_ms
            ms = (time.perf_counter() - t0) / a.reps * 1e3
            print(f"round {rnd} parts {parts}: {ms:.3f} ms per render (clear..last band {ks / a.reps:.3f} ms), "
                  f"{W * H * a.iters / ms / 1e3:.1f} Msamples/s", flush=True)


if __name__ == "__main__":
    main()
