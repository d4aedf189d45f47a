#!/usr/bin/env python3
"""Do consecutive renders overlap when they alternate between two contexts
(each with its own stream and work area)?  The wave-pool kernel's ramp-up and
tail (its last, long paths on few lanes) leave CUs idle; a second render's
waves can fill them.  Prints the per-render time of K renders on one context
and alternating over two (kernel + clear only, no copy)."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import cudavolumerenderer_amd as cvr  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="manix")
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--shard", type=int, default=1)
    ap.add_argument("--grid", type=int, default=0, help="wave-pool workgroups per launch (0: full occupancy)")
    ap.add_argument("--contexts", type=int, nargs="*", default=[1, 2, 3, 4], help="renders in flight to time")
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    scene = cvr.Scene.synthetic(a.scene)
    W = H = a.res
    iv, r2v = cvr.default_camera(W, H)
    ctxs = []
    for k in range(max(a.contexts)):
        c = cvr.Context(0, "regenerationSK")
        if k:
            c.share_medium(ctxs[0])
        elif scene.is_sparse:
            c.set_medium_sparse(scene.sparse_medium)
        elif k == 0:
            c.set_medium(scene.medium)
        c.set_camera(iv, r2v, (W, H))
        if a.grid:
            c.set_option(cvr.OPT_GRID, a.grid)
        c.init()
        c.use_own_stream()
        c.set_resolution(W, H)
        c.set_iterations(a.iters)
        if a.shard > 1:
            c.set_path_range(0, W * H * a.iters)
            c.set_block_shard(0, a.shard)
        ctxs.append(c)

    def run(cs, steps):
        for c in cs:
            c.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            c = cs[i % len(cs)]
            c.clear_output()
            c.launch_render()
        for c in cs:
            c.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3

    n_paths = W * H * a.iters / a.shard
    for rnd in range(a.rounds):
        ts = [run(ctxs[:n], a.steps) for n in a.contexts]
        print(f"round {rnd} grid {a.grid or 'full'} shard 1/{a.shard}: " +
              ", ".join(f"{n} in flight {t:.3f} ms ({n_paths / t / 1e3:.0f} Msamples/s)" for n, t in zip(a.contexts, ts)),
              flush=True)

if __name__ == "__main__":
    main()
