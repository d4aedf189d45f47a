#!/usr/bin/env python3
"""Kernel time of the wave-pool launch under different pixel-block orders
(cvr_set_block_order): natural, costly blocks first (cost from a pilot trace
of sample 0), costly last, random.  Results are identical under every order
(the RNG is bound to the path id); only the schedule changes."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import cudavolumerenderer_amd as cvr  # noqa: E402


def block_costs(ctx, W, H, samples=1, w_seg=8.0):
    rec = ctx.trace_paths(0, W * H * samples)
    img = rec["image_id"].astype(np.int64)
    cost = rec["n_steps"].astype(np.float64) + w_seg * rec["n_segments"]
    px, py = img % W, img // W
    b = (py // 8) * (W // 8) + px // 8
    return np.bincount(b, weights=cost, minlength=(W // 8) * (H // 8))


ctx_blocks_x = [0]


def order(ctx, tile_cost, rank, world, how, rng):
    nb, nq, qbeg = ctx.launch_blocks()
    local_cost = tile_cost[rank + world * np.arange(nb)]
    perm = np.arange(nb, dtype=np.uint32)
    for q in range(nq):
        a, e = qbeg[q], qbeg[q + 1]
        idx = np.arange(a, e)
        if how == "desc":
            idx = idx[np.argsort(-local_cost[a:e], kind="stable")]
        elif how == "asc":
            idx = idx[np.argsort(local_cost[a:e], kind="stable")]
        elif how == "random":
            idx = rng.permutation(idx)
        elif how == "zorder":  # 2-D Morton order of the band's blocks (compact in-flight footprint)
            bx_n = ctx_blocks_x[0]
            tb = rank + world * idx  # tile block ids
            bx, by = tb % bx_n, tb // bx_n
            code = np.zeros(len(idx), np.int64)
            for bit in range(16):
                code |= ((bx >> bit) & 1) << (2 * bit) | ((by >> bit) & 1) << (2 * bit + 1)
            idx = idx[np.argsort(code, kind="stable")]
        perm[a:e] = idx
    return perm


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="manix")
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--shards", type=int, nargs="*", default=[1, 8])
    ap.add_argument("--orders", nargs="*", default=["natural", "desc", "asc", "random", "zorder"])
    a = ap.parse_args()
    scene = cvr.Scene.synthetic(a.scene)
    W = H = a.res
    iv, r2v = cvr.default_camera(W, H)
    c = cvr.Context(0, "regenerationSK")
    c.set_medium_sparse(scene.sparse_medium) if scene.is_sparse else c.set_medium(scene.medium)
    c.set_camera(iv, r2v, (W, H))
    c.init()
    c.set_resolution(W, H)
    c.set_iterations(a.iters)
    t0 = time.perf_counter()
    cost = block_costs(c, W, H)
    print(f"pilot trace {time.perf_counter() - t0:.2f} s; block cost max/mean {cost.max() / cost.mean():.2f}", flush=True)
    rng = np.random.default_rng(1)
    for world in a.shards:
        c.set_path_range(0, W * H * a.iters)
        c.set_block_shard(0, world)
        ctx_blocks_x[0] = W // 8
        perms = {h: order(c, cost, 0, world, h, rng) for h in a.orders}
        times = {h: [] for h in perms}
        ref = None
        for r in range(a.rounds + 1):
            for h, p in perms.items():
                c.set_block_order(p)
                c.clear_output()
                c.launch_render()
                st = c.stats()
                if ref is None:
                    ref = (st.steps, st.segments)
                assert (st.steps, st.segments) == ref, (h, st.steps, ref)
                if r:
                    times[h].append(st.kernel_ms)
        c.set_block_order(None)
        print(f"shard 1/{world}: " + ", ".join(f"{h} {np.median(t):.3f} ms" for h, t in times.items()), flush=True)


if __name__ == "__main__":
    main()
