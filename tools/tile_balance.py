#!/usr/bin/env python3
"""Per-tile kernel time of a tiled render (C4: manix proxy 2048^2, 256 it,
4x2 tiles) and the speed-up that tile k -> GPU k could reach on N GPUs
(sum of tile times / the largest per-rank sum).

  python tools/tile_balance.py [--res 2048] [--iters 256] [--tiles 4 2]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import cudavolumerenderer_amd as cvr  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--res", type=int, default=2048)
    ap.add_argument("--iters", type=int, default=256)
    ap.add_argument("--tiles", type=int, nargs=2, default=[4, 2])
    ap.add_argument("--scene", default="manix")
    a = ap.parse_args()
    W = H = a.res
    scene = cvr.Scene.synthetic(a.scene)
    iv, r2v = cvr.default_camera(W, H)
    ctx = cvr.Context(0, "regenerationSK")
    ctx.set_medium(scene.medium)
    ctx.set_camera(iv, r2v, (W, H))
    ctx.init()
    n = a.tiles[0] * a.tiles[1]
    ctx.render_tiles(W, H, tuple(a.tiles), a.iters, 0, n)  # warm-up
    times = []
    for k in range(n):
        _, st = ctx.render_tiles(W, H, tuple(a.tiles), a.iters, k, n)
        times.append(st.kernel_ms)
        print(f"tile {k}: {st.kernel_ms:8.2f} ms  steps {st.steps}", flush=True)
    tot = sum(times)
    for g in (2, 4, 8):
        per = [sum(times[k] for k in range(r, n, g)) for r in range(g)]
        print(f"{g} GPUs, tile k -> rank k mod {g}: speed-up {tot / max(per):.2f} (ideal {g})")


if __name__ == "__main__":
    main()
