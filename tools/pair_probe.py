#!/usr/bin/env python3
"""CVR_OPT_WAVE_PAIR probe: the paired-wave kernel against the one-wave pool at
growing launch sizes (counters equal?, watchdog / dropped-entry reports in the
truncated counter, wall time), one line per size, flushed as it goes.
  python tools/pair_probe.py [--scene manix] [--sizes 256x4,512x4,1024x1,1024x4,1024x20]"""
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
    ap.add_argument("--sizes", default="256x4,512x4,1024x1,1024x4,1024x20")
    ap.add_argument("--grid", type=int, default=0)
    a = ap.parse_args()
    scene = cvr.Scene.synthetic(a.scene)
    for sz in a.sizes.split(","):
        res, it = map(int, sz.split("x"))
        iv, r2v = cvr.default_camera(res, res)
        row = []
        for pair in (0, 1):
            c = cvr.Context(0, "regenerationSK")
            c.set_medium(scene.medium)
            c.set_camera(iv, r2v, (res, res))
            c.set_option(cvr.OPT_WAVE_PAIR, pair)
            if a.grid:
                c.set_option(cvr.OPT_GRID, a.grid)
            c.init()
            c.set_resolution(res, res)
            c.set_iterations(it)
            ts = []
            for _ in range(3):
                c.clear_output()
                t0 = time.perf_counter()
                c.launch_render()
                st = c.stats()
                ts.append((time.perf_counter() - t0) * 1e3)
            row.append((min(ts), st))
            c.close()
        (t0, s0), (t1, s1) = row
        same = all(getattr(s0, k) == getattr(s1, k) for k in ("paths", "segments", "steps", "density", "albedo",
                                                             "escaped", "truncated"))
        print(f"{a.scene} {res}^2 x{it}: one-wave {t0:8.3f} ms  pair {t1:8.3f} ms  counters equal {same}  "
              f"pair truncated {s1.truncated} paths {s1.paths}/{s0.paths} segments {s1.segments}/{s0.segments}",
              flush=True)


if __name__ == "__main__":
    main()
