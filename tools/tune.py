#!/usr/bin/env python3
"""Scheduler/option sweep on the C2 workload (manix proxy, 1024^2, 20 it), one
process, interleaved rounds (cdna_hip_programming.md §5.4 rule 24).

  python tools/tune.py [--rounds 3] [--variants "regenerationSK:ev=16,chunk=128" ...]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import cudavolumerenderer_amd as cvr  # noqa: E402

DEFAULT = [
    "naiveSK:",
    "regenerationSK:bounds=0",
    "regenerationSK:bounds=1",
    "regenerationSK:",
    "regenerationSK:bounds=3",
    "regenerationSK:bounds=4",
    "regenerationSK:cells=0",
    "regenerationSK:bounds=3,cells=0",
    "regenerationSK:ev=32",
    "regenerationSK:ev=48",
    "regenerationSK:ev=62",
    "regenerationSK:sched=2",
    "regenerationSK:sched=2,tail=8",
    "regenerationSK:sched=2,tail=32",
]


def parse(v):
    k, _, opts = v.partition(":")
    d = {}
    for kv in filter(None, opts.split(",")):
        a, b = kv.split("=")
        d[a] = int(b)
    return k, d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--res", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--scene", default="manix")
    ap.add_argument("--variants", nargs="*", default=DEFAULT)
    ap.add_argument("--lib", default=None, help="alternative libcvr.so (experiment builds)")
    a = ap.parse_args()
    if a.lib:
        import cudavolumerenderer_amd._lib as lb
        lb.LIB_PATH = os.path.abspath(a.lib)
    scene = cvr.Scene.synthetic(a.scene)
    W = H = a.res
    iv, r2v = cvr.default_camera(W, H)
    ctxs = []
    for v in a.variants:
        k, d = parse(v)
        c = cvr.Context(0, k)
        c.set_option(cvr.OPT_CELLS, d.get("cells", 1))
        if "ualb" in d:
            c.set_option(cvr.OPT_UNIFORM_ALBEDO, d["ualb"])
        if "bounds" in d:
            c.set_option(cvr.OPT_BOUNDS, d["bounds"])
        if scene.is_sparse or d.get("sparse", 0):
            c.set_medium_sparse(scene.sparse_medium)
        else:
            c.set_medium(scene.medium)
        c.set_camera(iv, r2v, (W, H))
        if "ev" in d:
            c.set_option(cvr.OPT_EVENT_THRESHOLD, d["ev"])
        if "chunk" in d:
            c.set_option(cvr.OPT_CHUNK, d["chunk"])
        if "grid" in d:
            c.set_option(cvr.OPT_GRID, d["grid"])
        if "sched" in d:
            c.set_option(cvr.OPT_SCHEDULER, d["sched"])
        if "order" in d:
            c.set_option(cvr.OPT_ORDER, d["order"])
        if "queues" in d:
            c.set_option(cvr.OPT_QUEUES, d["queues"])
        if "sub" in d:
            c.set_option(cvr.OPT_SUBQUEUES, d["sub"])
        if "drain" in d:
            c.set_option(cvr.OPT_DRAIN, d["drain"])
        if "waves" in d:
            c.set_option(cvr.OPT_WAVES, d["waves"])
        if "batch" in d:
            c.set_option(cvr.OPT_BATCH, d["batch"])
        if "tail" in d:
            c.set_option(cvr.OPT_TAIL, d["tail"])
        if "morton" in d:
            c.set_option(cvr.OPT_MORTON, d["morton"])
        if "pool" in d:
            c.set_option(cvr.OPT_POOL, d["pool"])
        if "pair" in d:
            c.set_option(cvr.OPT_WAVE_PAIR, d["pair"])
        if "sorder" in d:
            c.set_option(cvr.OPT_SAMPLE_ORDER, d["sorder"])
        if "em" in d:
            c.set_option(cvr.OPT_EMPTY_MASK, d["em"])
        c.set_option(cvr.OPT_TIMING, d.get("timing", 1))
        c.init()
        c.set_resolution(W, H)
        c.set_iterations(a.iters)
        if "shard" in d:  # block shard `rank` of `shard` (bench.py's strong-scaling split), one GPU
            c.set_path_range(0, W * H * a.iters)
            c.set_block_shard(d.get("rank", 0), d["shard"])
        ctxs.append((v, c))
    times = {v: [] for v, _ in ctxs}
    extra = {}
    for r in range(a.rounds + 1):
        print(f"round {r}/{a.rounds}", file=sys.stderr, flush=True)  # (progress: long runs stay observable)
        for v, c in ctxs:
            c.clear_output()
            t0 = time.perf_counter()
            c.launch_render()
            st = c.stats()
            wall = (time.perf_counter() - t0) * 1e3
            if r > 0:
                times[v].append(wall)
                extra[v] = (st.kernel_ms, st.iterations, st.track_ms, st.events_ms, st.steps, st.escaped, st.fetches,
                            st.density)
    cu, grid = ctxs[-1][1].device_info()
    print(f"CUs {cu}, persistent grid {grid} blocks; steps/launch {st.steps}, density {st.density}")
    for v, _ in ctxs:
        t = np.array(times[v])
        kms, its, tms, ems, steps, esc, fetches, dens = extra[v]
        gsteps = steps / (np.median(t) * 1e-3) / 1e9
        print(f"{v:42s} wall {np.median(t):8.3f} ms (min {t.min():7.3f}) dev {kms:8.3f}  it {its:4d} "
              f"track {tms:7.3f} events {ems:7.3f}  {W * H * a.iters / np.median(t) / 1e3:7.1f} Msamples/s "
              f"{gsteps:6.2f} Gsteps/s  esc {esc} fetch {fetches / max(dens, 1):.3f}", flush=True)


if __name__ == "__main__":
    main()
