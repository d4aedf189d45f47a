#!/usr/bin/env python3
"""Host time of each call in bench.py's pipelined step (diagnostic): which
call blocks the host when the kernels are short."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import cudavolumerenderer_amd as cvr  # noqa: E402
from cudavolumerenderer_amd.distributed import HostImage, reduce_to_host  # noqa: E402


def main():
    res = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    scene_name = sys.argv[2] if len(sys.argv) > 2 else "manix"
    iters = 20 if scene_name != "bucky" else 4
    dev = torch.device("cuda", 0)
    scene = cvr.Scene.synthetic(scene_name)
    W = H = res
    iv, r2v = cvr.default_camera(W, H)
    streams = [torch.cuda.Stream(device=dev) for _ in range(3)]
    torch.cuda.set_stream(streams[0])
    ctxs = []
    for i, s in enumerate(streams):
        c = cvr.Context(0, "regenerationSK")
        if i == 0:
            c.set_medium(scene.medium)
        else:
            c.share_medium(ctxs[0])
        c.set_camera(iv, r2v, (W, H))
        c.init()
        c.set_stream(s.cuda_stream)
        c.set_resolution(W, H)
        c.set_iterations(iters)
        ctxs.append(c)
    n = W * H * 4
    host = HostImage(torch, None, n, 0, 1)
    bufs = [torch.zeros(n, device=dev) for _ in range(3)]
    copy_stream = torch.cuda.Stream(device=dev, priority=-1)
    ev_r = [torch.cuda.Event() for _ in range(3)]
    ev_c = [torch.cuda.Event() for _ in range(3)]
    names = ["wait", "set_output", "clear", "launch", "record", "copy_wait", "reduce", "record2"]
    acc = {k: 0.0 for k in names}
    steps = 60
    for i in range(steps + 10):
        k, c, rs = i % 3, ctxs[i % 3], streams[i % 3]
        t = [time.perf_counter()]
        if i >= 3:
            rs.wait_event(ev_c[k])
        t.append(time.perf_counter())
        c.set_output(bufs[k].data_ptr())
        t.append(time.perf_counter())
        c.clear_output()
        t.append(time.perf_counter())
        c.launch_render()
        t.append(time.perf_counter())
        ev_r[k].record(rs)
        t.append(time.perf_counter())
        copy_stream.wait_event(ev_r[k])
        t.append(time.perf_counter())
        with torch.cuda.stream(copy_stream):
            reduce_to_host(bufs[k], None, host, float(iters), None)
        t.append(time.perf_counter())
        ev_c[k].record(copy_stream)
        t.append(time.perf_counter())
        if i >= 10:
            for j, nm in enumerate(names):
                acc[nm] += t[j + 1] - t[j]
    torch.cuda.synchronize()
    print(f"{scene_name} {res}^2: host ms per step: " + ", ".join(f"{k} {1e3 * v / steps:.3f}" for k, v in acc.items()),
          flush=True)


if __name__ == "__main__":
    main()
