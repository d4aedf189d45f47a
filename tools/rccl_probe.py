"""The N>1 collectives bench.py uses, run over RCCL on whatever GPUs the
launch has (one rank per GPU; a 1-GPU box runs world size 1):
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N \\
      --master-addr 127.0.0.1 --master-port 29561 tools/rccl_probe.py
Process-group init with the high-priority RCCL stream, the reduce-scatter
into the shared pinned host image on a high-priority copy stream, the MAX
time reduction and the barriers; checks the host image against the sum."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cudavolumerenderer_amd.distributed import HostImage, init_process_group, reduce_to_host  # noqa: E402


def main():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    init_process_group(dist, "nccl", dev)
    n = 1024 * 1024 * 4
    host = HostImage(torch, dist, n, rank, world)
    acc = torch.full((host.chunk * world,), float(rank + 1), device=dev)
    part = torch.empty(host.chunk, device=dev)
    cs = torch.cuda.Stream(device=dev, priority=-1)
    cs.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(cs):
        reduce_to_host(acc, part, host, 2.0, dist)
    torch.cuda.synchronize()
    dist.barrier()
    want = sum(range(1, world + 1)) / 2.0
    got = host.slice(rank)[: min(host.chunk, n - rank * host.chunk)]
    assert bool((got == want).all()), (float(got.min()), float(got.max()), want)
    t = torch.tensor([float(rank)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    assert float(t.item()) == world - 1
    host.close(dist)
    dist.destroy_process_group()
    if rank == 0:
        print(f"rccl probe ok: world {world}, reduce-scatter of {n} floats into the host image")


if __name__ == "__main__":
    main()
