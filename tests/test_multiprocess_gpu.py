"""bench.py's multi-rank step, run for real: two fresh processes on the leased
GPU (gloo, since RCCL needs one device per rank), each building its own
libcvr context and rendering its shard on the torch stream through the same
step code the N-GPU benchmark runs (block shard -> k_wpool -> own blocks
normalised into the shared host image; tile x block shards -> reduce-scatter
-> slice copy; max-over-ranks time).
The image both ranks leave in host memory must equal the single-process
cvr_render_image within the fp32 summation-order bound."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from parity_util import assert_pixels_close

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


# "bare": the driver's own command, `python3 bench.py --gpus 2 ...` with no launcher: bench.py
# starts its two ranks itself (spawn_ranks); "torchrun": the torch.distributed.run form
@pytest.mark.parametrize("shard,tiles,launcher", [("paths", (1, 1), "bare"), ("tilepaths", (2, 2), "torchrun")])
def test_two_ranks_one_gpu_bench_step_equals_single_render(cvr, tmp_path, shard, tiles, launcher):
    W = H = 256
    iters = 4
    out = str(tmp_path / "img.npy")
    pre = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port())] if launcher == "torchrun" else \
          [sys.executable]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = pre + [os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1", "--backend", "gloo", "--same-device",
           "--resolution", str(W), str(H), "--iterations", str(iters), "--shard", shard,
           "--number-of-tiles", str(tiles[0]), str(tiles[1]), "--no-cpu-baseline", "--dump-image", out]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    js = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(js) == 1, r.stdout[-3000:]  # one JSON line: rank 0's, relayed
    line = json.loads(js[0])
    assert line["n_gpus"] == 2 and line["scaling"] == "strong" and line["value"] > 0
    if shard == "paths":
        assert line["weak"]["value"] > 0
    # the scaling run's self-diagnosis (bench.py rank_diagnostics)
    rk = line["ranks"]
    assert rk["world_size_reported"] == 2 and rk["backend"] == "gloo" and rk["streams_per_process"] >= 1
    keys = ["kernel_ms_min_max", "output_ms_min_max"]
    if shard != "paths":  # block shards write their own blocks: no reduce-scatter
        keys += ["reduce_scatter_ms_min_max", "slice_copy_ms_min_max"]
    for k in keys:
        lo, hi = rk[k]
        assert 0 < lo <= hi, k
    assert rk["image_check"]["match"], rk["image_check"]
    img = np.load(out)
    scene = cvr.Scene.synthetic("manix")
    ctx = cvr.Context(0, "regenerationSK")
    ctx.set_medium(scene.medium)
    iv, r2v = cvr.default_camera(W, H)
    ctx.set_camera(iv, r2v, (W, H))
    ctx.init()
    ref, st = ctx.render_image(W, H, tiles, iters)
    assert_pixels_close(img[..., :3], ref[..., :3], iters, f"2 ranks {shard}")
    assert np.nanmax(ref[..., :3]) > 0
    assert line["nan_pixels"] == int(np.isnan(ref[..., :3]).any(-1).sum())
