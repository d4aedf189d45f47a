"""`python3 bench.py --gpus N` without a launcher (the driver's own command) starts its
N ranks itself: bench.spawn_ranks gives each child RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_* as torch.distributed.run would, relays rank 0's JSON line and exits with the
worst child status; with fewer visible GPUs than N it refuses instead of running one
rank.  CPU only: the children here are a stand-in script, and this container has no GPU."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

CHILD = """
import json, os, sys
import torch.distributed as dist
r, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", rank=r, world_size=n)   # env:// rendezvous on MASTER_*
dist.barrier()
if r == 0:
    print(json.dumps({"n_gpus": dist.get_world_size(), "argv": sys.argv[1:],
                      "local": [os.environ["LOCAL_RANK"], os.environ["MASTER_ADDR"]]}), flush=True)
dist.destroy_process_group()
sys.exit(int(os.environ.get("FAIL_RANK_RC", "0")) if str(r) == os.environ.get("FAIL_RANK") else 0)
"""


def _run_spawn(tmp_path, n, extra_env=None):
    script = tmp_path / "child.py"
    script.write_text(CHILD)
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "sys.exit(bench.spawn_ranks(['--gpus', '%d', '--x'], %d, True, script=%r))" % (ROOT, n, n, str(script)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(extra_env or {})
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, env=env)


def test_spawn_starts_n_ranks_and_relays_rank0_line(tmp_path):
    r = _run_spawn(tmp_path, 3)
    assert r.returncode == 0, r.stderr[-2000:]
    js = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(js) == 1
    line = json.loads(js[0])
    assert line["n_gpus"] == 3 and line["argv"] == ["--gpus", "3", "--x"]
    assert line["local"] == ["0", "127.0.0.1"]


def test_spawn_exit_status_is_the_worst_rank(tmp_path):
    r = _run_spawn(tmp_path, 2, {"FAIL_RANK": "1", "FAIL_RANK_RC": "7"})
    assert r.returncode == 7
    assert "rank 1 exited with status 7" in r.stderr


def test_bare_bench_refuses_more_ranks_than_gpus():
    # no GPU here: --gpus 2 must not silently run one rank
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HIP_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "refusing to run fewer ranks" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_one_gpu_run_does_not_spawn(monkeypatch):
    called = []
    monkeypatch.setattr(bench, "spawn_ranks", lambda *a, **k: called.append(a) or 0)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "1", "--help"])
    try:
        bench.main()
    except SystemExit:
        pass
    assert not called
