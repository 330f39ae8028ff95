"""bench.py's own launcher (CPU): `bench.py --gpus N` with WORLD_SIZE unset starts N ranks
through torch.distributed.run (one process per GPU, rendezvous on 127.0.0.1) before any GPU
call, relays rank 0's single JSON line and returns the launcher's exit status.  --dry-run
makes every rank stop before torch is imported, so the plumbing runs here without a GPU."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def test_launch_command_is_one_node_torch_distributed_run():
    cmd = bench.launch_command(["--gpus", "8", "--steps", "5"], 8, 29555)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd
    assert cmd[cmd.index("--nproc-per-node") + 1] == "8"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29555"
    assert cmd[-5:] == [os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "5"]


@pytest.mark.parametrize("n", [2, 3])
def test_bare_bench_spawns_its_ranks(n):
    p = subprocess.run([sys.executable, "bench.py", "--gpus", str(n), "--dry-run"], cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, p.stdout  # the driver reads ONE JSON line
    r = json.loads(lines[0])
    assert r == {"dry_run": True, "world": n, "rank": 0, "local_rank": 0, "master_addr": "127.0.0.1",
                 "gpus": n}


def test_gpus_and_world_size_must_agree():
    env = _env()
    env.update(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "4", "--dry-run"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and "WORLD_SIZE=2" in p.stderr
