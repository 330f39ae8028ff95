"""bench.py end to end on the GPU (small cfg2 workload): the local N=1 step and the
N>1 code path (NCCL process group, pipelined reduce_scatter, modq) run through
torch.distributed.run with one rank; both must pass bench's own end-to-end check
(decrypt of the owned aggregate ciphertexts vs plain FedAvg of every learner)."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _run(args, timeout=300):
    env = dict(os.environ)
    p = subprocess.run(args, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, p.stdout[-2000:]  # the driver reads ONE JSON line
    return json.loads(lines[0])


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


COMMON = ["--workload", "cfg2", "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--api-cts", "4"]


def test_bench_single_gpu_line():
    r = _run([sys.executable, "bench.py"] + COMMON)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in r, k
    assert r["n_gpus"] == 1 and r["steps"] == 3 and r["value"] > 0
    assert r["roofline"]["bound"] == "hbm" and 0 < r["roofline"]["frac"] < 1
    assert r["check"]["max_abs_err"] < 1e-8
    assert r["decrypt_decode_flooded_ms_per_ct"] > 0


def test_bench_distributed_path_one_rank():
    """The default N > 1 headline, learner-sharded (NCCL group, pipelined reduce_scatter,
    modq), with the ciphertext-sharded alternative measured beside it and the C-ABI
    communicator cross-checked on the same partial sums."""
    r = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
              "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "1",
              "--force-dist", "--pieces", "3", "--comm-check"] + COMMON)
    assert "reduce_scatter" in r["config"]["workload"] and "RCCL" in r["config"]["parallelism"]
    assert r["c_abi_comm_check"]["ok"], r["c_abi_comm_check"]
    assert r["check"]["max_abs_err"] < 1e-8 and r["check"]["cts_checked_per_rank"] == 4
    alt = r["alternative_partitioning"]
    assert alt["parallelism"].startswith("ciphertext-sharded") and alt["value"] > 0
    assert alt["check"]["max_abs_err"] < 1e-8


def test_bench_ciphertext_sharded_path_one_rank():
    """--shard cts (no collective), with the RCCL learner-sharded alternative beside it."""
    r = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
              "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "1",
              "--force-dist", "--shard", "cts"] + COMMON)
    assert r["config"]["parallelism"] == "ciphertext-sharded dp1 (no collective)"
    assert r["check"]["max_abs_err"] < 1e-8
    alt = r["alternative_partitioning"]
    assert "RCCL" in alt["parallelism"] and alt["check"]["max_abs_err"] < 1e-8


def test_bench_learner_sharded_c_abi_combine_one_rank():
    """--combine shelfi: the learner-sharded step through the library's own RCCL
    communicator, pipelined inside libshelfi (shelfi_dev_combine_arena), id broadcast over the
    torch process group; bench's end-to-end check decrypts the unfolded share
    (shelfi_dev_decrypt_sum) and the line records the cross-check against torch's
    all_reduce + modq on the same partial sums."""
    for extra in ([], ["--shelfi-fold"]):
        r = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                  "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "1",
                  "--force-dist", "--shard", "learners", "--combine", "shelfi", "--pieces", "3",
                  "--no-alt", "--comm-check"] + extra + COMMON)
        assert r["check"]["max_abs_err"] < 1e-8 and r["check"]["cts_checked_per_rank"] == 4
        assert r["c_abi_comm_check"]["ok"], r["c_abi_comm_check"]
        assert "shelfi_dev_combine_arena" in r["config"]["workload"]


def test_bench_spawns_its_own_ranks():
    """Bare `bench.py --gpus N` (no launcher, WORLD_SIZE unset) starts its ranks itself through
    torch.distributed.run before any GPU call; --spawn takes that path at N = 1 on this box.
    The child's line (one rank: the local step) is relayed unchanged on stdout."""
    r = _run([sys.executable, "bench.py", "--gpus", "1", "--spawn", "--no-alt"] + COMMON)
    assert r["n_gpus"] == 1 and r["value"] > 0
    assert "c_abi_comm_check" not in r
    assert r["check"]["max_abs_err"] < 1e-8
