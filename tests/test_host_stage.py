"""The bytes API's host copy pool (fhe-fed_amd/csrc/host_stage.cpp CopyPool), host
only: tools/pool_bench.cpp copies 64 MiB in 2 / 8 / 32 MiB lists with 1-8 workers
(spin-then-sleep hand-off) and checks every byte, also for lists shared by only some
of the workers (the upload fills)."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT

HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_copy_pool_is_exact(tmp_path):
    exe = str(tmp_path / "pool_bench")
    csrc = os.path.join(ROOT, "fhe-fed_amd", "csrc")
    subprocess.run([HIPCC, "-O2", "-std=c++17", "-I" + csrc, "-o", exe,
                    os.path.join(ROOT, "tools", "pool_bench.cpp"), os.path.join(csrc, "host_stage.cpp"),
                    "-lpthread"], check=True, capture_output=True, timeout=300)
    p = subprocess.run([exe, "64", "1", "2", "4", "8"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "MISMATCH" not in p.stdout
    assert p.stdout.count("GB/s") == 4 * 3
    assert p.stdout.count("partial shares ok") == 4  # lists shared by 1, half and all workers
