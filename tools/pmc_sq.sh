#!/bin/bash
# SQ counters per kernel for the bench's encrypt/aggregate/decrypt kernels (one --pmc pass,
# kernel trace only): where the waves' cycles go (VALU issue, waits), per dispatch.
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/pmc_sq
mkdir -p "$out"
timeout -k 10 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY \
  SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-trace \
  --output-format csv -d "$out" -o sq -- /usr/bin/python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline \
  --api-cts 0 --no-check > "$out/bench.json" 2> "$out/bench.err"
