#!/bin/bash
# Two SQ counter passes (8 SQ counters each, kernel trace only) over tools/encdec_prof.py:
#   tools/pmc_sq2_encdec.sh TAG [env assignments...]  -> gpurun_out/sq2_TAG/{a,b}_counter_collection.csv
set -euo pipefail
tag=$1
shift
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/sq2_$tag
mkdir -p "$out"
for kv in "$@"; do export "$kv"; done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY \
  SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d "$out" -o a \
  -- /usr/bin/python3 tools/encdec_prof.py 714 1 > "$out/stdout_a.txt" 2> "$out/stderr_a.txt"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA \
  SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC --kernel-trace --output-format csv -d "$out" -o b \
  -- /usr/bin/python3 tools/encdec_prof.py 714 1 > "$out/stdout_b.txt" 2> "$out/stderr_b.txt"
python3 tools/sq2_table.py "$out"/a_counter_collection.csv "$out"/b_counter_collection.csv > "$out/summary.txt" || true
cat "$out/summary.txt"
