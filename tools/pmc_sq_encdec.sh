#!/bin/bash
# SQ counters (one --pmc pass, kernel trace only) over tools/encdec_prof.py, per kernel:
#   tools/pmc_sq_encdec.sh TAG [env assignments...]   -> gpurun_out/sq_TAG/ + summary.txt
set -euo pipefail
tag=$1
shift
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/sq_$tag
mkdir -p "$out"
for kv in "$@"; do export "$kv"; done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY \
  SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d "$out" -o sq \
  -- /usr/bin/python3 tools/encdec_prof.py 714 1 > "$out/stdout.txt" 2> "$out/stderr.txt"
python3 tools/sq_table.py "$out/sq_counter_collection.csv" > "$out/summary.txt" || true
