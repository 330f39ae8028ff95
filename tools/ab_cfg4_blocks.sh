#!/bin/bash
# cfg4 shape (2^16 / L6) A/B of the NTT block size (SHELFI_NTT_BLOCK_LOG_BIG, one process each,
# alternated 3 times): encrypt / decrypt (tools/encdec_prof.py) and EvalMult / ModReduce
# (tools/f4_time.py).  Usage: tools/ab_cfg4_blocks.sh [K]
set -euo pipefail
K=${1:-256}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export BATCH=32768 DEPTH=5
for i in 1 2 3; do
  for v in 11 12; do
    echo -n "SHELFI_NTT_BLOCK_LOG_BIG=$v  "
    SHELFI_NTT_BLOCK_LOG_BIG=$v timeout -k 10 120 python tools/encdec_prof.py "$K" 5 2>/dev/null
    echo -n "    f4: "
    SHELFI_NTT_BLOCK_LOG_BIG=$v timeout -k 10 120 python tools/f4_time.py 64 5 2>/dev/null
  done
done
