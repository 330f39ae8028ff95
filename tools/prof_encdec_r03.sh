#!/bin/bash
# Round 3 encrypt/decrypt baseline: us/ct of each call type (tools/encdec_prof.py, K = 714 at
# 2^15/L4) and the per-kernel rocprofv3 stats of the same command -> gpurun_out/$1/
set -e
OUT=${1:-prof_encdec}
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$OUT
timeout -k 10 120 python tools/encdec_prof.py 714 5 > gpurun_out/$OUT/encdec.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$OUT -o encdec -- /usr/bin/python3 tools/encdec_prof.py 714 3 > gpurun_out/$OUT/encdec_prof.txt 2>&1
python tools/kstat_summary.py $(find gpurun_out/$OUT -name "encdec_kernel_stats.csv" | head -1) > gpurun_out/$OUT/kernel_summary.txt
cat gpurun_out/$OUT/encdec.txt gpurun_out/$OUT/kernel_summary.txt
