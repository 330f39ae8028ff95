#!/bin/bash
# CRT tower-loop variants (SHELFI_CRT_LT = 0 runtime loop / 4 unrolled / p prefetch): decrypt
# time A/B in one process (bit-identical decode checked), then kernel stats of the same run.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04za
mkdir -p $O
cd $R
timeout -k 10 300 env VAR=SHELFI_CRT_LT VALS=0,4,p K=714 REPS=6 python tools/enc_variant_probe.py > $O/crt_ab.txt 2>&1 || exit 1
timeout -k 10 300 env VAR=SHELFI_CRT_LT VALS=0,4,p K=714 REPS=6 FLOOD=1 python tools/enc_variant_probe.py > $O/crt_ab_flood.txt 2>&1 || exit 1
cd /tmp
VAR=SHELFI_CRT_LT VALS=0,4,p K=714 REPS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o crt -- python3 $R/tools/enc_variant_probe.py > $O/prof.log 2>&1 || exit 1
find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/crt_kernel_stats.csv \;
echo done
