#!/bin/bash
# L2 hit rate of the encrypt/decrypt kernels (tools/encdec_prof.py, K = 714): one
# TCC_HIT/TCC_MISS pass per streaming-load variant (SHELFI_NT_STREAM 0/1) -> gpurun_out/l2/
set -e
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/l2
for v in 0 1; do
  SHELFI_NT_STREAM=$v timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv \
    -d gpurun_out/l2 -o nt$v -- /usr/bin/python3 tools/encdec_prof.py 714 1 > /dev/null 2>&1
done
ls -R gpurun_out/l2 | head -20
