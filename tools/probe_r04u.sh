#!/bin/bash
# Round 4: enc_cols_fused's tower-split form for small calls (SHELFI_ENC_TS): parity, then A/Bs at
# K = 4 (cfg2's per-learner call), 16, 64 and 714 -> gpurun_out/r04u/
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04u
mkdir -p $out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
run 400 python -u -m pytest tests/test_gpu_switches.py tests/test_gpu_parity.py tests/test_gpu_shapes.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
tail -1 $out/tests.log
for k in 4 16 64 714; do
  VAR=SHELFI_ENC_TS VALS=0,1 K=$k REPS=6 run 200 python tools/enc_variant_probe.py > $out/ts_k$k.txt 2>&1
  grep -v amdgpu.ids $out/ts_k$k.txt
done
echo probe_r04u done
