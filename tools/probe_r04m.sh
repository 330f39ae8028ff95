#!/bin/bash
# Round 4: the 512-thread two-ciphertext encrypt block pass (SHELFI_ENC_PP2=1): parity under the
# switch (odd K included), then a same-process A/B -> gpurun_out/r04m/
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04m
mkdir -p $out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
SHELFI_ENC_PP2=1 run 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_shapes.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/gpu_tests_pp2.log 2>&1
tail -1 $out/gpu_tests_pp2.log
VAR=SHELFI_ENC_PP2 K=715 REPS=2 run 200 python tools/enc_variant_probe.py > $out/pp2_odd.txt 2>&1
grep -v amdgpu.ids $out/pp2_odd.txt | head -1
VAR=SHELFI_ENC_PP2 K=714 REPS=8 run 300 python tools/enc_variant_probe.py > $out/pp2_ab.txt 2>&1
grep -v amdgpu.ids $out/pp2_ab.txt
echo probe_r04m done
