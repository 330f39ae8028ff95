#!/bin/bash
# Round 4: the NTT block passes with twiddles from L2 and 4 workgroups per CU (SHELFI_PP_TWG=1):
# parity under the switch, then same-process A/B of encrypt and decrypt -> gpurun_out/r04i/
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04i
mkdir -p $out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
SHELFI_PP_TWG=1 run 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_decode_towers.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/gpu_tests_twg.log 2>&1
tail -1 $out/gpu_tests_twg.log
VAR=SHELFI_PP_TWG K=714 REPS=8 run 300 python tools/enc_variant_probe.py > $out/twg_ab.txt 2>&1
grep -v amdgpu.ids $out/twg_ab.txt
VAR=SHELFI_PP_TWG K=714 REPS=8 FLOOD=1 run 300 python tools/enc_variant_probe.py > $out/twg_ab_flood.txt 2>&1
grep -v amdgpu.ids $out/twg_ab_flood.txt
echo probe_r04i done
