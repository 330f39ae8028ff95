#!/bin/bash
# Round 4: wave-local exchanges in the NTT block passes (SHELFI_NTT_WL=1): parity under the switch,
# then same-process A/Bs of encrypt and decrypt -> gpurun_out/r04r/
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04r
mkdir -p $out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
SHELFI_NTT_WL=1 run 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_decode_towers.py tests/test_gpu_decode_noise.py tests/test_gpu_param_sweep.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/gpu_tests_wl.log 2>&1
tail -1 $out/gpu_tests_wl.log
VAR=SHELFI_NTT_WL K=715 REPS=2 run 200 python tools/enc_variant_probe.py > $out/wl_odd.txt 2>&1
grep -v amdgpu.ids $out/wl_odd.txt | head -1
VAR=SHELFI_NTT_WL K=714 REPS=8 run 300 python tools/enc_variant_probe.py > $out/wl_ab.txt 2>&1
grep -v amdgpu.ids $out/wl_ab.txt
VAR=SHELFI_NTT_WL K=714 REPS=8 FLOOD=1 run 300 python tools/enc_variant_probe.py > $out/wl_ab_flood.txt 2>&1
grep -v amdgpu.ids $out/wl_ab_flood.txt
echo probe_r04r done
