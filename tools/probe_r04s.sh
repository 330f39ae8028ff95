#!/bin/bash
# Round 4: ntt_inv_cols_crt with one wave per decoded tower (192 threads at the 3-tower prefix) vs 256
# threads (SHELFI_CRT_WAVES=4): parity, then same-process A/Bs -> gpurun_out/r04s/
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04s
mkdir -p $out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
run 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_decode_towers.py tests/test_gpu_decode_noise.py tests/test_gpu_shapes.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
tail -1 $out/tests.log
VAR=SHELFI_CRT_WAVES VALS=4,3 K=714 REPS=8 run 300 python tools/enc_variant_probe.py > $out/crt_ab.txt 2>&1
grep -v amdgpu.ids $out/crt_ab.txt
VAR=SHELFI_CRT_WAVES VALS=4,3 K=714 REPS=6 FLOOD=1 run 300 python tools/enc_variant_probe.py > $out/crt_ab_flood.txt 2>&1
grep -v amdgpu.ids $out/crt_ab_flood.txt
echo probe_r04s done
