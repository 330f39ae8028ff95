#!/bin/bash
# Round 5: whole-vector FFT (parity suites + same-process A/B), then the bytes-API A/B per NUMA binding
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r05h
mkdir -p $out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
run 400 python -u -m pytest tests/test_gpu_switches.py tests/test_gpu_decode_noise.py tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_encode_large.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
tail -1 $out/tests.log
run 240 python -u tools/switch_ab.py base SHELFI_FFT_WHOLE=0 > $out/ab_fft.json 2>&1
tail -1 $out/ab_fft.json
bash tools/probe_r05g.sh
