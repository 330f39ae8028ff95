#!/bin/bash
# Round 5: bytes-API ring (default again) with device gather + async drain vs direct uploads, cold and warm
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r05m}
mkdir -p $out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
run 600 python -u -m pytest tests/test_gpu_switches.py tests/test_gpu_api_guards.py tests/test_gpu_palisade_wire.py tests/test_gpu_packed_wire.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
tail -1 $out/tests.log
for w in palisade shelfi packed; do
  run 400 python -u tools/bytes_api_cold.py --wire $w --rounds 4 base SHELFI_H2D_DIRECT=1 > $out/cold_$w.json 2> $out/cold_$w.err
  tail -1 $out/cold_$w.json
done
SHELFI_STAGE_TRACE=1 run 200 python -u tools/bytes_api_cold.py --rounds 1 base > $out/trace.json 2> $out/trace.err
echo probe_r05m done
