#!/bin/bash
# Round 5: staged uploads over two DMA lanes x ring slot size (cold / warm bytes-API aggregation)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r05o}
mkdir -p $out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
SHELFI_STAGE_LANES=2 run 600 python -u -m pytest tests/test_gpu_switches.py tests/test_gpu_api_guards.py tests/test_gpu_palisade_wire.py tests/test_gpu_packed_wire.py tests/test_gpu_parity.py tests/test_gpu_arena_u64.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
tail -1 $out/tests.log
for w in palisade shelfi; do
  run 500 python -u tools/bytes_api_cold.py --wire $w --rounds 4 base SHELFI_STAGE_LANES=2 SHELFI_STAGE_LANES=2,SHELFI_STAGE_SLOT_MIB=16 SHELFI_STAGE_SLOT_MIB=16 > $out/cold_$w.json 2> $out/cold_$w.err
  tail -1 $out/cold_$w.json
done
echo probe_r05o done
