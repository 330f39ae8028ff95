#!/bin/bash
# Round 5: a step's learners packed into full ring slots (one gather of pieces per step): tests, cold rates at
# the cfg3 / cfg2 / cfg5 shapes, slot size 16 vs 32 MiB, a copy trace of cfg2
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r05cq}
mkdir -p $out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
run 600 python -u -m pytest tests/test_gpu_switches.py tests/test_gpu_api_guards.py tests/test_gpu_palisade_wire.py tests/test_gpu_packed_wire.py tests/test_gpu_parity.py tests/test_gpu_fedavg.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
tail -1 $out/tests.log
run 400 python -u tools/bytes_api_cold.py --learners 16 --k 64 --rounds 6 base SHELFI_STAGE_SLOT_MIB=32 > $out/cfg3.json 2> $out/cfg3.err
tail -1 $out/cfg3.json
run 300 python -u tools/bytes_api_cold.py --learners 16 --k 64 --rounds 4 --wire shelfi base SHELFI_STAGE_SLOT_MIB=32 > $out/cfg3_shelfi.json 2> $out/cfg3_shelfi.err
tail -1 $out/cfg3_shelfi.json
run 300 python -u tools/bytes_api_cold.py --learners 16 --k 4 --rounds 6 base SHELFI_STAGE_SLOT_MIB=32 > $out/cfg2.json 2> $out/cfg2.err
tail -1 $out/cfg2.json
run 400 python -u tools/bytes_api_cold.py --learners 8 --k 64 --rounds 4 base SHELFI_STAGE_SLOT_MIB=32 > $out/cfg5.json 2> $out/cfg5.err
tail -1 $out/cfg5.json
run 300 rocprofv3 --memory-copy-trace --kernel-trace --output-format csv -d $out/tr -o cfg2 -- /usr/bin/python3 tools/bytes_api_cold.py --learners 16 --k 4 --rounds 2 base > $out/tr.txt 2>&1
echo probe_r05cq done
