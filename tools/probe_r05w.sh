#!/bin/bash
# Round 5: bytes-API learner sub-groups for single-chunk calls + slot-sized archive chunks (tests, cfg2/cfg5/cfg3 shapes)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r05w}
mkdir -p $out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
run 600 python -u -m pytest tests/test_gpu_switches.py tests/test_gpu_api_guards.py tests/test_gpu_palisade_wire.py tests/test_gpu_packed_wire.py tests/test_gpu_parity.py tests/test_gpu_arena_u64.py tests/test_gpu_fedavg.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
tail -1 $out/tests.log
run 300 python -u tools/bytes_api_cold.py --learners 16 --k 4 --rounds 6 base > $out/cfg2.json 2> $out/cfg2.err
tail -1 $out/cfg2.json
run 300 python -u tools/bytes_api_cold.py --learners 16 --k 4 --rounds 6 --wire shelfi base > $out/cfg2_shelfi.json 2> $out/cfg2_shelfi.err
tail -1 $out/cfg2_shelfi.json
run 400 python -u tools/bytes_api_cold.py --learners 8 --k 64 --rounds 4 base > $out/cfg5.json 2> $out/cfg5.err
tail -1 $out/cfg5.json
run 400 python -u tools/bytes_api_cold.py --learners 16 --k 64 --rounds 4 base > $out/cfg3.json 2> $out/cfg3.err
tail -1 $out/cfg3.json
echo probe_r05w done
