#!/bin/bash
# Round 5: cfg2-shaped bytes-API calls cut into 1 / 2 / 4 / 8 learner groups (temporary A/B)
# (SHELFI_WAVG_GROUPS_AB was a temporary switch of that A/B build; removed with the group split: DESIGN.md §5.3)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r05ct}
mkdir -p $out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
# (the switch is read per call: getenv inside the pipeline, so setting it between calls works)
run 300 python -u -m pytest tests/test_gpu_api_guards.py tests/test_gpu_switches.py tests/test_gpu_palisade_wire.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
tail -1 $out/tests.log
run 400 python -u tools/bytes_api_cold.py --learners 16 --k 4 --rounds 8 base SHELFI_WAVG_GROUPS_AB=1 SHELFI_WAVG_GROUPS_AB=2 SHELFI_WAVG_GROUPS_AB=8 > $out/cfg2.json 2> $out/cfg2.err
tail -1 $out/cfg2.json
run 300 python -u tools/bytes_api_cold.py --learners 16 --k 4 --rounds 8 --wire shelfi base SHELFI_WAVG_GROUPS_AB=1 SHELFI_WAVG_GROUPS_AB=2 SHELFI_WAVG_GROUPS_AB=8 > $out/cfg2_shelfi.json 2> $out/cfg2_shelfi.err
tail -1 $out/cfg2_shelfi.json
echo probe_r05ct done
