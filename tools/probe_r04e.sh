#!/bin/bash
# Round 4: the small-launch A/B (tools/wavg_small_ab.py), cfg2 bench in both layouts, then the
# round profile set (tools/profile_r02.sh r04e) -> gpurun_out/r04e/, gpurun_out/profile_r04e/
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04e
mkdir -p $out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
run 300 python -u -m pytest tests/test_gpu_arena_u64.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/gpu_tests.log 2>&1
tail -1 $out/gpu_tests.log
run 300 python tools/wavg_small_ab.py 9 100 > $out/wavg_small_ab.txt 2>&1
grep -v amdgpu.ids $out/wavg_small_ab.txt
for lay in arena separate; do
  run 300 python bench.py --workload cfg2 --layout $lay --no-cpu-baseline --api-cts 0 --f4-cts 0 > $out/bench_cfg2_$lay.json 2> $out/bench_cfg2_$lay.err
  python -c "import json; d=json.load(open('$out/bench_cfg2_$lay.json')); r=d['roofline']; print('$lay', d['value'], d['ms_per_step'], r['launch_ms_min'], r.get('frac'), r.get('arena_layout'))"
done
run 1000 bash tools/profile_r02.sh r04e
echo probe_r04e done
