#!/bin/bash
# Round 4: uint64-arena slot pads vs separate batches vs the packed arena at cfg2 (and C=8),
# then bench cfg2 in both layouts -> gpurun_out/r04f/
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04f
mkdir -p $out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
run 300 python -u -m pytest tests/test_gpu_arena_u64.py tests/test_gpu_param_sweep.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $out/gpu_tests.log 2>&1
tail -1 $out/gpu_tests.log
AB_PADS=0,32,512,4096,65536 run 300 python tools/wavg_small_ab.py 11 100 > $out/wavg_small_ab.txt 2>&1
AB_PADS=0,32,512,4096,65536 run 300 python tools/wavg_small_ab.py 11 50 16 8 >> $out/wavg_small_ab.txt 2>&1
grep -v amdgpu.ids $out/wavg_small_ab.txt
for lay in arena separate; do
  run 300 python bench.py --workload cfg2 --layout $lay --no-cpu-baseline --api-cts 0 --f4-cts 0 > $out/bench_cfg2_$lay.json 2> $out/bench_cfg2_$lay.err
  python -c "import json; d=json.load(open('$out/bench_cfg2_$lay.json')); r=d['roofline']; print('$lay', d['value'], d['ms_per_step'], r['launch_ms_min'], r.get('frac'), r.get('arena_layout'))"
done
echo probe_r04f done
