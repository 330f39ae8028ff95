#!/bin/bash
# Round 6, the final tree on one box: the GPU suite, smoke, the default bench line (unprofiled), cfg4 and cfg2.
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-r06final}
out=gpurun_out/$T
mkdir -p "$out"
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
run 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$out/gpu_tests.log" 2>&1
tail -1 "$out/gpu_tests.log"
run 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
tail -1 "$out/smoke.log"
run 400 python3 bench.py > "$out/bench.json" 2> "$out/bench.err"
for w in cfg4 cfg2; do
  run 300 python3 bench.py --workload $w --no-cpu-baseline > "$out/bench_$w.json" 2> "$out/bench_$w.err"
done
echo done
