#!/bin/bash
# Round 4 end (final binaries): the GPU suite at the final tree, smoke, the default bench line and cfg2 -> gpurun_out/r04zb/
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04zb
mkdir -p $out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
run 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $out/gpu_tests.log 2>&1
tail -1 $out/gpu_tests.log
run 300 python __graft_entry__.py smoke > $out/smoke.log 2>&1
tail -1 $out/smoke.log
run 400 python bench.py > $out/bench.json 2> $out/bench.err
run 300 python bench.py --workload cfg2 --no-cpu-baseline > $out/bench_cfg2.json 2> $out/bench_cfg2.err
for f in bench bench_cfg2; do
  python -c "import json; d=json.load(open('$out/$f.json')); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], r['frac'], d['encode_encrypt_ms_per_ct'], d['decrypt_decode_ms_per_ct'], d['decrypt_decode_flooded_ms_per_ct'])"
done
echo probe_r04zb done
