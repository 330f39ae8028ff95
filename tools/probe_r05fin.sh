#!/bin/bash
# Round 5 final tree: the GPU suite, smoke, the default bench line and the cfg2 / cfg5 lines -> gpurun_out/<tag>/
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r05fin2}
mkdir -p $out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
run 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $out/gpu_tests.log 2>&1
tail -1 $out/gpu_tests.log
run 300 python __graft_entry__.py smoke > $out/smoke.log 2>&1
tail -1 $out/smoke.log
run 400 python bench.py > $out/bench.json 2> $out/bench.err
for w in cfg2 cfg5; do
  run 300 python bench.py --workload $w --no-cpu-baseline > $out/bench_$w.json 2> $out/bench_$w.err
done
for f in bench bench_cfg2 bench_cfg5; do
  python -c "
import json; d=json.load(open('$out/$f.json')); r=d['roofline']; a=d.get('api_bytes_path') or {}
print('$f', d['value'], d['ms_per_step'], r['frac'], d['encode_encrypt_ms_per_ct'], d['decrypt_decode_ms_per_ct'], d['decrypt_decode_flooded_ms_per_ct'], a.get('input_GB_per_s'), (a.get('cold') or {}).get('input_GB_per_s'), (a.get('shelfi_wire') or {}).get('input_GB_per_s'), (a.get('packed_wire') or {}).get('input_GB_per_s'))"
done
echo probe_r05fin done
