#!/bin/bash
# Round 4: bench lines at this tree (cfg3 default, cfg2/cfg5/cfg4) and cfg2 with the separate uint64
# layout (wavg_kernel over learner batches) beside the packed arena -> gpurun_out/r04b/
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04b
mkdir -p $out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
run 400 python bench.py > $out/bench_cfg3.json 2> $out/bench_cfg3.err
cat $out/bench_cfg3.json
for w in cfg2 cfg5 cfg4; do
  run 300 python bench.py --workload $w --no-cpu-baseline --api-cts 0 --f4-cts 0 > $out/bench_$w.json 2> $out/bench_$w.err
done
run 300 python bench.py --workload cfg2 --layout separate --no-cpu-baseline --api-cts 0 --f4-cts 0 > $out/bench_cfg2_separate.json 2> $out/bench_cfg2_separate.err
for f in $out/bench_cfg2.json $out/bench_cfg2_separate.json $out/bench_cfg5.json $out/bench_cfg4.json; do
  python -c "import json,sys; d=json.load(open('$f')); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], r.get('achieved'), r.get('frac'), d.get('decrypt_decode_ms_per_ct'), d.get('decrypt_decode_flooded_ms_per_ct'), d.get('encode_encrypt_ms_per_ct'))"
done
echo probe_r04b done
