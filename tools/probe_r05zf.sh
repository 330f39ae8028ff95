#!/bin/bash
# Round 5: NORED split from K = 192 only: switch / parity / encrypt tests, small-K and cfg2 bench
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r05zf}
mkdir -p $out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
run 600 python -u -m pytest tests/test_gpu_switches.py tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_encode_large.py tests/test_gpu_shapes.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
tail -1 $out/tests.log
run 300 python bench.py --workload cfg2 --no-cpu-baseline > $out/bench_cfg2.json 2> $out/bench_cfg2.err
python -c "
import json; d=json.load(open('$out/bench_cfg2.json')); a=d.get('api_bytes_path') or {}
print('cfg2', d['value'], d['encode_encrypt_ms_per_ct'], d['decrypt_decode_ms_per_ct'], d['decrypt_decode_flooded_ms_per_ct'], a.get('input_GB_per_s'), (a.get('cold') or {}).get('input_GB_per_s'), (a.get('shelfi_wire') or {}).get('input_GB_per_s'), (a.get('packed_wire') or {}).get('input_GB_per_s'))"
echo probe_r05zf done
