#!/bin/bash
# Round 5: flooded decrypt, noise drawn on a side stream vs in line (bench, alternated)
# (SHELFI_FLOOD_SIDE belonged to the reverted side-stream build; the switch no longer exists: DESIGN.md §4.3 item 8)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r05zb}
mkdir -p $out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
run 300 python -u -m pytest tests/test_gpu_decode_noise.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
tail -1 $out/tests.log
SHELFI_FLOOD_SIDE=0 run 300 python -u -m pytest tests/test_gpu_decode_noise.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $out/tests_inline.log 2>&1
tail -1 $out/tests_inline.log
for i in 1 2; do
  for sd in 1 0; do
    SHELFI_FLOOD_SIDE=$sd run 400 python bench.py --no-cpu-baseline --api-cts 0 > $out/bench_side${sd}_$i.json 2> $out/bench_side${sd}_$i.err
    python -c "
import json; d=json.load(open('$out/bench_side${sd}_$i.json'))
print('side $sd run $i', d['value'], d['encode_encrypt_ms_per_ct'], d['decrypt_decode_ms_per_ct'], d['decrypt_decode_flooded_ms_per_ct'], d['roofline']['frac'])"
  done
done
echo probe_r05zb done
