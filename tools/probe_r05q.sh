#!/bin/bash
# Round 5: bench A/B of the staging ring's slot size (8 vs 16 MiB), alternated
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r05q}
mkdir -p $out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
for i in 1 2; do
  for sm in 8 16; do
    SHELFI_STAGE_SLOT_MIB=$sm run 400 python bench.py --no-cpu-baseline > $out/bench_s${sm}_$i.json 2> $out/bench_s${sm}_$i.err
    python -c "
import json; d=json.load(open('$out/bench_s${sm}_$i.json')); a=d['api_bytes_path']
print('slot $sm run $i', d['value'], d['encode_encrypt_ms_per_ct'], d['encode_encrypt_per_learner_call_ms_per_ct'], a['input_GB_per_s'], a.get('cold',{}).get('input_GB_per_s'), a['shelfi_wire']['input_GB_per_s'], a['packed_wire']['input_GB_per_s'], a['decrypt']['blob_GB_per_s'], a['packed_wire']['decrypt']['blob_GB_per_s'])"
  done
done
echo probe_r05q done
