#!/bin/bash
# Round 5: flooding normals drawn on a side stream, added inside fft_fwd_whole<true> (tests + bench A/B vs HEAD lib)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r05z}
mkdir -p $out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
run 600 python -u -m pytest tests/test_gpu_decode_noise.py tests/test_gpu_parity.py tests/test_gpu_switches.py tests/test_gpu_palisade_wire.py tests/test_gpu_fedavg.py tests/test_gpu_golden.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
tail -1 $out/tests.log
for i in 1 2; do
  run 400 python bench.py --no-cpu-baseline --api-cts 0 > $out/bench_$i.json 2> $out/bench_$i.err
  python -c "
import json; d=json.load(open('$out/bench_$i.json'))
print('run $i', d['value'], d['encode_encrypt_ms_per_ct'], d['decrypt_decode_ms_per_ct'], d['decrypt_decode_flooded_ms_per_ct'], d['roofline']['frac'])"
done
echo probe_r05z done
