#!/bin/bash
# Round 4 final profile set in one call: the GPU suite, tools/profile_r02.sh TAG (default bench under
# rocprofv3 --kernel-trace --stats, FETCH/WRITE passes for wavg and the encrypt/decrypt chains, one SQ
# pass), the cfg2/4/5 bench lines, the effective clock per encrypt/decrypt kernel, tools/profile_f4.sh TAG.
#   tools/profile_r04.sh r04z   -> gpurun_out/profile_r04z/, gpurun_out/f4_r04z/
set -uo pipefail
tag=${1:?round tag}
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/profile_$tag
mkdir -p "$out"
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
run 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$out/${tag}_gpu_tests.log" 2>&1
tail -1 "$out/${tag}_gpu_tests.log"
run 1100 bash tools/profile_r02.sh "$tag"
python3 -c "import json; d=json.load(open('$out/${tag}_bench.json')); r=d['roofline']; print('cfg3', d['value'], d['ms_per_step'], r['frac'], r.get('traffic'), d['encode_encrypt_ms_per_ct'], d['decrypt_decode_ms_per_ct'], d['decrypt_decode_flooded_ms_per_ct'])"
for w in cfg2 cfg4 cfg5; do
  run 300 python3 bench.py --workload "$w" --no-cpu-baseline > "$out/${tag}_bench_$w.json" 2> "$out/${tag}_bench_$w.err"
  python3 -c "import json; d=json.load(open('$out/${tag}_bench_$w.json')); r=d['roofline']; print('$w', d['value'], d['ms_per_step'], r['frac'], r.get('arena_layout'), d['encode_encrypt_ms_per_ct'], d['decrypt_decode_ms_per_ct'], d['decrypt_decode_flooded_ms_per_ct'])"
done
run 180 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d "$out/clock" -o clock -- /usr/bin/python3 tools/encdec_prof.py 714 9 > "$out/clock.txt" 2>&1
python3 tools/grbm_clock.py "$out/clock" -o "$out/encdec_clock.json" > "$out/${tag}_clock.txt" 2>&1
run 600 bash tools/profile_f4.sh "$tag"
echo "profile set $tag done"
