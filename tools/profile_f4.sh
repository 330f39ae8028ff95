#!/bin/bash
# §8 f4 profile set: kernel stats of tools/f4_time.py, then SQ_INSTS_VALU, FETCH_SIZE and WRITE_SIZE in
# separate --pmc passes over one mult + one rescale (K ciphertexts), attributed by tools/f4_counters.py.
# usage: tools/profile_f4.sh TAG [K]   -> gpurun_out/f4_TAG/
set -euo pipefail
tag=$1
K=${2:-128}
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/f4_$tag
mkdir -p "$out"
timeout -k 10 200 python3 tools/f4_time.py 256 5 "$out/f4_time.json" > "$out/f4_time.log" 2>&1
bash tools/prof_stats.sh "f4_$tag" /usr/bin/python3 tools/f4_time.py 256 3
cp gpurun_out/prof_f4_$tag/f4_${tag}_kernel_stats.csv gpurun_out/prof_f4_$tag/summary.txt "$out/"
for c in SQ_INSTS_VALU FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$out/pmc_$c" -o pmc -- /usr/bin/python3 tools/f4_time.py "$K" 0 > "$out/pmc_$c.log" 2>&1
done
python3 tools/f4_counters.py "$K" "$out"/pmc_*/pmc_counter_collection.csv -o "$out/f4_counters.json"
