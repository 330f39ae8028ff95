#!/bin/bash
# Round profile set (on the GPU box): the default bench under rocprofv3 kernel stats, HBM
# traffic passes (FETCH_SIZE and WRITE_SIZE in separate runs) for the wavg launch and the
# encrypt / decrypt chains, and one SQ pass.  Output: gpurun_out/profile_$TAG/
set -euo pipefail
tag=${1:?round tag}
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/profile_$tag
mkdir -p "$out"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o "$tag" \
  -- /usr/bin/python3 bench.py > "$out/${tag}_bench.json" 2> "$out/${tag}_bench.err"
python3 tools/kstat_summary.py "$out/${tag}_kernel_stats.csv" > "$out/${tag}_kernel_summary.txt"
B="--steps 2 --warmup 1 --no-cpu-baseline --api-cts 0 --no-check --place-output 0 --f4-cts 0"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$out" -o wfetch \
  -- /usr/bin/python3 bench.py $B > /dev/null 2> "$out/wfetch.err"
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$out" -o wwrite \
  -- /usr/bin/python3 bench.py $B > /dev/null 2> "$out/wwrite.err"
algo=$(python3 -c "import json,sys; print(json.load(open(sys.argv[1]))['roofline']['bytes_per_launch'])" "$out/${tag}_bench.json")
python3 tools/pmc_traffic.py "$out/wfetch_counter_collection.csv" "$out/wwrite_counter_collection.csv" \
  --kernel "wavg_packed" --workload cfg3 --learners 16 --algorithmic-bytes "$algo" \
  -o "$out/wavg_traffic.json" > /dev/null
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$out" -o efetch \
  -- /usr/bin/python3 tools/encdec_prof.py 714 1 > /dev/null 2> "$out/efetch.err"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$out" -o ewrite \
  -- /usr/bin/python3 tools/encdec_prof.py 714 1 > /dev/null 2> "$out/ewrite.err"
python3 tools/encdec_traffic.py "$out/efetch_counter_collection.csv" "$out/ewrite_counter_collection.csv" \
  -o "$out/encdec_traffic.json" > /dev/null
bash tools/pmc_sq_encdec.sh "$tag"
cp gpurun_out/sq_$tag/summary.txt "$out/${tag}_sq_encdec.txt"
python3 tools/encdec_valu.py gpurun_out/sq_$tag/sq_counter_collection.csv --before profiles/encdec_valu_r02.json \
  -o "$out/encdec_valu.json" > /dev/null
