#!/bin/bash
# rocprofv3 kernel stats of one command: tools/prof_stats.sh TAG CMD...  ->
# gpurun_out/prof_TAG/ (+ a concise summary in gpurun_out/prof_TAG/summary.txt)
set -euo pipefail
tag=$1
shift
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/prof_$tag
mkdir -p "$out"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o "$tag" -- "$@" > "$out/stdout.txt" 2> "$out/stderr.txt"
python3 tools/kstat_summary.py "$out/${tag}_kernel_stats.csv" > "$out/summary.txt"
