#!/bin/bash
# Profile the default bench command (the one the driver runs) under rocprofv3 and
# keep the bench JSON line and the kernel statistics of that same process.
#   tools/profile_round.sh r01        (on the GPU box; writes gpurun_out/profile_r01/)
set -euo pipefail
tag=${1:?round tag, e.g. r01}
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/profile_$tag
mkdir -p "$out"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o "$tag" \
  -- /usr/bin/python3 bench.py > "$out/${tag}_bench.json" 2> "$out/${tag}_bench.err"
