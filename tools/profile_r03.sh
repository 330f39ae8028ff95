#!/bin/bash
# Round profile set in one call (on the GPU box): tools/profile_r02.sh TAG (the default bench under
# rocprofv3 --kernel-trace --stats, FETCH_SIZE / WRITE_SIZE passes for wavg and the encrypt/decrypt
# chains, one SQ pass), then the cfg2/4/5 bench lines and tools/profile_f4.sh TAG.
#   tools/profile_r03.sh r03b   -> gpurun_out/profile_r03b/, gpurun_out/f4_r03b/
set -euo pipefail
tag=${1:?round tag}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/profile_r02.sh "$tag"
out=gpurun_out/profile_$tag
for w in cfg2 cfg4 cfg5; do
  timeout -k 10 300 python3 bench.py --workload "$w" --no-cpu-baseline > "$out/${tag}_bench_$w.json" 2> "$out/${tag}_bench_$w.err"
done
bash tools/profile_f4.sh "$tag"
echo "profile set $tag done"
