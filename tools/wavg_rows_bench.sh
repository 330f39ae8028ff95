#!/bin/bash
# wavg rows-per-block A/B through bench.py itself (one process per run, same box): for each
# workload, SHELFI_WAVG_ROWS = each variant, alternating over two rounds; prints the
# roofline fraction of every run.  usage: tools/wavg_rows_bench.sh "cfg3 cfg5 cfg2" "1 2 4"
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/wavg_rows_bench
B="--steps 100 --warmup 3 --no-cpu-baseline --api-cts 0 --no-check --f4-cts 0 --no-alt"
for rnd in 1 2; do
  for wl in $1; do
    vs="$2"
    [ "$rnd" = 2 ] && vs=$(echo "$2" | tr ' ' '\n' | tac | tr '\n' ' ')
    for r in $vs; do
      SHELFI_WAVG_ROWS=$r timeout -k 10 120 python3 bench.py --workload "$wl" $B \
        > "gpurun_out/wavg_rows_bench/${wl}_R${r}_${rnd}.json" 2> "gpurun_out/wavg_rows_bench/${wl}_R${r}_${rnd}.err"
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'R=%s' % sys.argv[3], 'round', sys.argv[4], d['roofline']['frac'], d['ms_per_step'])" \
        "gpurun_out/wavg_rows_bench/${wl}_R${r}_${rnd}.json" "$wl" "$r" "$rnd"
    done
  done
done
