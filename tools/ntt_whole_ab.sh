# Round 6: whole-polynomial NTT probe vs the two-pass NTT, timed (events), then one
# kernel-trace --stats run and one SQ counter pass over the same script (1 rep), into gpurun_out/nw/
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/nw
mkdir -p "$out"
timeout -k 10 180 python tools/ntt_whole_ab.py 714 7 > "$out/ab.json" 2> "$out/ab.err"
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o kt \
  -- /usr/bin/python3 tools/ntt_whole_ab.py 714 2 > "$out/kt.json" 2> "$out/kt.err"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY \
  SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d "$out" -o sq \
  -- /usr/bin/python3 tools/ntt_whole_ab.py 714 1 > /dev/null 2> "$out/sq.err"
python3 tools/sq_table.py "$out/sq_counter_collection.csv" > "$out/sq_summary.txt" || true
echo done
