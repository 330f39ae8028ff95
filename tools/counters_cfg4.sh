#!/bin/bash
# Round 6: the encrypt / decrypt chains' counters at cfg4 (2^16 / L6, K = 32 = bench's
# cfg4 learner): FETCH_SIZE and WRITE_SIZE passes -> encdec_traffic_cfg4.json (algorithmic bytes per ct:
# 2 L N 8 + S 8 = 6,553,600), one SQ pass -> encdec_valu_cfg4.json, the GRBM clock pass ->
# encdec_clock_cfg4.json, all in gpurun_out/cnt_cfg4/ (copied to profiles/ for bench.py --workload cfg4).
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/cnt_cfg4
mkdir -p "$out"
export BATCH=32768 DEPTH=5
K=32
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$out" -o efetch \
  -- /usr/bin/python3 tools/encdec_prof.py $K 1 > /dev/null 2> "$out/efetch.err"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$out" -o ewrite \
  -- /usr/bin/python3 tools/encdec_prof.py $K 1 > /dev/null 2> "$out/ewrite.err"
python3 tools/encdec_traffic.py "$out/efetch_counter_collection.csv" "$out/ewrite_counter_collection.csv" \
  --cts $K --bytes-per-ct 6553600 -o "$out/encdec_traffic_cfg4.json" > /dev/null
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY \
  SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-trace --output-format csv -d "$out" -o sq \
  -- /usr/bin/python3 tools/encdec_prof.py $K 1 > /dev/null 2> "$out/sq.err"
python3 tools/sq_table.py "$out/sq_counter_collection.csv" > "$out/sq_summary.txt" || true
python3 tools/encdec_valu.py "$out/sq_counter_collection.csv" --cts $K -o "$out/encdec_valu_cfg4.json" > /dev/null
timeout -s KILL 180 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d "$out/clock" -o clock \
  -- /usr/bin/python3 tools/encdec_prof.py $K 9 > "$out/clock.txt" 2>&1
python3 tools/grbm_clock.py "$out/clock" -o "$out/encdec_clock_cfg4.json" > "$out/clock_summary.txt" 2>&1
echo "cfg4 counters done"
