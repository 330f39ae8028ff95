# Round 6: cfg4 encrypt with the 32-row v tables (default: X5 + VT 2) vs v's columns in enc_cols_fused
# (The VT 2 path these runs measured -- 32-row v tables in the blocks pass -- was not kept: profiles/r06b/vt5_*.)
# (SHELFI_ENC_VT=0), K = 32 and 256, + kernel stats / traffic of the default: bash tools/ab_vt5.sh [tag]
set -e
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-vt5}
export BATCH=32768 DEPTH=5
for K in 32 256; do
  for v in 1 0; do
    SHELFI_ENC_VT=$v timeout -k 10 120 python tools/encdec_prof.py $K 20 > gpurun_out/${T}_k${K}_vt$v.txt 2>&1
  done
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}k256 -o run \
  -- /usr/bin/python3 tools/encdec_prof.py 256 10 > gpurun_out/${T}_k256_prof.txt 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/${T}_pmc -o efetch \
  -- /usr/bin/python3 tools/encdec_prof.py 32 1 > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/${T}_pmc -o ewrite \
  -- /usr/bin/python3 tools/encdec_prof.py 32 1 > /dev/null 2>&1
python3 tools/encdec_traffic.py gpurun_out/${T}_pmc/efetch_counter_collection.csv gpurun_out/${T}_pmc/ewrite_counter_collection.csv \
  --cts 32 --bytes-per-ct 6553600 -o gpurun_out/${T}_pmc/encdec_traffic_cfg4.json > /dev/null
