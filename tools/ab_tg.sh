# Round 6: enc_cols_fused with its towers split over 1 / 2 / 3 workgroup groups (SHELFI_ENC_TG), cfg4 K = 32 / 256
# Measured 2026-10-18 (profiles/r06b/tg_*.txt) and removed: tg 2/3 slower at every K (cfg4 K=32 encrypt 10.84 -> 11.47/11.70 us/ct, K=256 9.01 -> 9.30/9.80, cfg3 K=714 2.92 -> 3.16) -- each group re-samples the ChaCha stream and re-reads the message
set -e
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-tg}
for K in 32 256; do
  for g in 1 2 3; do
    SHELFI_ENC_TG=$g BATCH=32768 DEPTH=5 timeout -k 10 120 python tools/encdec_prof.py $K 20 > gpurun_out/${T}_k${K}_tg$g.txt 2>&1
  done
done
for g in 1 2; do
  SHELFI_ENC_TG=$g timeout -k 10 120 python tools/encdec_prof.py 714 5 > gpurun_out/${T}_cfg3_tg$g.txt 2>&1
done
