# Round 6: cfg4 (2^16 / L6) encrypt: enc_prep + 3 column passes (X5=0) vs the exchanged-stage fused columns
# (The SHELFI_ENC_BL12 / SHELFI_DEC_BL12 / SHELFI_DEC_XC switches and the SHELFI_ENC_X5=2 build were removed after these A/Bs: profiles/r06b.)
# kernel at 3 (X5=1) / 2 (X5=2) waves per SIMD, K = 32 and 256; kernel stats of X5=1: bash tools/ab_x5.sh [tag]
set -e
cd /root/repo
export TMPDIR=/tmp
T=${1:-x5}
for K in 32 256; do
  for v in 0 1 2; do
    SHELFI_ENC_X5=$v BATCH=32768 DEPTH=5 timeout -k 10 120 python tools/encdec_prof.py $K 20 > gpurun_out/${T}_k${K}_x5_$v.txt 2>&1
  done
done
for v in 1 2; do
SHELFI_ENC_X5=$v BATCH=32768 DEPTH=5 timeout -k 10 180 rocprofv3 --kernel-trace --stats \
  --output-format csv -d gpurun_out/${T}k256_$v -o run -- python tools/encdec_prof.py 256 10 > gpurun_out/${T}_k256_prof_$v.txt 2>&1
done
