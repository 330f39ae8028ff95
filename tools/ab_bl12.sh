# Round 6: cfg4 (2^16 / L6) encrypt / decrypt with 2^11 (default) vs 2^12 blocks, K = 32 and 256, plus
# (The SHELFI_ENC_BL12 / SHELFI_DEC_BL12 / SHELFI_DEC_XC switches and the SHELFI_ENC_X5=2 build were removed after these A/Bs: profiles/r06b.)
# kernel stats of the 2^12 form: bash tools/ab_bl12.sh [tag]
set -e
cd /root/repo
export TMPDIR=/tmp
T=${1:-bl12}
for K in 32 256; do
  for v in 0 1; do
    SHELFI_ENC_BL12=$v SHELFI_DEC_BL12=$v BATCH=32768 DEPTH=5 timeout -k 10 120 python tools/encdec_prof.py $K 20 \
      > gpurun_out/${T}_k${K}_bl12_$v.txt 2>&1
  done
done
SHELFI_ENC_BL12=1 SHELFI_DEC_BL12=1 BATCH=32768 DEPTH=5 timeout -k 10 180 rocprofv3 --kernel-trace --stats \
  --output-format csv -d gpurun_out/${T}k256 -o run -- python tools/encdec_prof.py 256 10 > gpurun_out/${T}_k256_prof.txt 2>&1
