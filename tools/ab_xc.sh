# Round 6: cfg4 decrypt's last pass: the lane-swapped-stage 16-row form (default) vs 32 register rows
# (The SHELFI_ENC_BL12 / SHELFI_DEC_BL12 / SHELFI_DEC_XC switches and the SHELFI_ENC_X5=2 build were removed after these A/Bs: profiles/r06b.)
# (SHELFI_DEC_XC=0), K = 32 and 256, + kernel stats of the default: bash tools/ab_xc.sh [tag]
set -e
cd /root/repo
export TMPDIR=/tmp
T=${1:-xc}
for K in 32 256; do
  for v in 1 0; do
    SHELFI_DEC_XC=$v BATCH=32768 DEPTH=5 timeout -k 10 120 python tools/encdec_prof.py $K 20 > gpurun_out/${T}_k${K}_xc$v.txt 2>&1
  done
done
BATCH=32768 DEPTH=5 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}k256 -o run \
  -- python tools/encdec_prof.py 256 10 > gpurun_out/${T}_k256_prof.txt 2>&1
