# Round 6: cfg4 encrypt with the X5 columns kernel: persistent blocks pass split in NORED / reduced launches
# (default), one reduced persistent launch (SHELFI_ENC_NORED=0), the one-shot pass (SHELFI_ENC_PP=0); K = 32, 256
set -e
cd /root/repo
export TMPDIR=/tmp
T=${1:-x5pp}
for K in 32 256; do
  BATCH=32768 DEPTH=5 timeout -k 10 120 python tools/encdec_prof.py $K 20 > gpurun_out/${T}_k${K}_def.txt 2>&1
  SHELFI_ENC_NORED=0 BATCH=32768 DEPTH=5 timeout -k 10 120 python tools/encdec_prof.py $K 20 > gpurun_out/${T}_k${K}_nored0.txt 2>&1
  SHELFI_ENC_PP=0 BATCH=32768 DEPTH=5 timeout -k 10 120 python tools/encdec_prof.py $K 20 > gpurun_out/${T}_k${K}_pp0.txt 2>&1
done
