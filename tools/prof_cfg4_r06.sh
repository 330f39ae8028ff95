# Round 6: per-kernel times of cfg4's (2^16 / L6) device encrypt / decrypt at K = 32 (bench's cfg4 learner)
# and K = 256: bash tools/prof_cfg4_r06.sh [tag]
set -e
cd /root/repo
export TMPDIR=/tmp
T=${1:-p4}
BATCH=32768 DEPTH=5 timeout -k 10 120 python tools/encdec_prof.py 32 20 > gpurun_out/${T}_k32_plain.txt 2>&1
BATCH=32768 DEPTH=5 timeout -k 10 120 python tools/encdec_prof.py 256 10 > gpurun_out/${T}_k256_plain.txt 2>&1
BATCH=32768 DEPTH=5 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}k32 -o run -- python tools/encdec_prof.py 32 20 > gpurun_out/${T}_k32_prof.txt 2>&1
BATCH=32768 DEPTH=5 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}k256 -o run -- python tools/encdec_prof.py 256 10 > gpurun_out/${T}_k256_prof.txt 2>&1
