# Round 6: device encrypt / decrypt per-call times at small K (cfg2's K = 4, cfg4's K = 32) and cfg3's K = 714
set -e
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-skt}
timeout -k 10 120 python tools/encdec_prof.py 4 50 > gpurun_out/${T}_k4.txt 2>&1
BATCH=32768 DEPTH=5 timeout -k 10 120 python tools/encdec_prof.py 32 20 > gpurun_out/${T}_k32_cfg4.txt 2>&1
timeout -k 10 120 python tools/encdec_prof.py 714 5 > gpurun_out/${T}_k714.txt 2>&1
