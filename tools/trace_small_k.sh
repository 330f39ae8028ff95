# Round 6: kernel timeline of small device encrypt / decrypt calls (cfg2's K = 4 per learner at 2^15 / L4,
# cfg4's K = 32 at 2^16 / L6): where a small call's time goes between kernels.  bash tools/trace_small_k.sh [tag]
set -e
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-sk}
timeout -k 10 120 python tools/encdec_prof.py 4 20 > gpurun_out/${T}_k4_plain.txt 2>&1
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/${T}k4 -o run \
  -- /usr/bin/python3 tools/encdec_prof.py 4 20 > gpurun_out/${T}_k4_prof.txt 2>&1
