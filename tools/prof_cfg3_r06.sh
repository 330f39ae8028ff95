# Round 6: per-kernel times of cfg3's (2^15 / L4) device encrypt / decrypt at K = 714 (bench's cfg3 learner)
set -e
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-p3}
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}k714 -o run \
  -- /usr/bin/python3 tools/encdec_prof.py 714 10 > gpurun_out/${T}_k714_prof.txt 2>&1
