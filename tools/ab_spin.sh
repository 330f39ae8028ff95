# Round 6: the device API's end-of-call wait blocking (hipStreamSynchronize) vs polling hipStreamQuery
# (SHELFI_SPIN_SYNC=1), cfg2 K = 4, cfg4 K = 32, cfg3 K = 714, alternated twice
# Measured 2026-10-18 (profiles/r06b/spin_*.txt) and removed: polling was slower at K = 4 (encrypt 17.1-17.4 -> 17.8-18.3 us/ct, decrypt 10.3-10.4 -> 11.0-11.4) and at cfg4 K = 32, noise at K = 714
set -e
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-spin}
for rep in 0 1; do
  for sp in 0 1; do
    SHELFI_SPIN_SYNC=$sp timeout -k 10 120 python tools/encdec_prof.py 4 200 > gpurun_out/${T}_k4_s${sp}_r$rep.txt 2>&1
    SHELFI_SPIN_SYNC=$sp BATCH=32768 DEPTH=5 timeout -k 10 120 python tools/encdec_prof.py 32 50 > gpurun_out/${T}_k32_s${sp}_r$rep.txt 2>&1
    SHELFI_SPIN_SYNC=$sp timeout -k 10 120 python tools/encdec_prof.py 714 10 > gpurun_out/${T}_k714_s${sp}_r$rep.txt 2>&1
  done
done
