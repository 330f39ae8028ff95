# Round 6: the persistent block passes (default) vs the one-shot ones (SHELFI_DEC_PP=0, SHELFI_ENC_PP=0) at
# small batches: cfg4 K = 32 (bench's cfg4 learner), cfg2 K = 4, cfg3 K = 64; alternated twice
set -e
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-ppk}
for rep in 0 1; do
  for v in 1 0; do
    SHELFI_DEC_PP=$v SHELFI_ENC_PP=$v BATCH=32768 DEPTH=5 timeout -k 10 120 python tools/encdec_prof.py 32 40 > gpurun_out/${T}_k32_pp${v}_r$rep.txt 2>&1
    SHELFI_DEC_PP=$v SHELFI_ENC_PP=$v timeout -k 10 120 python tools/encdec_prof.py 4 100 > gpurun_out/${T}_k4_pp${v}_r$rep.txt 2>&1
    SHELFI_DEC_PP=$v SHELFI_ENC_PP=$v timeout -k 10 120 python tools/encdec_prof.py 64 20 > gpurun_out/${T}_k64_pp${v}_r$rep.txt 2>&1
  done
done
