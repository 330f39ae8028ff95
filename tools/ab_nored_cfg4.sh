# Round 6: encrypt's NORED tower split (default from K = 192) vs one reduced blocks pass (SHELFI_ENC_NORED=0)
# at 2^16 / L6 (K = 256, 512) and 2^15 / L4 (K = 714); alternated three times
set -e
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-nr}
for rep in 0 1 2; do
  for v in 1 0; do
    for K in 256 512; do
      SHELFI_ENC_NORED=$v BATCH=32768 DEPTH=5 timeout -k 10 120 python tools/encdec_prof.py $K 7 > gpurun_out/${T}_c4_k${K}_n${v}_r$rep.txt 2>&1
    done
    SHELFI_ENC_NORED=$v timeout -k 10 120 python tools/encdec_prof.py 714 7 > gpurun_out/${T}_c3_k714_n${v}_r$rep.txt 2>&1
  done
done
