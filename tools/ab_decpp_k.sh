# Round 6: decrypt's persistent first INTT pass (default) vs the one-shot pass (SHELFI_DEC_PP=0) over batch
# sizes, cfg3 shape (2^15 / L4) K = 96 .. 714 and cfg4 (2^16 / L6) K = 64 .. 256; alternated twice
set -e
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-dpk}
for rep in 0 1; do
  for v in 1 0; do
    for K in 96 128 192 256 384 714; do
      SHELFI_DEC_PP=$v timeout -k 10 120 python tools/encdec_prof.py $K 9 > gpurun_out/${T}_c3_k${K}_pp${v}_r$rep.txt 2>&1
    done
    for K in 64 128 256; do
      SHELFI_DEC_PP=$v BATCH=32768 DEPTH=5 timeout -k 10 120 python tools/encdec_prof.py $K 9 > gpurun_out/${T}_c4_k${K}_pp${v}_r$rep.txt 2>&1
    done
  done
done
