# Round 6: a library variant (SHELFI_LIB_AB=path, built by hand into build_ab/) against the in-tree build,
# encdec_prof alternated three times: tools/ab_lib.sh TAG path K [BATCH DEPTH]
set -e
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=$1; V=$2; K=${3:-714}
export BATCH=${4:-16384} DEPTH=${5:-3}
for rep in 0 1 2; do
  timeout -k 10 120 python tools/encdec_prof.py $K 7 > gpurun_out/${T}_base_r$rep.txt 2>&1
  SHELFI_LIB_AB=$V timeout -k 10 120 python tools/encdec_prof.py $K 7 > gpurun_out/${T}_var_r$rep.txt 2>&1
done
