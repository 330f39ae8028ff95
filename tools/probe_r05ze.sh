#!/bin/bash
# Round 5: small-batch encrypt with one blocks-pass launch (SHELFI_ENC_NORED=0: every tower reduced) vs the
# NORED split's two launches
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r05ze}
mkdir -p $out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
for k in 4 16 64 128 256; do
  for nr in 1 0 1 0; do
    SHELFI_ENC_NORED=$nr run 120 python tools/encdec_prof.py $k 31 > $out/k${k}_nr$nr.txt 2>&1
    echo "K=$k ENC_NORED=$nr $(tail -1 $out/k${k}_nr$nr.txt)" >> $out/nored_k.txt
  done
done
cat $out/nored_k.txt
echo probe_r05ze done
