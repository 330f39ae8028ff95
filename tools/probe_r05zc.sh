#!/bin/bash
# Round 5: small-batch encrypt / decrypt (cfg2's 4 cts per learner): whole-vector FFTs vs the multi-pass FFTs
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r05zc}
mkdir -p $out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
for k in 4 16 64 256; do
  for fw in 1 0; do
    SHELFI_FFT_WHOLE=$fw run 120 python tools/encdec_prof.py $k 21 > $out/k${k}_w$fw.txt 2>&1
    echo "K=$k FFT_WHOLE=$fw $(tail -1 $out/k${k}_w$fw.txt)" >> $out/small_k.txt
  done
done
cat $out/small_k.txt
SHELFI_FFT_WHOLE=1 run 120 rocprofv3 --kernel-trace --stats -d $out/prof1 -o k4 -- /usr/bin/python3 tools/encdec_prof.py 4 21 > $out/prof1.txt 2>&1
SHELFI_FFT_WHOLE=0 run 120 rocprofv3 --kernel-trace --stats -d $out/prof0 -o k4 -- /usr/bin/python3 tools/encdec_prof.py 4 21 > $out/prof0.txt 2>&1
echo probe_r05zc done
