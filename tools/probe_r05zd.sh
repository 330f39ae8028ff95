#!/bin/bash
# Round 5: whole-vector FFTs from K = 128 only (tests; the K crossover at 96 / 128 / 192)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r05zd}
mkdir -p $out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
run 600 python -u -m pytest tests/test_gpu_switches.py tests/test_gpu_decode_noise.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $out/tests.log 2>&1
tail -1 $out/tests.log
for k in 96 128 192; do
  for fw in 1 0; do
    SHELFI_FFT_WHOLE=$fw run 120 python tools/encdec_prof.py $k 21 > $out/k${k}_w$fw.txt 2>&1
    echo "K=$k FFT_WHOLE=$fw $(tail -1 $out/k${k}_w$fw.txt)" >> $out/small_k.txt
  done
done
cat $out/small_k.txt
echo probe_r05zd done
