#!/bin/bash
# Round 4 first probe set (one gpurun call): GPU test suite, then the A/Bs of this round's kernel
# changes -> gpurun_out/r04a/
#   wavg_packed: round 3's four-accumulator kernel vs the three-accumulator / LDS-running-sum one,
#                and the new kernel's learner unroll depth (tools/wavg_packed_ab.py);
#   FFT LDS swizzle: SHELFI_FFT_SWZ=0 vs 1 for encrypt and the flooded decrypt (enc_variant_probe.py);
#   encrypt / decrypt / flooded decrypt us per ciphertext (tools/encdec_prof.py).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04a
mkdir -p $out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
run 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $out/gpu_tests.log 2>&1
tail -3 $out/gpu_tests.log
AB_ENV=SHELFI_PACK_KERNEL AB_VARIANTS=r3,v4 run 300 python tools/wavg_packed_ab.py 7 20 > $out/wavg_kernel_ab.txt 2>&1
cat $out/wavg_kernel_ab.txt
AB_ENV=SHELFI_PACK_UNROLL AB_VARIANTS=1,2,4,8 AB_SHAPES=cfg2,cfg5,cfg3 run 300 python tools/wavg_packed_ab.py 5 20 > $out/wavg_unroll_ab.txt 2>&1
cat $out/wavg_unroll_ab.txt
VAR=SHELFI_FFT_SWZ VALS=0,1 K=714 run 300 python tools/enc_variant_probe.py > $out/fft_swz_ab.txt 2>&1
VAR=SHELFI_FFT_SWZ VALS=0,1 K=714 FLOOD=1 run 300 python tools/enc_variant_probe.py >> $out/fft_swz_ab.txt 2>&1
cat $out/fft_swz_ab.txt
run 200 python tools/encdec_prof.py 714 5 > $out/encdec.txt 2>&1
cat $out/encdec.txt
echo probe_r04a done
