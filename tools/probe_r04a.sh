#!/bin/bash
# Round 4 probe set (one gpurun call, after the GPU test suite): A/Bs of this round's kernel changes
# -> gpurun_out/r04a/
#   wavg_packed: round 3's four-accumulator kernel vs the three-accumulator / LDS-running-sum one
#                (SHELFI_PACK_KERNEL=r3 vs default), and the new kernel's learner unroll depth;
#   FFT LDS swizzle: SHELFI_FFT_SWZ=0 vs 1 (encrypt, and the flooded decrypt);
#   the fused forward butterfly: this tree's library vs the previous commit's
#     (fhe-fed_amd/SHELFI_FHE/ab/libshelfi_base.so via SHELFI_LIB_AB), alternating processes;
#   exact vs flooded decrypt alternated in one process (tools/dec_flood_ab.py).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04a
mkdir -p $out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
AB_ENV=SHELFI_PACK_KERNEL AB_VARIANTS=r3,v4 run 300 python tools/wavg_packed_ab.py 7 20 > $out/wavg_kernel_ab.txt 2>&1
cat $out/wavg_kernel_ab.txt
AB_ENV=SHELFI_PACK_UNROLL AB_VARIANTS=1,2,4,8 AB_SHAPES=cfg2,cfg5,cfg3,cfg4 run 300 python tools/wavg_packed_ab.py 5 20 > $out/wavg_unroll_ab.txt 2>&1
cat $out/wavg_unroll_ab.txt
AB_ENV=SHELFI_PACK_SPLIT AB_VARIANTS=1,2 run 300 python tools/wavg_packed_ab.py 7 20 > $out/wavg_split_ab.txt 2>&1
cat $out/wavg_split_ab.txt
VAR=SHELFI_FFT_SWZ VALS=0,1 K=714 run 200 python tools/enc_variant_probe.py > $out/fft_swz_ab.txt 2>&1
VAR=SHELFI_FFT_SWZ VALS=0,1 K=714 FLOOD=1 run 200 python tools/enc_variant_probe.py >> $out/fft_swz_ab.txt 2>&1
cat $out/fft_swz_ab.txt
for i in 1 2 3; do
  echo "base:" >> $out/bfly_lib_ab.txt
  SHELFI_LIB_AB=$PWD/fhe-fed_amd/SHELFI_FHE/ab/libshelfi_base.so run 120 python tools/encdec_prof.py 714 5 >> $out/bfly_lib_ab.txt 2>&1
  echo "new:" >> $out/bfly_lib_ab.txt
  run 120 python tools/encdec_prof.py 714 5 >> $out/bfly_lib_ab.txt 2>&1
done
grep -v amdgpu.ids $out/bfly_lib_ab.txt
run 200 python tools/dec_flood_ab.py 714 12 > $out/dec_flood_ab.txt 2>&1
cat $out/dec_flood_ab.txt
echo probe_r04a done
