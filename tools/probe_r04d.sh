#!/bin/bash
# Round 4: GPU suite, then bench cfg3 + the wavg kernel A/B with multi-switch variants and the
# decrypt host-overhead change (this tree vs the round-start library) -> gpurun_out/r04d/
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04d
mkdir -p $out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
run 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $out/gpu_tests.log 2>&1
tail -2 $out/gpu_tests.log
AB_VARIANTS="SHELFI_PACK_KERNEL=r3,SHELFI_PACK_KERNEL=v4,SHELFI_PACK_KERNEL=v4+SHELFI_PACK_UNROLL=8" run 300 python tools/wavg_packed_ab.py 9 20 > $out/wavg_kernel_ab.txt 2>&1
cat $out/wavg_kernel_ab.txt
for i in 1 2; do
  echo "base:" >> $out/lib_ab.txt
  SHELFI_LIB_AB=$PWD/fhe-fed_amd/SHELFI_FHE/ab/libshelfi_base.so run 120 python tools/dec_flood_ab.py 714 8 >> $out/lib_ab.txt 2>&1
  echo "new:" >> $out/lib_ab.txt
  run 120 python tools/dec_flood_ab.py 714 8 >> $out/lib_ab.txt 2>&1
done
grep -v amdgpu.ids $out/lib_ab.txt
run 400 python bench.py > $out/bench_cfg3.json 2> $out/bench_cfg3.err
for w in cfg2 cfg5 cfg4; do
  run 300 python bench.py --workload $w --no-cpu-baseline --api-cts 0 --f4-cts 0 > $out/bench_$w.json 2> $out/bench_$w.err
  run 300 python bench.py --workload $w --layout separate --no-cpu-baseline --api-cts 0 --f4-cts 0 > $out/bench_${w}_separate.json 2> $out/bench_${w}_separate.err
done
for f in $out/bench_cfg*.json; do
  python -c "import json; d=json.load(open('$f')); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], r.get('frac'), r.get('arena_layout'), d.get('decrypt_decode_ms_per_ct'), d.get('decrypt_decode_flooded_ms_per_ct'), d.get('encode_encrypt_ms_per_ct'))"
done
echo probe_r04d done
