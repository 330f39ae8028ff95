#!/bin/bash
# Round 5: bytes-API upload settings alternated in one process, per NUMA binding -> gpurun_out/r05g/
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r05g
mkdir -p $out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
S="base SHELFI_H2D_DIRECT=0 SHELFI_WAVG_CHUNK_MIB=128 SHELFI_WAVG_CHUNK_MIB=1024"
for n in none local remote; do
  run 200 python -u tools/bytes_api_ab.py --numa $n $S >> $out/ab.jsonl 2> $out/ab_$n.err
done
run 200 python -u tools/bytes_api_ab.py --numa local --wire packed $S >> $out/ab.jsonl 2> $out/ab_packed.err
run 200 python -u tools/bytes_api_ab.py --numa local --wire shelfi $S >> $out/ab.jsonl 2> $out/ab_shelfi.err
cat $out/ab.jsonl
