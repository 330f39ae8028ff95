#!/bin/bash
# Round 5: staged-upload fill threads (the pageable -> pinned copies compete with the DMA reading pinned memory)
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r05r}
mkdir -p $out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
# the Stager reads SHELFI_H2D_COPY_THREADS when it is created: a different slot size re-creates it
run 500 python -u tools/bytes_api_cold.py --wire palisade --rounds 4 base SHELFI_STAGE_SLOT_MIB=17,SHELFI_H2D_COPY_THREADS=2 SHELFI_STAGE_SLOT_MIB=18,SHELFI_H2D_COPY_THREADS=3 SHELFI_STAGE_SLOT_MIB=19,SHELFI_H2D_COPY_THREADS=6 SHELFI_STAGE_SLOT_MIB=20,SHELFI_H2D_COPY_THREADS=8 SHELFI_STAGE_SLOT_MIB=32 > $out/cold_threads.json 2> $out/cold_threads.err
tail -1 $out/cold_threads.json
SHELFI_STAGE_TRACE=1 run 200 python -u tools/bytes_api_cold.py --rounds 1 base > $out/trace.json 2> $out/trace.err
grep wavg-bytes $out/trace.err | head -3
grep "in 2" $out/trace.err | head -3
echo probe_r05r done
