#!/bin/bash
# Round 5: bytes-API chunk per learner for the cfg2 (16 x 4) and cfg5 (8 x 64) shapes through the ring
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r05v}
mkdir -p $out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
run 400 python -u tools/bytes_api_cold.py --learners 16 --k 4 --rounds 6 base SHELFI_WAVG_CHUNK_MIB=32 SHELFI_WAVG_CHUNK_MIB=64 > $out/cfg2.json 2> $out/cfg2.err
tail -1 $out/cfg2.json
run 400 python -u tools/bytes_api_cold.py --learners 8 --k 64 --rounds 4 base SHELFI_WAVG_CHUNK_MIB=112 SHELFI_WAVG_CHUNK_MIB=64 SHELFI_WAVG_CHUNK_MIB=112,SHELFI_STAGE_SLOT_MIB=32 > $out/cfg5.json 2> $out/cfg5.err
tail -1 $out/cfg5.json
echo probe_r05v done
