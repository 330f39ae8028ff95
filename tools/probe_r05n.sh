#!/bin/bash
# Round 5: pinned H2D rate by copy size (blit kernel or DMA engine?) and the staging ring's slot size
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:-r05n}
mkdir -p $out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
run 200 python -u tools/h2d_pinned_probe.py > $out/pinned.json 2> $out/pinned.err
cat $out/pinned.json
run 200 rocprofv3 --kernel-trace --stats -d $out/prof_pinned -o pinned -- python3 -u tools/h2d_pinned_probe.py > $out/pinned_prof.json 2> $out/pinned_prof.err
run 400 python -u tools/bytes_api_cold.py --wire palisade --rounds 4 base SHELFI_STAGE_SLOT_MIB=16 SHELFI_STAGE_SLOT_MIB=32 > $out/cold_slot.json 2> $out/cold_slot.err
tail -1 $out/cold_slot.json
echo probe_r05n done
