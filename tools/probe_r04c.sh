#!/bin/bash
# Round 4: is the flooded decrypt's gap in bench.py a clock effect?  Effective clock per decrypt
# kernel (GRBM_GUI_ACTIVE / 8 / wall) for exact and flooded calls, alternated and in bench.py's block
# order -> gpurun_out/r04c/
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04c
mkdir -p $out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
ORDER=block run 200 python tools/dec_flood_ab.py 714 7 > $out/dec_flood_block.txt 2>&1
cat $out/dec_flood_block.txt
run 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $out/alt -o alt -- /usr/bin/python3 tools/dec_flood_ab.py 714 6 > $out/alt.txt 2>&1
python tools/grbm_clock.py $out/alt > $out/clock_alt.txt 2>&1; tail -12 $out/clock_alt.txt
ORDER=block run 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $out/block -o block -- /usr/bin/python3 tools/dec_flood_ab.py 714 6 > $out/block.txt 2>&1
python tools/grbm_clock.py $out/block > $out/clock_block.txt 2>&1; tail -12 $out/clock_block.txt
echo probe_r04c done
