#!/bin/bash
# Round 4: VALU issue rates of more instruction forms, and the effective clock per encrypt/decrypt
# kernel in the steady-state loop (714-ct calls, and 90-ct chunks whose pbuf stays in the LLC)
# -> gpurun_out/r04h/
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04h
mkdir -p $out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
run 120 tools/valu_rates2 > $out/valu_rates2.txt 2>&1
cat $out/valu_rates2.txt
run 180 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $out/steady -o steady -- /usr/bin/python3 tools/encdec_prof.py 714 9 > $out/steady.txt 2>&1
grep "us/ct" $out/steady.txt
python3 tools/grbm_clock.py $out/steady -o $out/encdec_clock.json > $out/clock_steady.txt 2>&1; grep -A8 "median encrypt" $out/clock_steady.txt
SHELFI_DEV_CHUNK_MIB=280 run 180 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $out/chunk90 -o chunk90 -- /usr/bin/python3 tools/encdec_prof.py 714 9 > $out/chunk90.txt 2>&1
grep "us/ct" $out/chunk90.txt
python3 tools/grbm_clock.py $out/chunk90 -o $out/encdec_clock_chunk90.json > $out/clock_chunk90.txt 2>&1; grep -A8 "median encrypt" $out/clock_chunk90.txt
echo probe_r04h done
