#!/bin/bash
# Round 4: where encrypt's wall time goes (kernel trace of steady 714-ct encrypts vs wall, host
# overhead probe) and the FFT passes' LDS bank conflicts after the swizzle -> gpurun_out/r04g/
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04g
mkdir -p $out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
run 120 python3 tools/enc_overhead_probe.py > $out/enc_overhead.txt 2>&1
grep -v amdgpu.ids $out/enc_overhead.txt
run 180 rocprofv3 --kernel-trace --stats --output-format csv -d $out/tl -o tl -- /usr/bin/python3 tools/encdec_prof.py 714 7 > $out/tl.txt 2>&1
grep "us/ct" $out/tl.txt
run 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --kernel-trace --output-format csv -d $out/lds -o lds -- /usr/bin/python3 tools/encdec_prof.py 714 1 > $out/lds.txt 2>&1
echo probe_r04g done
