#!/bin/bash
# Round 5: the GPU suite, the bytes API per upload setting, and TCC counters of a slow and a fast
# (arena, output) placement pair -> gpurun_out/r05f/
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r05f
mkdir -p $out
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
run 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > $out/gpu_tests.log 2>&1
tail -1 $out/gpu_tests.log
run 300 python -u tools/bytes_api_probe.py > $out/bytes.log 2>&1
grep setting $out/bytes.log
run 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum --kernel-trace --output-format csv -d $out/pmc_rd -o rd -- /usr/bin/python3 tools/placement_pmc.py > $out/pmc_rd.txt 2>&1
run 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_WRREQ_STALL_sum --kernel-trace --output-format csv -d $out/pmc_wr -o wr -- /usr/bin/python3 tools/placement_pmc.py > $out/pmc_wr.txt 2>&1
grep candidate $out/pmc_rd.txt $out/pmc_wr.txt
echo probe_r05f done
