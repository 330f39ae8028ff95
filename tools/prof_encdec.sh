#!/bin/bash
# Encrypt/decrypt kernel profile of one cfg3 learner (tools/encdec_prof.py): VALU issue
# rates, kernel stats, FETCH_SIZE and WRITE_SIZE passes -> gpurun_out/prof1/
set -e
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof1
hipcc -O3 --offload-arch=gfx950 -o /tmp/valu_rates tools/valu_rates.hip
timeout -k 10 120 /tmp/valu_rates > gpurun_out/prof1/valu_rates.txt 2>&1
timeout -k 10 120 python tools/encdec_prof.py 714 5 > gpurun_out/prof1/encdec.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof1 -o encdec -- /usr/bin/python3 tools/encdec_prof.py 714 3 > gpurun_out/prof1/encdec_prof.txt 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/prof1 -o fetch -- /usr/bin/python3 tools/encdec_prof.py 714 1 > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/prof1 -o write -- /usr/bin/python3 tools/encdec_prof.py 714 1 > /dev/null 2>&1
ls -R gpurun_out/prof1 | head -30
