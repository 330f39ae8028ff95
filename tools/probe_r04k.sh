#!/bin/bash
# Round 4: the N > 1 bench path on one GPU (torch.distributed.run world 1, RCCL): the learner-sharded
# combine with both exchanges (headline + alternative_exchange), the C-ABI combine with the packed
# exchange, then the GPU suite -> gpurun_out/r04k/
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/r04k
mkdir -p $out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; if [ $rc -ne 0 ]; then echo "step failed rc=$rc: $*"; exit $rc; fi; }
T="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 1 --force-dist"
run 400 $T --steps 20 --warmup 2 --no-cpu-baseline --api-cts 0 --f4-cts 0 > $out/dist1_sum.json 2> $out/dist1_sum.err
run 400 $T --steps 20 --warmup 2 --no-cpu-baseline --api-cts 0 --f4-cts 0 --combine shelfi --exchange packed > $out/dist1_shelfi_packed.json 2> $out/dist1_shelfi_packed.err
for f in $out/dist1_*.json; do
  python -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['config'].get('parallelism'), d['config'].get('exchange'), json.dumps(d.get('alternative_exchange'))[:300], json.dumps(d.get('alternative_partitioning'))[:200], d.get('check'))"
done
#run 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $out/gpu_tests.log 2>&1
#tail -2
echo probe_r04k done
