#!/bin/bash
# Multi-GPU launch recipe for bench.py on ONE node (the driver's SCALE protocol):
# torch.distributed.run starts one child process per GPU (no exec after GPU init).
#   tools/scale_recipe.sh 8                      # headline: learner-sharded + pipelined RCCL reduce_scatter
#   tools/scale_recipe.sh 8 --combine shelfi     # the same pipelined combine inside libshelfi (C ABI)
#   tools/scale_recipe.sh 8 --shard cts          # ciphertext-sharded, no collective
# The default run also cross-checks the C-ABI communicator (c_abi_comm_check in the JSON).
set -euo pipefail
N=${1:-8}
shift || true
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd "$(dirname "$0")/.."
exec python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 \
    --master-port "${MASTER_PORT:-29533}" bench.py --gpus "$N" "$@"
