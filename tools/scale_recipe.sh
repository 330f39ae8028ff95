#!/bin/bash
# Multi-GPU launch recipe for bench.py on ONE node (the driver's SCALE protocol).
# Equivalent to a bare `python bench.py --gpus N ...`, which spawns the same
# torch.distributed.run itself (bench.py spawn_ranks: one child process per GPU, the parent
# never touches the GPU).
#   tools/scale_recipe.sh 8                      # headline: learner-sharded + pipelined RCCL reduce_scatter
#   tools/scale_recipe.sh 8 --combine shelfi     # the same pipelined combine inside libshelfi (C ABI)
#   tools/scale_recipe.sh 8 --shard cts          # ciphertext-sharded, no collective
#   tools/scale_recipe.sh 8 --comm-check         # + cross-check of the C-ABI communicator (opt-in)
set -euo pipefail
N=${1:-8}
shift || true
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd "$(dirname "$0")/.."
exec python -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" --master-addr 127.0.0.1 \
    --master-port "${MASTER_PORT:-29533}" bench.py --gpus "$N" "$@"
