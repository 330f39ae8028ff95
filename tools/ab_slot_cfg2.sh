# Round 6: the bytes-API aggregation's ring slot size at the cfg2 shape (16 x 4 archives, 134 MB per call):
# 8 / 16 (default) / 32 MiB slots, alternated three times (tools/bytes_api_overhead.py --cts 4, warm blobs)
set -e
# Measured 2026-10-18 (profiles/r06f/slot2_*): no size wins beyond the +-4% noise (16 MiB 43.2 / 43.1 / 39.8 GB/s, 32 MiB 43.5 / 41.1 / 41.8, 8 MiB 40.9 / 40.5 / 42.0)
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-slot2}
for rep in 0 1 2; do
  for m in 16 32 8; do
    SHELFI_STAGE_SLOT_MIB=$m timeout -k 10 120 python tools/bytes_api_overhead.py --cts 4 > gpurun_out/${T}_m${m}_r$rep.json 2>&1
  done
done
