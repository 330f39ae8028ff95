# Round 6: device encrypt/decrypt launch chains cut to SHELFI_DEV_CHUNK_MIB of scratch (is a chunk's
# dbuf / pbuf round trip served by the 256 MiB Infinity Cache?), cfg3 K = 714, alternated twice
# Measured 2026-10-18 (profiles/r06b/chunk_*.txt): every cut is slower (cfg3 K = 714 encrypt 2.80 -> 3.32 / 3.88 / 4.33 / 5.59 us/ct, decrypt 0.99 -> 0.99 / 1.07 / 1.16 / 1.30 at 256 / 128 / 96 / 64 MiB)
set -e
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-chunk}
for rep in 0 1; do
  for m in 4096 256 128 96 64; do
    SHELFI_DEV_CHUNK_MIB=$m timeout -k 10 120 python tools/encdec_prof.py 714 5 > gpurun_out/${T}_m${m}_r$rep.txt 2>&1
  done
done
