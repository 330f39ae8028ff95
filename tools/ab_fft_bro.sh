# Round 6: the whole-vector encode FFT writing its output bit-reversed (default) so enc_cols_fused reads it
# Measured 2026-10-18 and removed (profiles/r06f/bro/): bit-reversed stores slowed fft_inv_whole 122.7 -> 225.6 us per 714 cts and enc_cols_fused 475 -> 536 us; encrypt 2.76-2.81 -> 2.96-3.08 us/ct (K = 714), 3.10-3.18 -> 3.33 (K = 256)
# contiguously, vs natural order (SHELFI_FFT_BRO=0): cfg3 K = 714 and K = 256, alternated three times, then
# kernel stats of one run each
set -e
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=${1:-bro}
for rep in 0 1 2; do
  for v in 1 0; do
    SHELFI_FFT_BRO=$v timeout -k 10 120 python tools/encdec_prof.py 714 7 > gpurun_out/${T}_k714_b${v}_r$rep.txt 2>&1
    SHELFI_FFT_BRO=$v timeout -k 10 120 python tools/encdec_prof.py 256 9 > gpurun_out/${T}_k256_b${v}_r$rep.txt 2>&1
  done
done
for v in 1 0; do
  SHELFI_FFT_BRO=$v timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof$v -o p \
    -- /usr/bin/python3 tools/encdec_prof.py 714 3 > /dev/null 2>&1
done
