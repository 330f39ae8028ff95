#!/bin/bash
# A/B of a launch-time switch on the cfg3 encrypt/decrypt timings (tools/encdec_prof.py):
#   tools/ab_encdec.sh VAR VAL1 VAL2 [VAL3 ...]   (alternated 3 times, one process each)
set -euo pipefail
var=$1; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in 1 2 3; do
  for v in "$@"; do
    echo -n "$var=$v  "
    env "$var=$v" timeout -k 10 120 python tools/encdec_prof.py 714 5 2>/dev/null
  done
done
