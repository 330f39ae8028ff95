#!/bin/bash
# Library A/B across processes (round 5): this tree's libshelfi.so vs fhe-fed_amd/SHELFI_FHE/ab/libshelfi_base.so
# (another build, SHELFI_LIB_AB), alternated 3 times, each a tools/switch_ab.py 'base' run (us per ct,
# encrypt / decrypt / flooded at K = 714).  Output lines: "<which> <json>".
#   bash tools/lib_ab.sh > out.txt
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in 1 2 3; do
  for which in base new; do
    if [ $which = base ]; then
      r=$(SHELFI_LIB_AB=$PWD/fhe-fed_amd/SHELFI_FHE/ab/libshelfi_base.so timeout -k 10 200 python -u tools/switch_ab.py --rounds 5 base 2>/dev/null | tail -1) || exit 1
    else
      r=$(timeout -k 10 200 python -u tools/switch_ab.py --rounds 5 base 2>/dev/null | tail -1) || exit 1
    fi
    echo "$which $r"
  done
done
