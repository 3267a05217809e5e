#!/bin/bash
# Cache-policy A/B of the WCT variants built by build_variant.sh (w<mask>): C4 at 512 and 64
# pairs, one process per library, alternating.   bash scripts/debug/nt_ab.sh ROUNDS LIB...
set -u
rounds=$1; shift
for r in $(seq 1 "$rounds"); do
  for lib in "$@"; do
    WTMI_LIB_PATH=$lib timeout -k 10 120 python scripts/debug/c4_sizes.py r$r 512 64 || exit 1
  done
done
