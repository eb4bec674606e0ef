#!/bin/bash
# A/B of liboctpt builds on the GPU box: scripts/ab.sh "CONFIG:SPP ..." LIB...  (LIB = path or "cur")
# Each config runs in one process per library, interleaved twice; prints Mrays/s lines.
set -o pipefail
CFGS=$1; shift
for rep in 1 2; do
  for cs in $CFGS; do
    c=${cs%%:*}; spp=${cs##*:}
    for lib in "$@"; do
      if [ "$lib" = cur ]; then unset OCTPT_LIB; else export OCTPT_LIB=$lib; fi
      echo "== $c $spp $lib"
      timeout -k 10 300 python scripts/spp_sweep.py $c $spp $spp --ktime 2>&1 | grep spp | tail -1 || exit 1
    done
  done
done
