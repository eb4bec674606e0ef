#!/bin/bash
# A/B of liboctpt builds and env settings on the GPU box:
#   scripts/ab_env.sh "CONFIG:SPP ..." "LIB|ENV=V,ENV2=V ..." ...   (LIB = path or "cur")
# Each config runs in one process per variant, interleaved twice; prints Mrays/s lines.
set -o pipefail
CFGS=$1; shift
for rep in 1 2; do
  for cs in $CFGS; do
    c=${cs%%:*}; spp=${cs##*:}
    for var in "$@"; do
      lib=${var%%|*}; envs=${var#*|}; [ "$envs" = "$var" ] && envs=""
      echo "== $c $spp $var"
      ( if [ "$lib" != cur ]; then export OCTPT_LIB=$lib; fi
        for kv in ${envs//,/ }; do export "$kv"; done
        timeout -k 10 300 python scripts/spp_sweep.py $c $spp $spp --ktime 2>&1 | grep spp | tail -1 ) || exit 1
    done
  done
done
