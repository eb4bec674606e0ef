#!/bin/bash
# Usage (GPU box, repo root): scripts/gpu_pmc_write.sh TAG "CFG ..." LIB...  (LIB = cur or a variant .so)
# One rocprofv3 --pmc pass (COUNTERS: passes separated by spaces, counters of one pass by +; default
# WRITE_SIZE) per (config, library) over a one-step bench (no issued probe,
# no CPU baseline), each under its own time limit; summarised by scripts/pmc_write_summary.py.
set -o pipefail
TAG=$1; CFGS=$2; shift 2
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
export TMPDIR=/tmp
for c in $CFGS; do
  for lib in "$@"; do
    if [ "$lib" = cur ]; then unset OCTPT_LIB; name=cur; else export OCTPT_LIB=$R/$lib; name=$(basename $(dirname $lib)); fi
    for ctr in ${COUNTERS:-WRITE_SIZE}; do
      d=$OUT/${c}_${name}_${ctr}
      timeout -s KILL 240 rocprofv3 --pmc ${ctr//+/ } -d $d -o run -- python3 bench.py --config $c --steps 1 --warmup 0 \
        --no-cpu-baseline --no-issued ${BENCH_ARGS} > $d.json 2> $d.err || { tail -20 $d.err; exit 1; }
      echo "$c $name $ctr done"
    done
  done
done
python3 scripts/pmc_write_summary.py $OUT
