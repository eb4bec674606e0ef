#!/bin/bash
# Usage (GPU box, repo root): scripts/gpu_bench_configs.sh TAG "CFG[:flags] ..." -- one bench line per config
# (flags: c = --compact), each under its own time limit, stopping at the first failure.
set -o pipefail
TAG=$1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
for spec in $2; do
  cfg=${spec%%:*}; fl=""; [ "$spec" != "$cfg" ] && fl=${spec#*:}
  extra=""; [[ "$fl" == *c* ]] && extra="--compact"
  name=$cfg${fl:+_$fl}
  timeout -k 10 500 python3 bench.py --config $cfg $extra --steps ${STEPS:-2} --warmup 1 ${BENCH_ARGS} > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { tail -20 $OUT/bench_$name.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/bench_$name.json')); r=d['roofline']; print('$name', d['value'], 'Mrays/s', d['ms_per_step'], 'ms', 'frac', r['frac'], 'issued', (r.get('issued') or {}).get('frac'), 'ext', r['launches'], r['kernel_ms_avg'], 'share', r['share_of_gpu_time'])"
done
