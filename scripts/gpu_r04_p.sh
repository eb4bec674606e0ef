#!/bin/bash
# Round 4 final profile: scripts/gpu_profile.sh (C3 PMC passes, bench, kernel trace + stats; FULL=1: the
# 4K C4 and C5 benches), then the C5b full-size bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
FULL=1 bash $R/scripts/gpu_profile.sh ${1:-r04p} || exit 1
cd $R
timeout -k 10 400 python3 bench.py --config C5b --steps 2 --warmup 1 > gpurun_out/${1:-r04p}/bench_full_C5b.json 2> gpurun_out/${1:-r04p}/bench_full_C5b.err || exit 1
for f in bench bench_full_C4 bench_full_C5 bench_full_C5b; do
  python3 -c "import json; d=json.load(open('gpurun_out/${1:-r04p}/$f.json')); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], r['frac'], (r.get('issued') or {}).get('frac'), r['launches'], r['kernel_ms_avg'], r['shade']['kernel_ms_avg'])"
done
