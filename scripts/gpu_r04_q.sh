#!/bin/bash
# Round 4: PMC traffic of C5 and C5b at the bench's own workload (4K x 1024 spp, one step: the whole
# frame's launch mix), then the C5 / C5b bench lines that read it.
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-r04q}
bash $R/scripts/gpu_pmc_config.sh C5 1024 $T || exit 1
bash $R/scripts/gpu_pmc_config.sh C5b 1024 $T || exit 1
cd $R
for c in C5 C5b; do
  timeout -k 10 400 python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/$T/bench_full_$c.json 2> gpurun_out/$T/bench_full_$c.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/$T/bench_full_$c.json')); r=d['roofline']; print('$c', d['value'], r['frac'], r['traffic'], r['l2_hit_rate'], r['launches'])"
done
