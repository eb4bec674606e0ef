#!/bin/bash
# Extend-variant sweep on the GPU box: $CONFIG (default C3) at $SPP (default 64) spp per setting (env assignments as arguments,
# one setting per argument, fields separated by commas), one JSON line each into $OUT.
# Usage: scripts/extend_sweep.sh OUT "OCTPT_EXTEND=spec,OCTPT_SPEC_BATCH=16" ...
OUT=$1; shift
for setting in "$@"; do
  envs=$(echo "$setting" | tr ',' ' ')
  line=$(env $envs timeout -k 10 120 python3 bench.py --no-cpu-baseline --config ${CONFIG:-C3} --spp ${SPP:-64} --steps 3 --warmup 1 2>/dev/null) || exit $?
  python3 -c "import json,sys; d=json.loads(sys.argv[2]); r=d['roofline']; print(json.dumps({'setting': sys.argv[1], 'mrays': d['value'], 'extend_ms': r['kernel_ms_avg'], 'shade_ms': r['shade']['kernel_ms_avg'], 'ms_per_step': d['ms_per_step']}))" "$setting" "$line" >> $OUT
  tail -1 $OUT
done
