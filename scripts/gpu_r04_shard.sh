#!/bin/bash
# Round 4: where an 8-way shard's time goes: a kernel trace of scripts/shard_emulation.py
# (the full C3 frame, then every 1/8 shard, each rendered twice), summarised per render by
# scripts/timeline.py; then the shard emulation itself for the speed-up ceiling.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r04s}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 $R/scripts/shard_emulation.py --ns 1 8 \
    > $OUT/shard_trace.json 2> $OUT/shard_trace.err || { tail -20 $OUT/shard_trace.err; exit 1; }
T=$(find $OUT/trace -name '*kernel_trace.csv' | head -1)
python3 $R/scripts/timeline.py "$T" > $OUT/timeline.json || exit 1
python3 - $OUT/timeline.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for i, r in enumerate(d["per_render"]):
    print(i, r["wall_us"], "gaps", r["gaps_us"], "tail", r["tail_us"], {k: v for k, v in r["busy_us"].items()}, r["launches"])
PY
timeout -k 10 300 python3 $R/scripts/shard_emulation.py --config C3 --ns 1 2 4 8 > $OUT/shard_C3.json 2> $OUT/shard_C3.err || exit 1
tail -1 $OUT/shard_C3.json
