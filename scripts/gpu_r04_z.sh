#!/bin/bash
# Round 4 final build: the 8-way shard emulation of C3 (the ceiling of the driver's N = 8 run).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04z}
mkdir -p $O
cd $R
timeout -k 10 300 python3 scripts/shard_emulation.py --config C3 --ns 1 2 4 8 > $O/shard_C3.json 2> $O/shard_C3.err || { tail -20 $O/shard_C3.err; exit 1; }
tail -1 $O/shard_C3.json
