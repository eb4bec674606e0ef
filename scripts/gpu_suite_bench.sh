#!/bin/bash
# Usage (on the GPU box via gpurun, from the repo root): scripts/gpu_suite_bench.sh TAG [CONFIG]
# The -m gpu suite, then one bench line of CONFIG (default C3) with the CPU baseline and the issued-bytes
# probe; every step under its own time limit, stopping at the first failure.
set -o pipefail
TAG=${1:-run}
CFG=${2:-C3}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gputest.log 2>&1 || { tail -30 $OUT/gputest.log; exit 1; }
tail -3 $OUT/gputest.log
timeout -k 10 400 python3 bench.py --config $CFG --steps 5 --warmup 1 > $OUT/bench_$CFG.json 2> $OUT/bench_$CFG.err || { tail -20 $OUT/bench_$CFG.err; exit 1; }
cat $OUT/bench_$CFG.json
