#!/bin/bash
# Round 4: rehearsal of the driver's 8-rank bench on the one-GPU box: bench.py --gpus 8 (eight spawned ranks
# sharing the GPU, gathering over gloo since RCCL needs distinct devices), full C3, with rank 0's capi_multi
# measurement over 8 entries of device 0.  Checks that the N = 8 path runs end to end and prints one line.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04t}
mkdir -p $O
cd $R
timeout -k 10 600 python3 bench.py --gpus 8 --dist-backend gloo --steps 2 --warmup 1 --no-cpu-baseline --no-issued \
    > $O/bench_n8_gloo.json 2> $O/bench_n8_gloo.err || { tail -30 $O/bench_n8_gloo.err; exit 1; }
cat $O/bench_n8_gloo.json
