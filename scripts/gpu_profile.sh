#!/bin/bash
# Usage: scripts/gpu_profile.sh TAG  -- run on the GPU box (via gpurun) from the repo root.
# 1) PMC passes (FETCH_SIZE, WRITE_SIZE, SQ, TCC) of a 1-step bench -> profiles/pmc_C3.json, so
# 2) the bench (default args, with CPU baseline) reports this run's traffic, and
# 3) kernel-trace/stats of the same bench command.
set -o pipefail
TAG=${1:-r01}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P="--no-cpu-baseline --steps 1 --warmup 0"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 $R/bench.py $P > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 $R/bench.py $P > $OUT/pmc_write.json 2> $OUT/pmc_write.err || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS -d $OUT/pmc_sq -o run --output-format csv -- python3 $R/bench.py $P > $OUT/pmc_sq.json 2> $OUT/pmc_sq.err || exit $?
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/pmc_tcc -o run --output-format csv -- python3 $R/bench.py $P > $OUT/pmc_tcc.json 2> $OUT/pmc_tcc.err || exit $?
python3 $R/scripts/pmc_traffic.py $OUT/pmc_fetch $OUT/pmc_write C3 $OUT/pmc_C3.json > /dev/null || exit $?
cp $OUT/pmc_C3.json $R/profiles/pmc_C3.json
timeout -k 10 300 python3 $R/bench.py > $OUT/bench.json 2> $OUT/bench.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/bench.py > $OUT/trace_bench.json 2> $OUT/trace.err || exit $?
echo done
