#!/bin/bash
# Usage: scripts/gpu_profile.sh TAG  -- run on the GPU box (via gpurun) from the repo root.
# 1) (CALIB=1) FETCH_SIZE calibration (tools/fetch_calib) under rocprofv3;
# 2) PMC passes (FETCH_SIZE, WRITE_SIZE, SQ, TCC) of a 1-step bench;
# 3) the bench (default args, with CPU baseline) and kernel-trace/stats of the same bench command.
# The traffic JSON (profiles/pmc_C3.json) is computed afterwards from the returned CSVs.
set -o pipefail
TAG=${1:-r02}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
# (CALIB=1: the FETCH_SIZE calibration too; build tools/fetch_calib first, profiles/fetch_calib.json has round 2's)
if [ -n "$CALIB" ]; then
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/calib -o run --output-format csv -- $R/tools/fetch_calib > $OUT/calib.out 2> $OUT/calib.err || exit $?
fi
P="--no-cpu-baseline --no-issued --steps 1 --warmup 0"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 $R/bench.py $P > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 $R/bench.py $P > $OUT/pmc_write.json 2> $OUT/pmc_write.err || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS -d $OUT/pmc_sq -o run --output-format csv -- python3 $R/bench.py $P > $OUT/pmc_sq.json 2> $OUT/pmc_sq.err || exit $?
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/pmc_tcc -o run --output-format csv -- python3 $R/bench.py $P > $OUT/pmc_tcc.json 2> $OUT/pmc_tcc.err || exit $?
# traffic per launch (calibrated FETCH_SIZE factor 1, profiles/fetch_calib.json) + L2 hit rate, read by
# the bench lines below (and committed from $OUT by scripts/collect_profiles.sh)
[ -n "$CALIB" ] && { python3 $R/scripts/fetch_calib.py $OUT/calib.out $OUT/calib $OUT/fetch_calib.json > /dev/null || echo "fetch calibration summary failed" >&2; }
python3 $R/scripts/pmc_traffic.py $OUT/pmc_fetch $OUT/pmc_write C3 $OUT/pmc_C3.json 1.0 "calibrated by tools/fetch_calib.hip (profiles/fetch_calib.json): scattered 8-B and 16-B reads are counted at 64 B per request, factor 1; 16-B coalesced streams at half, factor 2" $OUT/pmc_tcc > /dev/null || exit $?
cp $OUT/pmc_C3.json $R/profiles/pmc_C3.json
timeout -k 10 400 python3 $R/bench.py --steps 10 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 > $OUT/trace_bench.json 2> $OUT/trace.err || exit $?
# the two 4K configs at full size on this one GPU (the 8-GPU cases of BASELINE.json)
if [ -n "$FULL" ]; then
  timeout -k 10 400 python3 $R/bench.py --config C4 --steps 2 --warmup 1 > $OUT/bench_full_C4.json 2> $OUT/bench_full_C4.err || exit $?
  timeout -k 10 400 python3 $R/bench.py --config C5 --steps 2 --warmup 1 > $OUT/bench_full_C5.json 2> $OUT/bench_full_C5.err || exit $?
fi
echo done
