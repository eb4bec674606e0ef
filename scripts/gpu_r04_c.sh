#!/bin/bash
# Round 4: step-cap test with the picket world, multi-device tests, the hit-record check build, the stale-hit
# probe (pre-fix variants), smoke, C3 bench lines (one process; C-ABI multi with two entries).
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r04c}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_beam.py::test_beam_step_cap tests/test_gpu_multi.py tests/test_gpu_hitcheck.py tests/test_gpu_lean.py tests/test_gpu_bench.py \
    -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 180 python -u scripts/stale_hit_probe.py > $OUT/stale_probe.json 2> $OUT/stale_probe.err || { tail -20 $OUT/stale_probe.err; exit 1; }
cat $OUT/stale_probe.json
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --capi-devices 2 --no-cpu-baseline > $OUT/bench_capi2.json 2> $OUT/bench_capi2.err \
    || { tail -20 $OUT/bench_capi2.err; exit 1; }
cat $OUT/bench_capi2.json
