#!/bin/bash
# Round 4: the beam's full-frame / near-axis / step-cap oracle cases, the multi-device C ABI
# (octpt_create_multi) tests, smoke, then C3 bench lines: one process per GPU and the C-ABI multi path
# (two entries on the one GPU).  Every GPU step under its own limit; a failure ends the script.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r04b}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_beam.py -k "fullframe or near_axis or step_cap" tests/test_gpu_multi.py \
    -x -v --timeout 400 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --capi-devices 2 --no-cpu-baseline > $OUT/bench_capi2.json 2> $OUT/bench_capi2.err \
    || { tail -20 $OUT/bench_capi2.err; exit 1; }
cat $OUT/bench_capi2.json
