#!/bin/bash
# Round 4, beam step cap: (1) the variant built without the skipped-iteration bound
# (build_variants/nofix, beam_pack's bound forced to 0) must fail test_beam_step_cap -- the test catches
# the defect; (2) the beam suite, full-frame oracle cases included, with the product library; (3) one
# C3 bench line.  Every GPU step under its own limit; a crash or timeout ends the script.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r04a}
mkdir -p $OUT
cd $R
OCTPT_LIB=build_variants/nofix/liboctpt.so timeout -k 10 300 python -u -m pytest tests/test_gpu_beam.py -k step_cap -x -q \
    --timeout 240 --timeout-method thread > $OUT/nofix.log 2>&1
rc=$?
echo "nofix exit $rc" | tee -a $OUT/nofix.log
case $rc in 0|1) ;; *) exit 1 ;; esac
timeout -k 10 840 python -u -m pytest tests/test_gpu_beam.py -x -v --timeout 400 --timeout-method thread > $OUT/beam.log 2>&1 \
    || { tail -40 $OUT/beam.log; exit 1; }
tail -3 $OUT/beam.log
timeout -k 10 300 python3 bench.py --steps 5 --warmup 1 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
