#!/bin/bash
# Round 4: the whole -m gpu suite (as the driver runs it at round end) and smoke().
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r04e}
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $OUT/gputest.log 2>&1 \
    || { tail -40 $OUT/gputest.log; exit 1; }
tail -3 $OUT/gputest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
