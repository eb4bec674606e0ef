#!/bin/bash
# Round 4: two wavefront lanes (OCTPT_LANES=2): parity subset under lanes, A/B of the
# frame rate (one lane / two lanes at half grid / two lanes at full grid), then the whole -m gpu suite
# under two lanes.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04l}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_lanes.py \
    -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_lanes_subset.txt 2>&1 \
    || { tail -40 $O/pytest_lanes_subset.txt; exit 1; }
tail -3 $O/pytest_lanes_subset.txt
bash scripts/ab_env.sh "C3:256 C5:64 C5b:64 C4:64" "cur|" "cur|OCTPT_LANES=2" "cur|OCTPT_LANES=2,OCTPT_LANE_GRID=full" \
    > $O/ab_lanes.txt 2>&1 || { tail $O/ab_lanes.txt; exit 1; }
cat $O/ab_lanes.txt
OCTPT_LANES=2 timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest_lanes_all.txt 2>&1 \
    || { tail -40 $O/pytest_lanes_all.txt; exit 1; }
tail -3 $O/pytest_lanes_all.txt
