#!/bin/bash
# Round 4: the steering snapshot kernel (wf_snapshot_kernel) against the two strided copies it replaced
# (build_variants/snapmemcpy): parity subset, frame-rate A/B, and a C5 kernel timeline of each (gaps).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04g}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_drain.py tests/test_gpu_lean.py tests/test_gpu_oom.py \
    -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_snap.txt 2>&1 || { tail -40 $O/pytest_snap.txt; exit 1; }
tail -2 $O/pytest_snap.txt
bash scripts/ab_env.sh "C5:64 C5b:64 C4:64 C3:256" "cur|" "build_variants/snapmemcpy/liboctpt.so|" > $O/ab_snap.txt 2>&1 \
    || { tail $O/ab_snap.txt; exit 1; }
cat $O/ab_snap.txt
cd /tmp && export TMPDIR=/tmp
for v in cur snapmemcpy; do
  if [ $v = cur ]; then unset OCTPT_LIB; else export OCTPT_LIB=$R/build_variants/$v/liboctpt.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/trace_$v -o run -- \
      python3 $R/scripts/spp_sweep.py C5 64 64 > $O/trace_$v.txt 2>&1 || { tail -20 $O/trace_$v.txt; exit 1; }
  T=$(find $O/trace_$v -name '*kernel_trace.csv' | head -1)
  python3 $R/scripts/timeline.py "$T" --skip 1 > $O/timeline_$v.json || exit 1
  python3 -c "
import json; d=json.load(open('$O/timeline_$v.json'))
for r in d['per_render']: print('$v', r['wall_us'], 'gaps', r['gaps_us'], 'tail', r['tail_us'], r['launches'])"
done
cd $R
bash scripts/gpu_r04_shard.sh ${1:-r04g}_shard || exit 1
