#!/bin/bash
# Round 4: (1) the whole -m gpu suite and smoke on the final build (beam stack sized by depth);
# (2) beam_kernel time, depth-sized LDS stack (cur) against the fixed 24-level one (build_variants/beamfixed);
# (3) the drain in block-model scenes (OCTPT_DRAIN_MODELS=1) at C5's full size, interleaved twice.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04r}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_all.txt 2>&1 \
    || { tail -40 $O/pytest_all.txt; exit 1; }
tail -2 $O/pytest_all.txt
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -2 $O/smoke.txt
cd /tmp && export TMPDIR=/tmp
for v in cur beamfixed; do
  if [ $v = cur ]; then unset OCTPT_LIB; else export OCTPT_LIB=$R/build_variants/$v/liboctpt.so; fi
  for c in C3 C5b; do
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/beam_${v}_$c -o run -- \
        python3 $R/scripts/spp_sweep.py $c 4 4 4 > $O/beam_${v}_$c.txt 2>&1 || { tail -20 $O/beam_${v}_$c.txt; exit 1; }
    echo "$v $c $(grep -h beam_kernel $O/beam_${v}_$c/run_kernel_stats.csv | cut -d, -f2-4)" | tee -a $O/beam_lds.txt
  done
done
unset OCTPT_LIB
cd $R
for rep in 1 2; do
  for dm in 0 1; do
    OCTPT_DRAIN_MODELS=$dm timeout -k 10 300 python3 bench.py --config C5 --steps 2 --warmup 1 --no-cpu-baseline --no-issued \
        > $O/bench_C5_dm${dm}_$rep.json 2> $O/bench_C5_dm$dm.err || { tail $O/bench_C5_dm$dm.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_C5_dm${dm}_$rep.json')); r=d['roofline']; s=d['stats_rank0']; print('drain_models=$dm', d['value'], d['ms_per_step'], 'ext launches/frame', r['launches'] // 2, 'ext avg', r['kernel_ms_avg'], 'drain segs', s['drain']['segments'])" | tee -a $O/drain_models.txt
  done
done
