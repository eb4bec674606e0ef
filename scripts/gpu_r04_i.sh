#!/bin/bash
# Round 4: ticket-free seeding (wf_seed_kernel, every tile inside the image) against the ticket per wave
# (build_variants/seedticket): the whole -m gpu suite, a frame-rate A/B, and the seed kernel's time from a
# C3 kernel trace of each.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04i}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_all.txt 2>&1 \
    || { tail -40 $O/pytest_all.txt; exit 1; }
tail -2 $O/pytest_all.txt
bash scripts/ab.sh "C3:256 C5b:64 C4:64" cur build_variants/seedticket/liboctpt.so > $O/ab_seed.txt 2>&1 || { tail $O/ab_seed.txt; exit 1; }
cat $O/ab_seed.txt
cd /tmp && export TMPDIR=/tmp
for v in cur seedticket; do
  if [ $v = cur ]; then unset OCTPT_LIB; else export OCTPT_LIB=$R/build_variants/$v/liboctpt.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$v -o run -- \
      python3 $R/scripts/spp_sweep.py C3 256 256 > $O/trace_$v.txt 2>&1 || { tail -20 $O/trace_$v.txt; exit 1; }
  grep -h "seed\|Name" $O/trace_$v/run_kernel_stats.csv | cut -c1-200
done
unset OCTPT_LIB
