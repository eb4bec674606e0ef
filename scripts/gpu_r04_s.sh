#!/bin/bash
# Round 4 final: the whole -m gpu suite on the build with one v_min for the loop-carried t_max (no
# canonicalisation), an A/B against the build without it (build_variants/canon), then the bench line
# (default arguments) and the kernel stats of the same command.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04s_final}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_all.txt 2>&1 \
    || { tail -40 $O/pytest_all.txt; exit 1; }
tail -2 $O/pytest_all.txt
bash scripts/ab.sh "C3:256 C5b:64 C4:64" cur build_variants/canon/liboctpt.so > $O/ab_canon.txt 2>&1 || { tail $O/ab_canon.txt; exit 1; }
cat $O/ab_canon.txt
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $O/trace_bench.json 2> $O/trace.err || { tail -20 $O/trace.err; exit 1; }
python3 $R/scripts/pmc_summary.py $O/trace > $O/kernel_summary.txt 2>/dev/null || true
head -12 $O/kernel_summary.txt
