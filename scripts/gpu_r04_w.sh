#!/bin/bash
# Round 4 final build: smoke, the bench line (default arguments) and the kernel stats of the same command.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04w}
mkdir -p $O
cd $R
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $O/trace_bench.json 2> $O/trace.err || { tail -20 $O/trace.err; exit 1; }
python3 $R/scripts/pmc_summary.py $O/trace > $O/kernel_summary.txt 2>/dev/null || true
head -12 $O/kernel_summary.txt
