#!/bin/bash
# Copy a gpu_profile.sh run (gpurun_out/TAG) into profiles/DEST: bench JSON, kernel stats,
# FETCH/WRITE counter CSVs, a per-kernel counter summary and profiles/pmc_C3.json (traffic).
set -e
TAG=$1; DEST=${2:-profiles/r01}; PREFIX=${3:-wavefront}
S=gpurun_out/$TAG
mkdir -p $DEST
cp $S/bench.json $DEST/bench_$PREFIX.json
cp $S/trace/run_kernel_stats.csv $DEST/${PREFIX}_kernel_stats.csv
cp $S/pmc_fetch/run_counter_collection.csv $DEST/${PREFIX}_pmc_fetch.csv
cp $S/pmc_write/run_counter_collection.csv $DEST/${PREFIX}_pmc_write.csv
python3 scripts/pmc_summary.py $S/trace $S/pmc_tcc $S/pmc_sq $S/pmc_fetch $S/pmc_write > $DEST/${PREFIX}_summary.txt
[ -f $S/pmc_C3.json ] && cp $S/pmc_C3.json profiles/pmc_C3.json
[ -f $S/fetch_calib.json ] && cp $S/fetch_calib.json profiles/fetch_calib.json
for c in C4 C5; do [ -f $S/bench_full_$c.json ] && cp $S/bench_full_$c.json $DEST/bench_full_$c.json; done
true
echo "collected $S -> $DEST"
