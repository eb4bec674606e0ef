#!/bin/bash
# Usage: scripts/gpu_pmc_config.sh CONFIG SPP TAG -- on the GPU box (via gpurun) from the repo root.
# FETCH_SIZE / WRITE_SIZE / TCC passes of a one-step bench of CONFIG at SPP spp, then
# profiles/pmc_CONFIG.json (traffic per extend launch, calibrated FETCH_SIZE factor 1, L2 hit rate),
# written into gpurun_out/TAG/ and into profiles/ on the box (read by bench.py's roofline.traffic).
set -o pipefail
C=$1; SPP=$2; TAG=${3:-r02}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG/pmc_$C
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P="--config $C --spp $SPP --no-cpu-baseline --steps 1 --warmup 0"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 $R/bench.py $P > $OUT/fetch.json 2> $OUT/fetch.err || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 $R/bench.py $P > $OUT/write.json 2> $OUT/write.err || exit $?
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $OUT/tcc -o run --output-format csv -- python3 $R/bench.py $P > $OUT/tcc.json 2> $OUT/tcc.err || exit $?
python3 $R/scripts/pmc_traffic.py $OUT/fetch $OUT/write $C $OUT/pmc_$C.json 1.0 "calibrated by tools/fetch_calib.hip (profiles/fetch_calib.json): scattered 8-B and 16-B reads are counted at 64 B per request, factor 1; $C at $SPP spp (the bench frame), one step" $OUT/tcc > /dev/null || exit $?
cp $OUT/pmc_$C.json $R/profiles/pmc_$C.json
echo "pmc $C done"
