#!/bin/bash
# kernel trace + SQ counters of the C3 sweep at a given spp (diagnostics)
set -o pipefail
TAG=${1:-dbg}; SPP=${2:-16}
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $R/scripts/spp_sweep.py C3 $SPP > $OUT/trace.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU -d $OUT/sq -o run --output-format csv -- python3 $R/scripts/spp_sweep.py C3 $SPP > $OUT/sq.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum -d $OUT/sq2 -o run --output-format csv -- python3 $R/scripts/spp_sweep.py C3 $SPP > $OUT/sq2.log 2>&1 || exit $?
echo ok
