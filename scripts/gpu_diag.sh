#!/bin/bash
# Diagnostics of the C3 wavefront kernels: kernel stats + SQ counter passes per extend variant.
# Usage (on the GPU box): scripts/gpu_diag.sh TAG SPP LEAF_BATCH...
set -o pipefail
TAG=${1:-diag}; SPP=${2:-16}; shift 2
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for LB in "$@"; do
  export OCTPT_LEAF_BATCH=$LB
  timeout -k 5 90 rocprofv3 --kernel-trace --stats -d $OUT/lb$LB/trace -o run --output-format csv -- python3 $R/scripts/spp_sweep.py C3 $SPP > $OUT/lb$LB.log 2>&1 || exit $?
  timeout -k 5 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -d $OUT/lb$LB/p1 -o run --output-format csv -- python3 $R/scripts/spp_sweep.py C3 $SPP >> $OUT/lb$LB.log 2>&1 || exit $?
  timeout -k 5 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_WAVES SQ_INSTS_BRANCH -d $OUT/lb$LB/p2 -o run --output-format csv -- python3 $R/scripts/spp_sweep.py C3 $SPP >> $OUT/lb$LB.log 2>&1 || exit $?
done
timeout -k 5 60 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
echo ok
