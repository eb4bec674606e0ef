#!/bin/bash
# SQ counter passes of the C3 wavefront render (diagnostics).  Usage: gpu_diag_sq.sh TAG [SPP]
set -o pipefail
TAG=${1:-sq}; SPP=${2:-16}
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() { timeout -k 5 90 rocprofv3 --pmc "$@" -d $OUT/p$N -o run --output-format csv -- python3 $R/scripts/spp_sweep.py C3 $SPP > $OUT/p$N.log 2>&1; }
N=1 run SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU || exit $?
N=2 run SQ_INST_CYCLES_SALU SQ_BUSY_CU_CYCLES SQ_IFETCH SQ_INSTS_VSKIPPED SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_INSTS_SMEM || exit $?
N=3 run SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE SQ_BUSY_CYCLES || exit $?
echo ok
