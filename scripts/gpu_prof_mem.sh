#!/bin/bash
# memory-pipe counters of the C3 sweep (diagnostics): separate small --pmc passes
set -o pipefail
TAG=${1:-mem}; SPP=${2:-16}
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() { timeout -k 5 60 rocprofv3 --pmc "$@" -d $OUT/p$N -o run --output-format csv -- python3 $R/scripts/spp_sweep.py C3 $SPP > $OUT/p$N.log 2>&1; }
N=1 run TA_TA_BUSY_sum GRBM_GUI_ACTIVE || exit $?
N=2 run TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum || exit $?
N=3 run TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum || exit $?
N=4 run TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum || exit $?
N=5 run SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_BUSY_CU_CYCLES || exit $?
N=6 run TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum || exit $?
echo ok
