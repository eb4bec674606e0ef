#!/bin/bash
# Registers, scratch and occupancy of the wavefront kernels as the compiler reports them (kernel-resource-usage
# remarks): tools/resource_usage.sh [-DFLAG ...].  CPU only (a device-only compile of octpt_kernels.hip).
cd "$(dirname "$0")/.."
FLAGS=$(python3 -c "import __graft_entry__ as g; print(' '.join(f for f in g.HIPCC_FLAGS if f not in ('-shared', '-fPIC')))")
/opt/rocm/bin/hipcc $FLAGS "$@" -c octree_pathtracing_amd/csrc/octpt_kernels.hip -o /tmp/octpt_res.o --offload-device-only \
    -Rpass-analysis=kernel-resource-usage 2>&1 | sed 's/ \[-Rpass-analysis=kernel-resource-usage\]//' | awk '
  /Function Name:/ {n = $NF}
  /remark:     VGPRs:/ {v = $NF}
  /remark:     TotalSGPRs: / {sg = $NF}
  /ScratchSize/ {sc = $NF}
  /Occupancy/ {if (n ~ /extend|shade|seed|drain|beam/) printf "%-70s VGPR %3s SGPR %3s scratch %3s occ %s\n", substr(n, 1, 70), v, sg, sc, $NF}'
