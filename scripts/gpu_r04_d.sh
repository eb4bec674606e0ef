#!/bin/bash
# Round 4: shard timeline + emulation (scripts/gpu_r04_shard.sh), then an A/B of the step-cap bookkeeping's
# cost in extend (build_variants/oldcap: the round-3 cap test and no skipped-iteration bound) at C3 64 spp.
set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/scripts/gpu_r04_shard.sh ${1:-r04d} || exit 1
cd $R
bash scripts/ab.sh "C3:64 C5b:16" cur build_variants/u16/liboctpt.so build_variants/oldcap/liboctpt.so > gpurun_out/${1:-r04d}/ab_cap.txt 2>&1 || { tail gpurun_out/${1:-r04d}/ab_cap.txt; exit 1; }
cat gpurun_out/${1:-r04d}/ab_cap.txt
