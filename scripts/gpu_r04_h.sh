#!/bin/bash
# Round 4: the drain threshold on the 8-way C3 shard (the shard's extend tails), then the
# step-cap bookkeeping's cost (cur vs build_variants/u16, build_variants/oldcap) at C3 64 spp.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04h}
mkdir -p $O
cd $R
for d in 4096 16384 65536 262144; do
  echo "== OCTPT_DRAIN_RAYS=$d" >> $O/shard_drain.txt
  OCTPT_DRAIN_RAYS=$d timeout -k 10 200 python3 scripts/shard_emulation.py --config C3 --ns 1 8 2>> $O/shard_drain.err | tail -1 >> $O/shard_drain.txt || { tail -20 $O/shard_drain.err; exit 1; }
done
cat $O/shard_drain.txt
bash scripts/ab.sh "C3:64" cur build_variants/u16/liboctpt.so build_variants/oldcap/liboctpt.so > $O/ab_cap.txt 2>&1 || { tail $O/ab_cap.txt; exit 1; }
cat $O/ab_cap.txt
