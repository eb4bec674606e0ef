# scratch GPU command of the current step (run via gpurun from the repo root)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r02ab; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/shard_emulation.py --config C3 --ns 8 > $O/shard8.txt 2> $O/shard8.err || exit 1
tail -1 $O/shard8.txt
