set -e
mkdir -p gpurun_out/shard2
timeout -k 10 400 python -u scripts/shard_emulation.py --config C3 > gpurun_out/shard2/shard.json 2> gpurun_out/shard2/shard.err || { tail -20 gpurun_out/shard2/shard.err; exit 1; }
tail -1 gpurun_out/shard2/shard.json
