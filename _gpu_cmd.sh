set -e
mkdir -p gpurun_out/tail
rm -f gpurun_out/tail/sweep.jsonl
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tail/pytest.log 2>&1 || { tail -40 gpurun_out/tail/pytest.log; exit 1; }
tail -1 gpurun_out/tail/pytest.log
CONFIG=C3 SPP=256 scripts/extend_sweep.sh gpurun_out/tail/sweep.jsonl "OCTPT_NO_TAIL_GRIDS=1,C=C3" "C=C3" "OCTPT_NO_TAIL_GRIDS=1,C=C3" "C=C3"
CONFIG=C2 SPP=64 scripts/extend_sweep.sh gpurun_out/tail/sweep.jsonl "OCTPT_NO_TAIL_GRIDS=1,C=C2" "C=C2" "OCTPT_NO_TAIL_GRIDS=1,C=C2" "C=C2"
timeout -k 10 400 python -u scripts/shard_emulation.py --config C3 --ns 8 > gpurun_out/tail/shard.json 2> gpurun_out/tail/shard.err || { tail -20 gpurun_out/tail/shard.err; exit 1; }
tail -1 gpurun_out/tail/shard.json
OCTPT_NO_TAIL_GRIDS=1 timeout -k 10 400 python -u scripts/shard_emulation.py --config C3 --ns 8 > gpurun_out/tail/shard0.json 2> gpurun_out/tail/shard0.err || { tail -20 gpurun_out/tail/shard0.err; exit 1; }
tail -1 gpurun_out/tail/shard0.json
