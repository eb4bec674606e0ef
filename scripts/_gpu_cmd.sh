# scratch GPU command of the current step (run via gpurun from the repo root)
set -o pipefail
O=gpurun_out/r02x; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
timeout -k 10 300 python -u scripts/shard_emulation.py --config C3 > $O/shard_emulation_C3.txt 2> $O/shard.err || exit 1
tail -1 $O/shard_emulation_C3.txt > $O/shard_emulation_C3.json
timeout -k 10 400 python -u scripts/shard_emulation.py --config C4 > $O/shard_emulation_C4.txt 2>> $O/shard.err || exit 1
tail -1 $O/shard_emulation_C4.txt > $O/shard_emulation_C4.json
cat $O/shard_emulation_C3.json $O/shard_emulation_C4.json
