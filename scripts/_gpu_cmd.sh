# scratch GPU command of the current step (run via gpurun from the repo root)
set -o pipefail
O=gpurun_out/r02z; mkdir -p $O
timeout -k 10 400 python3 bench.py --config C5 --steps 2 --warmup 1 > $O/bench_full_C5.json 2> $O/bench_full_C5.err || exit 1
cut -c1-200 $O/bench_full_C5.json
