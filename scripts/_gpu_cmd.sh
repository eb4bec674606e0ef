# scratch GPU command of the current step (run via gpurun from the repo root)
set -o pipefail
O=gpurun_out/r02r; mkdir -p $O
bash scripts/gpu_pmc_config.sh C4 64 r02r || exit 1
bash scripts/gpu_pmc_config.sh C5 64 r02r || exit 1
timeout -k 10 400 python3 bench.py --config C4 --steps 2 --warmup 1 > $O/bench_full_C4.json 2> $O/bench_full_C4.err || exit 1
timeout -k 10 400 python3 bench.py --config C5 --steps 2 --warmup 1 > $O/bench_full_C5.json 2> $O/bench_full_C5.err || exit 1
cut -c1-300 $O/bench_full_C4.json $O/bench_full_C5.json
