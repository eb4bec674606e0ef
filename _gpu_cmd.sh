set -e
mkdir -p gpurun_out/full
timeout -k 10 400 python -u bench.py --config C4 --steps 1 --warmup 1 --cpu-seconds 10 > gpurun_out/full/bench_C4.json 2> gpurun_out/full/bench_C4.err || { tail -20 gpurun_out/full/bench_C4.err; exit 1; }
tail -1 gpurun_out/full/bench_C4.json | cut -c1-300
timeout -k 10 700 python -u bench.py --config C5 --steps 1 --warmup 1 --cpu-seconds 10 > gpurun_out/full/bench_C5.json 2> gpurun_out/full/bench_C5.err || { tail -20 gpurun_out/full/bench_C5.err; exit 1; }
tail -1 gpurun_out/full/bench_C5.json | cut -c1-300
