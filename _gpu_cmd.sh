set -e
mkdir -p gpurun_out/full2
timeout -k 10 400 python -u bench.py --config C4 --steps 1 --warmup 1 --cpu-seconds 10 > gpurun_out/full2/bench_C4.json 2> gpurun_out/full2/bench_C4.err || { tail -20 gpurun_out/full2/bench_C4.err; exit 1; }
timeout -k 10 700 python -u bench.py --config C5 --steps 1 --warmup 1 --cpu-seconds 10 > gpurun_out/full2/bench_C5.json 2> gpurun_out/full2/bench_C5.err || { tail -20 gpurun_out/full2/bench_C5.err; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/full2/bench_C3.json 2> gpurun_out/full2/bench_C3.err || { tail -20 gpurun_out/full2/bench_C3.err; exit 1; }
for c in C3 C4 C5; do echo $c $(tail -1 gpurun_out/full2/bench_$c.json | cut -c100-190); done
