# scratch GPU command of the current step (run via gpurun from the repo root)
set -o pipefail
mkdir -p gpurun_out/r02
timeout -k 10 600 python -u -m pytest tests/test_gpu_forms.py tests/test_gpu_builder.py tests/test_gpu_bench.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r02/new.log 2>&1 || { tail -60 gpurun_out/r02/new.log; exit 1; }
tail -3 gpurun_out/r02/new.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02/all.log 2>&1 || { tail -60 gpurun_out/r02/all.log; exit 1; }
tail -3 gpurun_out/r02/all.log
timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/r02/bench.json 2> gpurun_out/r02/bench.err || { tail -20 gpurun_out/r02/bench.err; exit 1; }
cat gpurun_out/r02/bench.json
