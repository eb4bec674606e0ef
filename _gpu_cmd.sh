set -e
mkdir -p gpurun_out/nee
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/nee/pytest.log 2>&1 || { tail -40 gpurun_out/nee/pytest.log; exit 1; }
tail -3 gpurun_out/nee/pytest.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/nee/bench.json 2> gpurun_out/nee/bench.err
cut -c1-300 gpurun_out/nee/bench.json
