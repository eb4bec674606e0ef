set -e
mkdir -p gpurun_out/models
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/models/pytest.log 2>&1 || { tail -60 gpurun_out/models/pytest.log; exit 1; }
tail -3 gpurun_out/models/pytest.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/models/bench.json 2> gpurun_out/models/bench.err
cut -c1-200 gpurun_out/models/bench.json
