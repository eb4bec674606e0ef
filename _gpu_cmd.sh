set -e
mkdir -p gpurun_out/branch
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/branch/pytest.log 2>&1 || { tail -50 gpurun_out/branch/pytest.log; exit 1; }
tail -2 gpurun_out/branch/pytest.log
