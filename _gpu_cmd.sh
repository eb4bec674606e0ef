set -e
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r01g_pytest.log 2>&1 || { tail -40 gpurun_out/r01g_pytest.log; exit 1; }
tail -1 gpurun_out/r01g_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r01g_smoke.log 2>&1 || { tail -20 gpurun_out/r01g_smoke.log; exit 1; }
tail -1 gpurun_out/r01g_smoke.log
timeout -k 10 1000 bash scripts/gpu_profile.sh r01g > gpurun_out/r01g_profile.log 2>&1 || { tail -30 gpurun_out/r01g_profile.log; exit 1; }
tail -1 gpurun_out/r01g/bench.json | cut -c1-700
