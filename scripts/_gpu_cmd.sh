# scratch GPU command of the current step (run via gpurun from the repo root)
set -o pipefail
O=gpurun_out/r02n; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -v --timeout 300 --timeout-method thread > $O/fuzz.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert" $O/fuzz.log | tail -60
exit $rc
