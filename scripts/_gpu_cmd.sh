# scratch GPU command of the current step (run via gpurun from the repo root)
set -o pipefail
O=gpurun_out/r02f; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_scene_build.py -x -v -s --timeout 300 --timeout-method thread > $O/scene_build.log 2>&1 || { tail -40 $O/scene_build.log; exit 1; }
grep -E "PASS|FAIL|ms" $O/scene_build.log | tail -30
