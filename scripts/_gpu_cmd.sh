# scratch GPU command of the current step (run via gpurun from the repo root)
set -o pipefail
O=gpurun_out/r02e; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
bash scripts/gpu_profile.sh r02 || exit 1
cut -c1-600 gpurun_out/r02/bench.json
