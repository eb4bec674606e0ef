set -e
bash scripts/gpu_profile.sh r01c
cut -c1-300 gpurun_out/r01c/bench.json
