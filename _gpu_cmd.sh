set -e
timeout -k 10 300 python -m pytest tests/test_gpu_builder.py -x -q 2>&1 | tail -2
timeout -k 10 300 python scripts/build_bench.py
