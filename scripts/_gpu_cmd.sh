set -o pipefail
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
echo "== C3"; OCTPT_DEBUG=1 timeout -k 10 120 python scripts/spp_sweep.py C3 64 256 --ktime 2>&1 | grep -E "spp|octpt:" | sort -u || exit 1
