set -e
timeout -k 10 400 python -m pytest tests -m gpu -x -q 2>&1 | tail -4
echo "== C5"; OCTPT_DEBUG=1 timeout -k 10 300 python scripts/spp_sweep.py C5 16 64 --ktime
echo "== C5 preview"; timeout -k 10 120 python scripts/spp_sweep.py C5 1 1 1 --preview
