set -o pipefail
OCTPT_EXTEND=split timeout -k 10 240 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
echo "== C3 base"; timeout -k 10 120 python scripts/spp_sweep.py C3 64 64 --ktime 2>&1 | grep spp || exit 1
echo "== C3 split"; OCTPT_EXTEND=split timeout -k 10 120 python scripts/spp_sweep.py C3 64 64 --ktime 2>&1 | grep spp || exit 1
echo "== C4 split"; OCTPT_EXTEND=split timeout -k 10 120 python scripts/spp_sweep.py C4 16 --ktime 2>&1 | grep spp || exit 1
