set -o pipefail
timeout -k 10 200 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
for v in base w6; do
  L=""; [ $v != base ] && L=build_variants/$v/liboctpt.so
  for rf in 24 32; do
    echo "== $v refill $rf"; OCTPT_LIB=$L OCTPT_REFILL=$rf timeout -k 10 120 python scripts/spp_sweep.py C3 64 2>&1 | grep spp || exit 1
  done
done
