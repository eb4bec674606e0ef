set -e
timeout -k 10 300 python -m pytest tests -m gpu -x -q 2>&1 | tail -3
for v in default noff default noff; do
  if [ $v = default ]; then L=""; else L=build_variants/$v/liboctpt.so; fi
  echo "== $v"; OCTPT_LIB=$L timeout -k 10 120 python scripts/spp_sweep.py C3 256 --ktime
done
echo "== C4"; timeout -k 10 120 python scripts/spp_sweep.py C4 64 --ktime
OCTPT_LIB=build_variants/noff/liboctpt.so timeout -k 10 120 python scripts/spp_sweep.py C4 64 --ktime
