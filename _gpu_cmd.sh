set -e
echo "== C2"; timeout -k 10 120 python scripts/spp_sweep.py C2 64 --ktime
echo "== C4"; timeout -k 10 200 python scripts/spp_sweep.py C4 64 --ktime
echo "== C3 preview"; timeout -k 10 120 python scripts/spp_sweep.py C3 1 1 1 --preview
echo "== C4 preview"; timeout -k 10 120 python scripts/spp_sweep.py C4 1 1 1 --preview
