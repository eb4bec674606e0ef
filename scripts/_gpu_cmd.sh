set -o pipefail
echo "== base"; timeout -k 10 120 python scripts/spp_sweep.py C3 64 --ktime 2>&1 | grep spp || exit 1
echo "== xcdmix"; OCTPT_LIB=build_variants/xcdmix/liboctpt.so timeout -k 10 120 python scripts/spp_sweep.py C3 64 --ktime 2>&1 | grep spp || exit 1
