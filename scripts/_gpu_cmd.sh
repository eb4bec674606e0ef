# scratch GPU command of the current step (run via gpurun from the repo root)
set -o pipefail
O=gpurun_out/r02b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
echo "== lanes (fold 1)"; OCTPT_PROFILE_LANES=1 OCTPT_LIB=build_variants/prof/liboctpt.so timeout -k 10 300 python scripts/spp_sweep.py C3 64 --ktime 2>&1 | grep -E "spp|lanes" || exit 1
bash scripts/ab.sh "C3:64 C2:64 C4:32 C5:32" build_variants/fold0/liboctpt.so cur build_variants/fold2/liboctpt.so 2>&1 | tee $O/ab.log || exit 1
