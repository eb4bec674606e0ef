# scratch GPU command of the current step (run via gpurun from the repo root)
set -o pipefail
O=gpurun_out/r02s; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -2 $O/gputest.log
run() {  # tag config spp [env...]
  local tag=$1 cfg=$2 spp=$3; shift 3
  env "$@" timeout -k 10 300 python -u bench.py --config $cfg --spp $spp --steps 3 --warmup 1 --no-cpu-baseline > $O/b.json 2>> $O/bench.err || return 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], r['kernel_ms_avg'], r['shade']['kernel_ms_avg'], d['config']['segments_per_step'])" $O/b.json "$tag $cfg" | tee -a $O/ab.txt
}
for rep in 1 2; do
  for cfg in C3:256 C2:64 C4:64 C5:64; do
    c=${cfg%%:*}; s=${cfg##*:}
    run pair $c $s || exit 1
    run base $c $s OCTPT_LIB=build_variants/base/liboctpt.so || exit 1
  done
done
