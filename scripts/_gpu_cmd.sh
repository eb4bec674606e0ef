# scratch GPU command of the current step (run via gpurun from the repo root)
set -o pipefail
O=gpurun_out/r02i; mkdir -p $O
for cfg in C3 C3-in C5 C5-fp; do
  for mode in on off; do
    if [ $mode = off ]; then export OCTPT_START_CHAIN=0; else unset OCTPT_START_CHAIN; fi
    echo "== $cfg preview chain $mode" | tee -a $O/preview.txt
    timeout -k 10 200 python scripts/spp_sweep.py $cfg 1 1 1 1 1 1 --preview 2>&1 | grep spp | tail -4 | tee -a $O/preview.txt || exit 1
  done
done
unset OCTPT_START_CHAIN
run() {  # tag config spp [env...]
  local tag=$1 cfg=$2 spp=$3; shift 3
  env "$@" timeout -k 10 300 python -u bench.py --config $cfg --spp $spp --steps 3 --warmup 1 --no-cpu-baseline > $O/b.json 2>> $O/bench.err || return 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['roofline']['kernel_ms_avg'])" $O/b.json "$tag $cfg" | tee -a $O/ab.txt
}
for rep in 1 2; do
  for cfg in C3:256 C5:64; do
    c=${cfg%%:*}; s=${cfg##*:}
    run chain-off-rt $c $s OCTPT_START_CHAIN=0 || exit 1
    run chain-compiled-out $c $s OCTPT_LIB=build_variants/nochain/liboctpt.so || exit 1
  done
done
