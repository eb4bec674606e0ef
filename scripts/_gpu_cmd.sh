# scratch GPU command of the current step (run via gpurun from the repo root)
set -o pipefail
O=gpurun_out/r02aa; mkdir -p $O
run() {  # tag config spp [env...]
  local tag=$1 cfg=$2 spp=$3; shift 3
  env "$@" timeout -k 10 300 python -u bench.py --config $cfg --spp $spp --steps 3 --warmup 1 --no-cpu-baseline > $O/b.json 2>> $O/bench.err || return 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], r['kernel_ms_avg'], r['launches'])" $O/b.json "$tag $cfg" | tee -a $O/ab.txt
}
for rep in 1 2; do
for cfg in C3:256 C4:64; do
  c=${cfg%%:*}; s=${cfg##*:}
  run pool512M $c $s || exit 1
  run pool1G $c $s OCTPT_POOL=1073741824 || exit 1
  run pool256M $c $s OCTPT_POOL=268435456 || exit 1
done
done
