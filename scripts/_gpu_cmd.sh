# scratch GPU command of the current step (run via gpurun from the repo root)
set -o pipefail
O=gpurun_out/r02n; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_fuzz.py -v --timeout 300 --timeout-method thread > $O/fuzz.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|assert" $O/fuzz.log | tail -60
[ $rc = 0 ] || exit $rc
for cfg in C3:256 C4:64; do
  c=${cfg%%:*}; s=${cfg##*:}
  for mode in "" --compact; do
    timeout -k 10 300 python -u bench.py --config $c --spp $s --steps 3 --warmup 1 --no-cpu-baseline $mode > $O/b.json 2>> $O/bench.err || exit 1
    python -c "import json,sys; d=json.load(open(sys.argv[1])); st=d['stats_rank0']; print(sys.argv[2], d['value'], d['roofline']['kernel_ms_avg'], round(st['esvo_steps']/st['segments'],2), round((st['sphere_tests']+st['cuboid_tests'])/st['segments'],3), d['ms_per_step'])" $O/b.json "$c $mode" | tee -a $O/compact.txt
  done
done
