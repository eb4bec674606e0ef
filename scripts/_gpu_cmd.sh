# scratch GPU command of the current step (run via gpurun from the repo root)
set -o pipefail
O=gpurun_out/r02y; mkdir -p $O
for rep in 1 2; do
  for t in 4096 0; do
    OCTPT_DRAIN_RAYS=$t timeout -k 10 400 python3 bench.py --config C5 --steps 1 --warmup 1 --no-cpu-baseline > $O/b.json 2>> $O/err || exit 1
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/b.json "C5full drain$t" | tee -a $O/ab.txt
    OCTPT_DRAIN_RAYS=$t timeout -k 10 400 python3 bench.py --config C3 --steps 3 --warmup 1 --no-cpu-baseline > $O/b.json 2>> $O/err || exit 1
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" $O/b.json "C3 drain$t" | tee -a $O/ab.txt
  done
done
