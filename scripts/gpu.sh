#!/bin/bash
# The one GPU-box driver (run through gpurun from the repo root; replaces round 4's one-off gpu_r04_*.sh):
#   scripts/gpu.sh TAG TASK [TASK ...]
# Outputs go to gpurun_out/TAG/.  Tasks run in order, each under its own time limit; the first failure ends
# the call (no later GPU step runs after a fault, abort or timeout).
#   suite                 the whole -m gpu suite (as the driver runs it)          -> gputest.log
#   tests:SPEC            pytest on SPEC (a file / node id / "-k EXPR"), -m gpu    -> tests_<n>.log
#   smoke                 __graft_entry__.smoke()                                  -> smoke.log
#   bench:CFG[:STEPS]     one bench line of CFG (CPU baseline + issued probe)      -> bench_CFG.json
#   fast:CFG[:STEPS]      the same without the CPU baseline                         -> bench_CFG.json
#   stats:CFG[:STEPS[:LIB]]  rocprofv3 --kernel-trace --stats of that bench command  -> stats_CFG/
#                         (LIB = build_variants/NAME/liboctpt.so runs that build -> stats_CFG_NAME/)
#   pmc:CFG[:N]           FETCH_SIZE / WRITE_SIZE / TCC passes: the one-step bench (N = 1) or rank 0's shard of
#                         an N-way split (scripts/shard_step.py) -> pmc_CFG[_nN].json, also into profiles/
#   sq:CFG[:LIB]          the SQ counter pass of the one-step bench (of that build)  -> sq_CFG[_NAME]/
#   shard:CFG[:NS]        scripts/shard_emulation.py (NS = "1_2_4_8", the default)  -> shard_CFG.json
#   n8                    bench.py --gpus 8 --dist-backend gloo (the driver's N = 8 command on one GPU)
#   nrank:N[:CFG[:STEPS]] the same at N ranks with the CPU baseline, wall time recorded -> nrank_N_CFG.json/.time
#   run:CMD               any command (no colons in it), e.g. "python3 scripts/stale_hit_probe.py slotleak_check"
#                                                                                 -> run_<n>.log
#   ab:CFG/SPP,...:LIB,...  scripts/ab.sh A/B of library builds ("cur" = the in-tree library) -> ab_<n>.txt
#   abenv:CFG/SPP,...:VAR+VAR  scripts/ab_env.sh A/B of builds and env settings (VAR = LIB or LIB|ENV=V,ENV=V) -> ab_<n>.txt
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
PYT="python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread"
n=0
fail() { echo "FAILED: $1" >&2; [ -n "$2" ] && tail -30 "$2" >&2; exit 1; }
for task in "$@"; do
  n=$((n + 1))
  IFS=: read -r kind a b c <<< "$task"
  echo "[$(date +%T)] $task" >&2
  case $kind in
    suite) timeout -k 10 900 $PYT tests > $O/gputest.log 2>&1 || fail "$task" $O/gputest.log; tail -2 $O/gputest.log ;;
    tests) timeout -k 10 600 $PYT $a > $O/tests_$n.log 2>&1 || fail "$task" $O/tests_$n.log; tail -2 $O/tests_$n.log ;;
    smoke) timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || fail "$task" $O/smoke.log
           cat $O/smoke.log ;;
    bench|fast)
      X=""; [ $kind = fast ] && X="--no-cpu-baseline"
      timeout -k 10 600 python3 bench.py --config ${a:-C3} --steps ${b:-5} --warmup 1 $X > $O/bench_${a:-C3}.json \
          2> $O/bench_${a:-C3}.err || fail "$task" $O/bench_${a:-C3}.err
      cat $O/bench_${a:-C3}.json ;;
    stats)
      V=$a; if [ -n "$c" ]; then V=${a}_$(basename $(dirname $c)); fi
      (cd /tmp && export TMPDIR=/tmp && if [ -n "$c" ]; then export OCTPT_LIB=$R/$c; fi \
          && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/stats_$V -o run \
          --output-format csv -- python3 $R/bench.py --config $a --steps ${b:-5} --warmup 1 --no-cpu-baseline \
          > $O/stats_$V.json 2> $O/stats_$V.err) || fail "$task" $O/stats_$V.err
      cat $O/stats_$V.json ;;
    pmc)
      N=${b:-1}; SUF=""; [ $N -gt 1 ] && SUF=_n$N
      if [ $N -gt 1 ]; then CMD="$R/scripts/shard_step.py --config $a --n $N --k 0"; SRC="python3 scripts/shard_step.py --config $a --n $N --k 0 (rank 0's shard of an $N-way split, one step)"
      else CMD="$R/bench.py --config $a --steps 1 --warmup 0 --no-cpu-baseline --no-issued"; SRC="python3 bench.py --config $a --steps 1 (one full step)"; fi
      P=$O/pmc_$a$SUF
      for pass in "fetch FETCH_SIZE" "write WRITE_SIZE" "tcc TCC_HIT_sum TCC_MISS_sum"; do
        set -- $pass; d=$1; shift
        (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --pmc "$@" -d $P/$d -o run --output-format csv \
            -- python3 $CMD > $P.$d.out 2> $P.$d.err) || fail "$task $d" $P.$d.err
      done
      python3 scripts/pmc_traffic.py $P/fetch $P/write $a $O/pmc_$a$SUF.json 1.0 "calibrated by tools/fetch_calib.hip (profiles/fetch_calib.json): scattered 8-B and 16-B reads are counted at 64 B per request, factor 1" $P/tcc "$SRC" || fail "$task summary"
      cp $O/pmc_$a$SUF.json profiles/pmc_$a$SUF.json
      cat $P.fetch.out | tail -1 ;;
    sq)  # sq:CFG[:LIB]  (LIB = build_variants/NAME/liboctpt.so -> sq_CFG_NAME/)
      V=$a; if [ -n "$b" ]; then V=${a}_$(basename $(dirname $b)); fi
      (cd /tmp && export TMPDIR=/tmp && if [ -n "$b" ]; then export OCTPT_LIB=$R/$b; fi \
          && timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
          SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS -d $O/sq_$V -o run \
          --output-format csv -- python3 $R/bench.py --config $a --steps 1 --warmup 0 --no-cpu-baseline --no-issued \
          > $O/sq_$V.out 2> $O/sq_$V.err) || fail "$task" $O/sq_$V.err ;;
    shard)
      NS=${b:-1_2_4_8}
      timeout -k 10 600 python3 scripts/shard_emulation.py --config $a --ns ${NS//_/ } > $O/shard_$a.json \
          2> $O/shard_$a.err || fail "$task" $O/shard_$a.err
      tail -1 $O/shard_$a.json ;;
    n8)
      timeout -k 10 600 python3 bench.py --gpus 8 --dist-backend gloo --steps 2 --warmup 1 --no-cpu-baseline \
          > $O/bench_n8_gloo.json 2> $O/bench_n8_gloo.err || fail "$task" $O/bench_n8_gloo.err
      cat $O/bench_n8_gloo.json ;;
    nrank)  # nrank:N[:CFG[:STEPS]]: the driver's N-rank command as gloo ranks time-sharing this GPU, CPU baseline
            # included; the command's wall time goes to nrank_N_CFG.time
      t0=$(date +%s.%N)
      timeout -k 10 900 python3 bench.py --gpus $a --config ${b:-C3} --dist-backend gloo --steps ${c:-2} --warmup 1 \
          > $O/nrank_${a}_${b:-C3}.json 2> $O/nrank_${a}_${b:-C3}.err || fail "$task" $O/nrank_${a}_${b:-C3}.err
      echo "{\"command\": \"python3 bench.py --gpus $a --config ${b:-C3} --dist-backend gloo --steps ${c:-2} --warmup 1\", \"wall_s\": $(python3 -c "print(round($(date +%s.%N) - $t0, 1))")}" > $O/nrank_${a}_${b:-C3}.time
      cat $O/nrank_${a}_${b:-C3}.time; tail -c 600 $O/nrank_${a}_${b:-C3}.json ;;
    ab)
      timeout -k 10 1000 bash scripts/ab.sh "$(echo ${a//,/ } | tr / :)" ${b//,/ } > $O/ab_$n.txt 2>&1 || fail "$task" $O/ab_$n.txt
      cat $O/ab_$n.txt ;;
    abenv)  # abenv:CFG/SPP,...:VAR+VAR+...  (VAR = LIB or LIB|ENV=V,ENV2=V; scripts/ab_env.sh)
      IFS=+ read -r -a VARS <<< "$b"
      timeout -k 10 1000 bash scripts/ab_env.sh "$(echo ${a//,/ } | tr / :)" "${VARS[@]}" > $O/ab_$n.txt 2>&1 || fail "$task" $O/ab_$n.txt
      cat $O/ab_$n.txt ;;
    run) timeout -k 10 600 bash -c "$a" > $O/run_$n.log 2>&1 || fail "$task" $O/run_$n.log; tail -5 $O/run_$n.log ;;
    *) fail "unknown task $task" ;;
  esac
done
echo "[$(date +%T)] done" >&2
