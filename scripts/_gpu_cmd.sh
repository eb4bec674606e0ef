# scratch GPU command of the current step (run via gpurun from the repo root)
set -o pipefail
mkdir -p gpurun_out/r02p
R=$PWD
echo "== lanes"; OCTPT_PROFILE_LANES=1 OCTPT_LIB=build_variants/prof/liboctpt.so timeout -k 10 300 python scripts/spp_sweep.py C3 64 --ktime 2>&1 | grep -E "spp|lanes" || exit 1
cd /tmp && export TMPDIR=/tmp
for lib in base cur; do
  if [ $lib = cur ]; then unset OCTPT_LIB; else export OCTPT_LIB=$R/build_variants/base/liboctpt.so; fi
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS -d $R/gpurun_out/r02p/sq_$lib -o run --output-format csv -- python3 $R/scripts/spp_sweep.py C3 64 > $R/gpurun_out/r02p/sq_$lib.log 2>&1 || exit 1
  python3 $R/scripts/pmc_summary.py $R/gpurun_out/r02p/sq_$lib 2>&1 | grep -E "extend|==" 
done
