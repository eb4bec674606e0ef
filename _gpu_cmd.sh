set -e
mkdir -p gpurun_out/slp
rm -f gpurun_out/slp/sweep.jsonl
SPP=64 scripts/extend_sweep.sh gpurun_out/slp/sweep.jsonl "OCTPT_LIB=build_variants/cur/liboctpt.so" "OCTPT_LIB=build_variants/slp/liboctpt.so" "OCTPT_LIB=build_variants/cur/liboctpt.so" "OCTPT_LIB=build_variants/slp/liboctpt.so"
