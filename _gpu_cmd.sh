set -e
mkdir -p gpurun_out/ppop
rm -f gpurun_out/ppop/sweep.jsonl
SPP=256 scripts/extend_sweep.sh gpurun_out/ppop/sweep.jsonl "OCTPT_EXTEND=default" "OCTPT_LIB=build_variants/ppop/liboctpt.so" "OCTPT_EXTEND=default" "OCTPT_LIB=build_variants/ppop/liboctpt.so"
