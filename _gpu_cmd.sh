set -e
mkdir -p gpurun_out/popflat
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/popflat/pytest.log 2>&1 || { tail -40 gpurun_out/popflat/pytest.log; exit 1; }
tail -2 gpurun_out/popflat/pytest.log
rm -f gpurun_out/popflat/sweep.jsonl
SPP=64 scripts/extend_sweep.sh gpurun_out/popflat/sweep.jsonl "OCTPT_LIB=build_variants/push1/liboctpt.so" "OCTPT_LIB=build_variants/popflat/liboctpt.so" "OCTPT_LIB=build_variants/push1/liboctpt.so" "OCTPT_LIB=build_variants/popflat/liboctpt.so"
