set -e
mkdir -p gpurun_out/lsph
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "render_parity or golden or megakernel" --timeout 120 --timeout-method thread > gpurun_out/lsph/pytest.log 2>&1 || { tail -40 gpurun_out/lsph/pytest.log; exit 1; }
tail -2 gpurun_out/lsph/pytest.log
rm -f gpurun_out/lsph/sweep.jsonl
SPP=64 scripts/extend_sweep.sh gpurun_out/lsph/sweep.jsonl "OCTPT_LIB=build_variants/base/liboctpt.so" "OCTPT_LIB=build_variants/lsph/liboctpt.so" "OCTPT_LIB=build_variants/base/liboctpt.so" "OCTPT_LIB=build_variants/lsph/liboctpt.so"
