set -e
mkdir -p gpurun_out/pvb
OCTPT_LIB=build_variants/pvb/liboctpt.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "preview" --timeout 300 --timeout-method thread > gpurun_out/pvb/pytest.log 2>&1 || { tail -40 gpurun_out/pvb/pytest.log; exit 1; }
tail -1 gpurun_out/pvb/pytest.log
for c in C3 C4 C5; do for v in cur pvb cur pvb; do
echo "$c $v $(OCTPT_LIB=build_variants/$v/liboctpt.so timeout -k 10 200 python -u scripts/spp_sweep.py $c 1 1 1 1 --preview 2>/dev/null | tail -1)"
done; done
