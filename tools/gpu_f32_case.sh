cd "${GRAFT_REPO_ROOT}" || exit 1
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q -k float32_shape --timeout 100 --timeout-method thread > gpurun_out/f32_product.log 2>&1
SALP_LIB=exp_build/libsalp_nogate.so timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q -k float32_shape --timeout 100 --timeout-method thread > gpurun_out/f32_nogate.log 2>&1
tail -5 gpurun_out/f32_product.log gpurun_out/f32_nogate.log
