#!/bin/bash
# Round-6 call b: the tumbling-regime GPU tests, the step-wave suite (k_step_wave
# now marks a timed-out env invalid), the split probes of the r5ao variant and
# of the product, the update kernels' PMC with eager minibatch steps, and last
# one PMC pass with the graphed update (the round-5 SIGSEGV; nothing runs after).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r6b
timeout -k 10 600 python -u -m pytest tests/test_gpu_tumble.py tests/test_gpu_step_wave.py \
    tests/test_gpu_parity.py::test_device_math_equals_oracle_math -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/${T}_pytest.log 2>&1 || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -3 gpurun_out/${T}_pytest.log
SALP_LIB=exp_build/libsalp_r5ao.so ORACLE_LIB=exp_build/r5ao/oracle/libsalp_oracle.so timeout -k 10 400 \
    python -u tools/split_probe.py > gpurun_out/${T}_split_r5ao.json 2> gpurun_out/${T}_split_r5ao.err || exit 1
timeout -k 10 400 python -u tools/split_probe.py > gpurun_out/${T}_split_product.json 2> gpurun_out/${T}_split_product.err || exit 1
echo split probes done
TAG=$T GRAPHS=0 bash tools/gpu_pmc_update.sh || exit 1
echo "== graphed PMC pass (last step) $(date +%T)"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES --kernel-trace --output-format csv -d gpurun_out/pmcu_${T}_graphed -o run \
    -- python3 tools/bench_ppo.py --n-steps 32 --iters 1 > gpurun_out/pmcu_${T}_graphed.log 2>&1
echo "graphed rc=$?"
tail -40 gpurun_out/pmcu_${T}_graphed.log
