#!/bin/bash
# A/B of libsalp builds on one box: LIBS="product exp_build/libsalp_x.so ..."
# (product = the in-tree build), ROUNDS alternations of bench.py (chained
# rollout + lock-step).  TESTS=1 runs the GPU parity suite on the product first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
    timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        > gpurun_out/ab_tests.log 2>&1; rc=$?; tail -n 2 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq ${ROUNDS:-2}); do
    for lib in ${LIBS:-product}; do
        l=$lib; [ "$lib" = product ] && l=""
        SALP_LIB=$l timeout -k 10 180 python bench.py --steps ${STEPS:-8} --warmup 1 --no-cpu-baseline --no-parity-check \
            > gpurun_out/ab.log 2>&1 || { tail -n 5 gpurun_out/ab.log; exit 1; }
        python -c "import json;d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]);print('$lib', round(d['value']/1e6,3), round(d['lockstep_env_steps_per_sec']/1e6,3), d['kernel_ms_per_launch'], round(d.get('steady_state_env_steps_per_sec') or 0, -5)/1e6)"
    done
done
