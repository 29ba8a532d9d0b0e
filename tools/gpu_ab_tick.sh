#!/bin/bash
# Parity suite on the product build, then tick-only + rollout A/B against
# LIBS (SALP_LIB override) on the same box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
rc=$?; tail -n 2 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || exit $rc
for lib in ${LIBS}; do
    l=$lib; [ "$lib" = product ] && l=""
    SALP_LIB=$l timeout -k 10 120 python tools/tick_bench.py > gpurun_out/tick_ab.log 2>&1 || { tail -3 gpurun_out/tick_ab.log; exit 1; }
    echo "$lib tick $(python3 -c "import json;print(round(json.loads(open('gpurun_out/tick_ab.log').read().strip().splitlines()[-1])['us_per_tick_per_wave'],4))")"
done
ROUNDS=${ROUNDS:-2} STEPS=10 LIBS="${LIBS}" bash tools/gpu_libab.sh
