#!/bin/bash
# Sorted lock-step order: its parity tests, then lock-step rates in env order
# vs sorted at 65 536 and 262 144 envs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/sort_tests.log 2>&1; rc=$?; tail -n 3 gpurun_out/sort_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/lockstep_bench.py | tee gpurun_out/sort_bench.log
