#!/bin/bash
# Settled steady ticks: GPU tests, then bench A/B against exp_build/libsalp_base.so.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ab3_tests.log 2>&1; rc=$?; tail -3 gpurun_out/ab3_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in new base; do
    if [ $v = base ]; then export SALP_LIB=exp_build/libsalp_base.so; else unset SALP_LIB; fi
    timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/ab3_$v$r.log 2>&1 || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/ab3_$v$r.log').read().strip().splitlines()[-1]);print('$v',$r,round(d['value']/1e6,2),round(d['kernel_ms_per_launch'],3),round(d['lockstep_env_steps_per_sec']/1e6,2),round(d['step_given_actions_env_steps_per_sec']/1e6,2))"
  done
done
