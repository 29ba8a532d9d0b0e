#!/bin/bash
# Lock-step (drop-in step path) throughput of the product build and variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for v in base ${VARIANTS}; do
    lib=""
    [ "$v" != base ] && lib="exp_build/libsalp_$v.so"
    SALP_LIB=$lib timeout -k 10 180 python bench.py --steps 4 --warmup 1 --no-cpu-baseline > gpurun_out/lock_$v.log 2>&1 || { tail -3 gpurun_out/lock_$v.log; exit 1; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/lock_$v.log').read().strip().splitlines()[-1]); print('$v', 'rollout', round(d['value']/1e6,2), 'lockstep', round(d['lockstep_env_steps_per_sec']/1e6,2))"
done
