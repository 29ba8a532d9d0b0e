#!/bin/bash
# k_rollout steady budget sweep (SALP_STEADY_Q8: steady ticks per full tick of a
# wave's chunk budget, x256) on the product build; one bench line per value.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for r in $(seq ${ROUNDS:-2}); do
    for q in ${QS:-360 400 440 480 520}; do
        SALP_STEADY_Q8=$q timeout -k 10 120 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline \
            --no-parity-check --no-ppo --no-lockstep ${BENCH_ARGS} > gpurun_out/qs.log 2>&1 || { tail -n 5 gpurun_out/qs.log; exit 1; }
        python -c "import json;d=json.loads(open('gpurun_out/qs.log').read().strip().splitlines()[-1]);print('q', $q, round(d['value']/1e6,3), round(d['kernel_ms_per_launch'],3))" | tee -a gpurun_out/q_sweep.txt
    done
done
