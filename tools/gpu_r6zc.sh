#!/bin/bash
# Round-6 call zc: salp_kernels.hip under other machine schedulers
# (exp_lib/libsalp_{minreg,memclause}.so: iterative-minreg, max-memory-clause)
# against the product build: bench.py (headline and PPO leg), alternated twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
T=r6zc
for r in 1 2; do
    for v in base minreg memclause; do
        if [ $v = base ]; then unset SALP_LIB; else export SALP_LIB=exp_lib/libsalp_$v.so; fi
        timeout -k 10 400 python bench.py --no-cpu-baseline --no-parity-check > gpurun_out/${T}_${v}_$r.json \
            2> gpurun_out/${T}_${v}_$r.err || { tail -5 gpurun_out/${T}_${v}_$r.err; exit 1; }
        python -c "import json;d=json.loads(open('gpurun_out/${T}_${v}_$r.json').read().strip().splitlines()[-1]);p=d['ppo'];print('$v', round(d['value']/1e6,2), round((d.get('steady_state_env_steps_per_sec') or 0)/1e6,2), 'ppo', round(p['value']/1e6,2), p['timing_s_max_over_ranks'])"
    done
done
