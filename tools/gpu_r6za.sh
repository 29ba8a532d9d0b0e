#!/bin/bash
# Round-6 call za: the library built per source with the PPO update's source
# under the max-ILP scheduler (grasp_lab_salp_amd/build.py FILE_FLAGS) against
# the one-command build of the same sources (exp_lib/libsalp_base.so,
# tools/build_base.sh): the PPO tests, then bench.py alternated twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r6za
timeout -k 10 600 python -u -m pytest tests/test_gpu_ppo_mlp.py tests/test_gpu_gae_ppo.py tests/test_gpu_ppo_multirank.py -m gpu -x -v \
    --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 || { tail -60 gpurun_out/${T}_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/${T}_pytest_gpu.log
for r in 1 2; do
    for v in base new; do
        if [ $v = base ]; then export SALP_LIB=exp_lib/libsalp_base.so; else unset SALP_LIB; fi
        timeout -k 10 400 python bench.py --no-cpu-baseline --no-parity-check > gpurun_out/${T}_${v}_$r.json \
            2> gpurun_out/${T}_${v}_$r.err || { tail -5 gpurun_out/${T}_${v}_$r.err; exit 1; }
        python -c "import json;d=json.loads(open('gpurun_out/${T}_${v}_$r.json').read().strip().splitlines()[-1]);p=d['ppo'];print('$v', round(d['value']/1e6,2), round((d.get('steady_state_env_steps_per_sec') or 0)/1e6,2), 'ppo', round(p['value']/1e6,2), p['timing_s_max_over_ranks'])"
    done
done
