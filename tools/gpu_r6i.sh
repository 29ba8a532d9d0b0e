#!/bin/bash
# Round-6 call i: k_mlp_fwd_bwd as one block per network (actor / critic, 4
# waves, two blocks per CU) against the round's 8-wave block
# (exp_build/libsalp_base.so): the PPO tests, then bench_ppo.py A / B
# (update time, graphed) twice, and the kernel statistics of both builds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r6i
timeout -k 10 600 python -u -m pytest tests/test_gpu_ppo_mlp.py tests/test_gpu_gae_ppo.py tests/test_gpu_ppo_multirank.py tests/test_gpu_dropin.py -m gpu -x -v \
    --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 || { tail -60 gpurun_out/${T}_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/${T}_pytest_gpu.log
for r in 1 2; do
    SALP_LIB=exp_build/libsalp_base.so timeout -k 10 300 python tools/bench_ppo.py --n-steps 32 --iters 2 \
        > gpurun_out/${T}_ppo_base_$r.json 2> gpurun_out/${T}_ppo_base_$r.err || exit 1
    timeout -k 10 300 python tools/bench_ppo.py --n-steps 32 --iters 2 \
        > gpurun_out/${T}_ppo_new_$r.json 2> gpurun_out/${T}_ppo_new_$r.err || exit 1
    for v in base new; do
        python -c "import json;d=json.loads(open('gpurun_out/${T}_ppo_${v}_$r.json').read().strip().splitlines()[-1]);print('$v', {k: d[k] for k in ('value', 'timing_s') if k in d})"
    done
done
for v in base new; do
    if [ $v = base ]; then export SALP_LIB=exp_build/libsalp_base.so; else unset SALP_LIB; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_$v -o run -- \
        python3 tools/bench_ppo.py --n-steps 32 --iters 1 > gpurun_out/${T}_prof_$v.out 2>&1 || exit 1
done
unset SALP_LIB
for v in base new; do
    f=$(find gpurun_out/${T}_prof_$v -name 'run_kernel_stats.csv' | head -1)
    echo "== $v"; grep -E 'k_mlp' "$f" | cut -d, -f1-4
done
