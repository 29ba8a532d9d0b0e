#!/bin/bash
# Round-6 call l: k_mlp_fwd_bwd with the first tile's gather and the advantage
# partials issued before the weight staging and thread-0-only block sums
# (working tree) against HEAD (exp_build/libsalp_base.so, tools/build_base.sh):
# PPO tests, kernel statistics and bench_ppo.py of both, alternated.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r6l}
timeout -k 10 600 python -u -m pytest tests/test_gpu_ppo_mlp.py tests/test_gpu_gae_ppo.py tests/test_gpu_ppo_multirank.py -m gpu -x -v \
    --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 || { tail -60 gpurun_out/${T}_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/${T}_pytest_gpu.log
for r in 1 2; do
    for v in base new; do
        if [ $v = new ]; then unset SALP_LIB; else export SALP_LIB=${BASE_LIB:-exp_build/libsalp_base.so}; fi
        timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_${v}_$r -o run -- \
            python3 tools/bench_ppo.py --n-steps 32 --iters 1 > gpurun_out/${T}_prof_${v}_$r.out 2>&1 || exit 1
        f=$(find gpurun_out/${T}_prof_${v}_$r -name 'run_kernel_stats.csv' | head -1)
        echo "== $v $(grep -E 'k_mlp_fwd_bwd' "$f" | cut -d, -f2-4)"
    done
done
for r in 1 2; do
    for v in base new; do
        if [ $v = new ]; then unset SALP_LIB; else export SALP_LIB=${BASE_LIB:-exp_build/libsalp_base.so}; fi
        timeout -k 10 300 python tools/bench_ppo.py --n-steps 32 --iters 2 \
            > gpurun_out/${T}_ppo_${v}_$r.json 2> gpurun_out/${T}_ppo_${v}_$r.err || exit 1
        python -c "import json;d=json.loads(open('gpurun_out/${T}_ppo_${v}_$r.json').read().strip().splitlines()[-1]);print('$v', {k: d[k] for k in ('value', 'timing_s') if k in d})"
    done
done
