#!/bin/bash
# Round-6 call m: the update kernels.  HEAD (exp_build/libsalp_base.so, ABI 12:
# one-block k_mlp_apply, the previous k_mlp_fwd_bwd prologue) against the
# working tree with SALP_PPO_APPLY=one (r6l's k_mlp_fwd_bwd prologue /
# epilogue only) and with the many-block clip + Adam (default): PPO tests,
# kernel statistics and bench_ppo.py, alternated.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${T:-r6m}
timeout -k 10 600 python -u -m pytest tests/test_gpu_ppo_mlp.py tests/test_gpu_gae_ppo.py tests/test_gpu_ppo_multirank.py -m gpu -x -v \
    --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 || { tail -60 gpurun_out/${T}_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/${T}_pytest_gpu.log
run() {   # variant: env for it
    case $1 in
        base) export SALP_LIB=exp_build/libsalp_base.so SALP_AB_OLD_ABI=1; unset SALP_PPO_APPLY ;;
        one) unset SALP_LIB SALP_AB_OLD_ABI; export SALP_PPO_APPLY=one ;;
        blocks) unset SALP_LIB SALP_AB_OLD_ABI SALP_PPO_APPLY ;;
    esac
}
for r in 1 2; do
    for v in base one blocks; do
        run $v
        timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof_${v}_$r -o run -- \
            python3 tools/bench_ppo.py --n-steps 32 --iters 1 > gpurun_out/${T}_prof_${v}_$r.out 2>&1 || exit 1
        f=$(find gpurun_out/${T}_prof_${v}_$r -name 'run_kernel_stats.csv' | head -1)
        echo "== $v $r"; grep -E 'k_mlp' "$f" | cut -d, -f1-4 | sed 's/(anonymous namespace):://g' | cut -c1-120
    done
done
for r in 1 2; do
    for v in base one blocks; do
        run $v
        timeout -k 10 300 python tools/bench_ppo.py --n-steps 32 --iters 2 \
            > gpurun_out/${T}_ppo_${v}_$r.json 2> gpurun_out/${T}_ppo_${v}_$r.err || exit 1
        python -c "import json;d=json.loads(open('gpurun_out/${T}_ppo_${v}_$r.json').read().strip().splitlines()[-1]);print('$v', {k: d[k] for k in ('value', 'timing_s') if k in d})"
    done
done
