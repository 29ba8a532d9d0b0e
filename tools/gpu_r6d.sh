#!/bin/bash
# Round-6 call d: the GPU suite on the build with the all-angle roll / pitch
# sin / cos and k_rollout_split, then A / B runs: config 5's collection on the
# pair vs the split kernel (tools/collect_bench.py, 32 768 envs), and bench.py
# on the round-5 arithmetic (exp_build/libsalp_base.so, commit 9c73e83) vs this
# build, and this build with the split kernel as the PPO leg's two-wave kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r6d
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/${T}_pytest_gpu.log 2>&1 || { tail -60 gpurun_out/${T}_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/${T}_pytest_gpu.log
for r in 1 2; do
    for k in 1 2; do
        N=32768 K=32 KERNEL=$k timeout -k 10 200 python -u tools/collect_bench.py >> gpurun_out/${T}_collect_k$k.jsonl 2>/dev/null || exit 1
        tail -1 gpurun_out/${T}_collect_k$k.jsonl
    done
done
for r in 1 2; do
    SALP_LIB=exp_build/libsalp_base.so timeout -k 10 400 python bench.py --no-cpu-baseline --no-parity-check \
        > gpurun_out/${T}_bench_base_$r.json 2> gpurun_out/${T}_bench_base_$r.err || exit 1
    timeout -k 10 400 python bench.py --no-cpu-baseline --no-parity-check \
        > gpurun_out/${T}_bench_new_$r.json 2> gpurun_out/${T}_bench_new_$r.err || exit 1
    SALP_TWO_WAVE_KERNEL=split timeout -k 10 400 python bench.py --no-cpu-baseline --no-parity-check \
        > gpurun_out/${T}_bench_split_$r.json 2> gpurun_out/${T}_bench_split_$r.err || exit 1
    for v in base new split; do
        python -c "import json;d=json.loads(open('gpurun_out/${T}_bench_${v}_$r.json').read().strip().splitlines()[-1]);p=d['ppo'];print('$v', round(d['value']/1e6,2), round((d.get('steady_state_env_steps_per_sec') or 0)/1e6,2), round(d['lockstep_env_steps_per_sec']/1e6,2), 'ppo', round(p['value']/1e6,2), p['timing_s_max_over_ranks'])"
    done
done
