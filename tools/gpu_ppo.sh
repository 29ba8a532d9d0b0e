#!/bin/bash
# PPO GPU session: the PPO tests, the config-5 rate (tools/bench_ppo.py) with a
# rocprofv3 kernel summary, and the torch-path kept-graph check at n_steps 32 x
# 10 epochs.  Each GPU step has its own time limit; a failure stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r3p}
step() {  # name seconds command...
    local name=$1 secs=$2
    shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc $(date +%T)"
    grep -v amdgpu.ids "gpurun_out/${TAG}_$name.log" | tail -n ${TAIL:-4} | cut -c1-600
    if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
step tests 600 python -u -m pytest ${PPO_TESTS:-tests/test_gpu_ppo_mlp.py tests/test_gpu_ppo_multirank.py tests/test_gpu_gae_ppo.py} -x -v --timeout 300 --timeout-method thread
step ppo 300 python -u tools/bench_ppo.py --n-envs 32768 --n-steps 256 --iters 2
if [ -z "$SKIP_PROF" ]; then
    step ppo_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/${TAG}_ppo_prof" -o run \
        -- python3 tools/bench_ppo.py --n-envs 32768 --n-steps 256 --iters 1
fi
if [ -z "$SKIP_GRAPH" ]; then
    VARIANTS=side N_STEPS=32 N_EPOCHS=10 UPDATES=8 step graph_keep 400 python -u tools/debug_ppo_graph_keep.py
fi
