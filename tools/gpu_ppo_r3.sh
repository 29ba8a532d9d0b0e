#!/bin/bash
# PPO session: the kept-graph experiment (tools/debug_ppo_graph_keep.py) and a
# config-5 learning trend (tools/bench_ppo.py --trend-iters).  Each step has
# its own time limit; a failure stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-r3p}
if [ -z "$SKIP_GRAPH" ]; then
    timeout -k 10 400 python -u tools/debug_ppo_graph_keep.py > gpurun_out/${TAG}_graph_keep.log 2>&1
    rc=$?; echo "graph_keep rc=$rc"; tail -n 6 gpurun_out/${TAG}_graph_keep.log; [ $rc -eq 0 ] || exit $rc
fi
if [ -z "$SKIP_TREND" ]; then
    timeout -k 10 500 python -u tools/bench_ppo.py --n-envs 32768 --n-steps ${N_STEPS:-256} --iters 2 \
        --trend-iters ${TREND:-24} --collect auto > gpurun_out/${TAG}_trend.json 2> gpurun_out/${TAG}_trend.err
    rc=$?; echo "trend rc=$rc"; tail -c 600 gpurun_out/${TAG}_trend.json; [ $rc -eq 0 ] || exit $rc
fi
