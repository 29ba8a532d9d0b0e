#!/bin/bash
# Round-3 GPU session: PMC passes of the headline kernel, the config-5
# learning trend, the torch-graph keep experiment and the salp_collect
# policy-cost A/B (SALP_LIB variants from tools/build_variant.py).
# Every GPU step has its own time limit; a failure stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r3h}
if [ -z "$SKIP_PMC" ]; then
    TAG=$TAG bash tools/gpu_pmc.sh || exit $?
fi
if [ -z "$SKIP_TREND" ]; then
    timeout -k 10 300 python -u tools/bench_ppo.py --n-envs 32768 --n-steps 256 --iters 2 \
        --trend-iters ${TREND:-30} --collect auto > gpurun_out/${TAG}_trend.json 2> gpurun_out/${TAG}_trend.err
    rc=$?; echo "trend rc=$rc"; tail -c 300 gpurun_out/${TAG}_trend.json; [ $rc -eq 0 ] || exit $rc
fi
if [ -z "$SKIP_GRAPH" ]; then
    UPDATES=4 timeout -k 10 300 python -u tools/debug_ppo_graph_keep.py > gpurun_out/${TAG}_graph_keep.log 2>&1
    rc=$?; echo "graph_keep rc=$rc"; tail -n 6 gpurun_out/${TAG}_graph_keep.log; [ $rc -eq 0 ] || exit $rc
fi
for lib in ${COLLECT_LIBS:-}; do
    for c in ${CHUNKS:-128 384}; do
        l=$lib; [ "$lib" = product ] && l=""
        SALP_LIB=$l SALP_COLLECT_CHUNK=$c timeout -k 10 200 python -u tools/collect_bench.py > gpurun_out/${TAG}_cb.jsonl 2>/dev/null
        rc=$?; [ $rc -eq 0 ] || { echo "collect_bench $lib rc=$rc"; exit $rc; }
        python -c "import json;[print('$lib','chunk',$c,d['n_envs'],d['collect_0'],d['collect_1'],d['rollout_cap_1'],d['step_random_1']) for d in map(json.loads,open('gpurun_out/${TAG}_cb.jsonl'))]" | tee -a gpurun_out/${TAG}_collect_ab.txt
    done
done
