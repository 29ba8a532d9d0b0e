#!/bin/bash
# tools/debug_ppo_graph_keep.py over collection / loss / GEMM variants (torch
# PPO path with the minibatch graph kept across updates); one JSON line each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
run() { env VARIANTS=side UPDATES=4 "$@" timeout -k 10 120 python -u tools/debug_ppo_graph_keep.py 2>/dev/null | grep variant >> gpurun_out/gk.jsonl || exit 1; }
if [ -n "$SWEEP5" ]; then
    run N_STEPS=32 N_EPOCHS=10 COLLECT_STREAM=1
    run N_STEPS=32 N_EPOCHS=10 COLLECT_STREAM=1 TORCH_BLAS_PREFER_HIPBLASLT=0
elif [ -n "$SWEEP4" ]; then
    run N_STEPS=32 N_EPOCHS=10 ACT_PATCH=nogemm VALUE_PATCH=1
    run N_STEPS=32 N_EPOCHS=10 VALUE_PATCH=1
elif [ -n "$SWEEP3" ]; then
    run N_STEPS=32 N_EPOCHS=10 NO_COLLECT=1
    run N_STEPS=32 N_EPOCHS=10 NO_COLLECT=1 COLLECT=chained
    run N_STEPS=32 N_EPOCHS=10 SYNC_ALLOC=1
elif [ -n "$SWEEP2" ]; then
    run N_STEPS=32 N_EPOCHS=10 NO_GUARD=1
    run N_STEPS=32 N_EPOCHS=10 ACT_PATCH=nogemm
    run N_STEPS=32 N_EPOCHS=10 ACT_PATCH=nogemm NO_GUARD=1
    run N_STEPS=32 N_EPOCHS=10 FUSED_LOSS=0 NO_GUARD=1
else
    run N_STEPS=8 N_EPOCHS=10
    run N_STEPS=32 N_EPOCHS=2
    run N_STEPS=32 N_EPOCHS=10 SPLITK=0
    run N_STEPS=32 N_EPOCHS=10 FUSED_LOSS=0
    run N_STEPS=32 N_EPOCHS=10 TORCH_BLAS_PREFER_HIPBLASLT=0
    run N_STEPS=32 N_EPOCHS=10 COLLECT=chained
fi
python -c "
import json
for l in open('gpurun_out/gk.jsonl'):
    d=json.loads(l); print({k:v for k,v in d['env'].items() if v}, [(c['graph_equals_eager'], c['graph_grads_finite']) for c in d['checks']], d['params_finite'])"
