#!/bin/bash
# k_rollout chunk sweep of the headline bench (rollout leg only) on the product
# build; CHUNKS / ROUNDS; one line per run appended to $OUT.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
OUT=${OUT:-gpurun_out/chunk_sweep.txt}
for r in $(seq ${ROUNDS:-2}); do
    for ch in ${CHUNKS:-96 128 160 192}; do
        timeout -k 10 120 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-parity-check \
            --no-ppo --no-lockstep --chunk $ch > gpurun_out/cs.log 2>&1 || { tail -n 5 gpurun_out/cs.log; exit 1; }
        python -c "import json;d=json.loads(open('gpurun_out/cs.log').read().strip().splitlines()[-1]);print('chunk', $ch, round(d['value']/1e6,3), round(d['kernel_ms_per_launch'],3))" | tee -a "$OUT"
    done
done
