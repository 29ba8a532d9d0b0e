#!/bin/bash
# Joint sweep of k_rollout's steady budget q (SALP_STEADY_Q8) and chunk on the
# headline bench (rollout leg only), product build; "q:chunk" pairs in QC,
# ROUNDS alternations; one line per run appended to $OUT.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
OUT=${OUT:-gpurun_out/qc_sweep.txt}
for r in $(seq ${ROUNDS:-2}); do
    for qc in ${QC:-560:96 560:128}; do
        q=${qc%%:*}; ch=${qc##*:}
        SALP_STEADY_Q8=$q timeout -k 10 120 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline \
            --no-parity-check --no-ppo --no-lockstep --chunk $ch > gpurun_out/qc.log 2>&1 || { tail -n 5 gpurun_out/qc.log; exit 1; }
        python -c "import json;d=json.loads(open('gpurun_out/qc.log').read().strip().splitlines()[-1]);print('q', $q, 'chunk', $ch, round(d['value']/1e6,3), round(d['kernel_ms_per_launch'],3))" | tee -a "$OUT"
    done
done
