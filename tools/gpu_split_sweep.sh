#!/bin/bash
# config 5's collection on k_rollout_split: collection chunk x steady budget,
# measured on bench.py's PPO leg itself (round 5 tuned the pair kernel the same way).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
T=${TAG:-r6g}
for chunk in ${CHUNKS:-128 176 256}; do
    for q in ${QS:-340 450 560}; do
        SALP_COLLECT_CHUNK=$chunk SALP_SPLIT_COLLECT_Q8=$q timeout -k 10 300 python bench.py --steps 2 --warmup 1 \
            --no-lockstep --no-cpu-baseline --no-parity-check > gpurun_out/${T}_sweep.json 2>/dev/null || exit 1
        python -c "import json;d=json.loads(open('gpurun_out/${T}_sweep.json').read().strip().splitlines()[-1]);p=d['ppo'];print('chunk $chunk q $q', round(p['value']/1e6,3), round(p['timing_s_max_over_ranks']['collect_s'],4), round(p['timing_s_max_over_ranks']['train_s'],4))" | tee -a gpurun_out/${T}_sweep.txt
    done
done
