#!/bin/bash
# Bench PPO leg under VAR=value for each of VALUES, ROUNDS alternations; lines in $OUT.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
OUT=${OUT:-gpurun_out/ppo_env_sweep.txt}
for r in $(seq ${ROUNDS:-2}); do
    for v in $VALUES; do
        env "$VAR=$v" timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-lockstep \
            --no-parity-check 2>/dev/null | grep '^{' | python -c "
import json,sys; d=json.load(sys.stdin)['ppo']; print('$VAR=$v', round(d['value']/1e6,3), round(d['timing_s_max_over_ranks']['collect_s'],4))" >> "$OUT" || exit 1
    done
done
