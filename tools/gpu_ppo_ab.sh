#!/bin/bash
# Config-5 PPO leg A/B of libsalp builds: ROUNDS alternations of bench.py with
# a short rollout leg, printing the PPO leg's env-steps/s and phase times.
# LIBS="product exp_build/libsalp_x.so ..."; one line per run in $OUT.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
OUT=${OUT:-gpurun_out/ppo_ab.txt}
for r in $(seq ${ROUNDS:-2}); do
    for lib in ${LIBS:-product}; do
        l=$lib; [ "$lib" = product ] && l=""
        v=$(SALP_AB_OLD_ABI=1 SALP_LIB=$l timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-cpu-baseline \
            --no-lockstep --no-parity-check 2>/dev/null | grep '^{' | python -c "
import json, sys
d = json.load(sys.stdin)['ppo']
t = d.get('timing_s_max_over_ranks', {})
print(round(d.get('value', d.get('env_steps_per_sec', 0)) / 1e6, 3), round(t.get('collect_s', 0), 4), round(t.get('train_s', 0), 4))") || exit 1
        echo "$lib $v" >> "$OUT"
    done
done
