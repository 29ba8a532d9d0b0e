#!/bin/bash
# The collection's chunk x pair steady budget on both measures, one box: bench.py's
# PPO leg (config 5, n_steps 256) and tools/collect_bench.py (32 env-steps per call).
# CQS="chunk:q ..."; ROUNDS alternations; one line per run in $OUT.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
OUT=${OUT:-gpurun_out/collect_cq_ab.txt}
for r in $(seq ${ROUNDS:-2}); do
    for cq in ${CQS:-176:340 192:400}; do
        c=${cq%%:*}; q=${cq##*:}
        p=$(SALP_COLLECT_CHUNK=$c SALP_PAIR_COLLECT_Q8=$q timeout -k 10 300 python bench.py --steps 2 --warmup 1 \
            --no-cpu-baseline --no-lockstep --no-parity-check 2>/dev/null | grep '^{' | python -c "
import json, sys
d = json.load(sys.stdin)['ppo']
print(round(d['value'] / 1e6, 3), round(d['timing_s_max_over_ranks']['collect_s'], 4))") || exit 1
        b=$(SALP_COLLECT_CHUNK=$c SALP_PAIR_COLLECT_Q8=$q SALP_ROLLOUT_KERNEL=1 N=32768 timeout -k 10 200 \
            python tools/collect_bench.py 2>/dev/null | grep n_envs | python -c "
import json, sys
print(json.load(sys.stdin)['collect_1'])") || exit 1
        echo "c=$c q=$q ppo $p collect_bench $b" >> "$OUT"
    done
done
