#!/bin/bash
# Config-5 PPO leg over the collection chunk x the pair steady budget (env overrides), two alternations.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=${OUT:-gpurun_out/ppo_cq_sweep.txt}
for r in 1 2; do
  for c in ${CHUNKS:-160 192 224}; do
    for q in ${QS:-360 400 440}; do
      v=$(SALP_COLLECT_CHUNK=$c SALP_PAIR_STEADY_Q8=$q timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-lockstep --no-parity-check 2>/dev/null | grep "^{" | python -c "import json,sys; d=json.load(sys.stdin)['ppo']; t=d['timing_s_max_over_ranks']; print(round(d['value']/1e6,3), round(t['collect_s'],4))") || exit 1
      echo "c=$c q=$q $v" >> $OUT
    done
  done
done
