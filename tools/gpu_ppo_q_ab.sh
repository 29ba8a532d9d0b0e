cd "${GRAFT_REPO_ROOT}" || exit 1
for r in 1 2 3; do for q in 320 352; do
  SALP_PAIR_STEADY_Q8=$q timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-lockstep --no-parity-check 2>/dev/null | grep '^{' | python -c "
import json,sys; d=json.load(sys.stdin)['ppo']; print('q=$q', round(d['value']/1e6,3), round(d['timing_s_max_over_ranks']['collect_s'],4))" >> gpurun_out/r4x_ppo_q.txt || exit 1
done; done
