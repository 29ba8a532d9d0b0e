#!/bin/bash
# salp_collect (policy inside the chained kernel) vs lock-step collection:
# GPU tests, then config-5 PPO (32 768 envs) with both collections at n_steps
# 32 (trend) and 2048.  Outputs under gpurun_out/<TAG>_*.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r2s}
timeout -k 10 300 python -u -m pytest tests/test_gpu_collect.py -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_collect_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_collect_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_collect_tests.log
[ -n "$TESTS_ONLY" ] && exit 0
for c in chained lockstep; do
  timeout -k 10 300 python -u tools/bench_ppo.py --collect $c --n-steps 32 --iters 2 --trend-iters ${TREND:-8} > gpurun_out/${TAG}_ppo32_$c.json 2> gpurun_out/${TAG}_ppo32_$c.err || { tail -5 gpurun_out/${TAG}_ppo32_$c.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_ppo32_$c.json').read().strip().splitlines()[-1]);print('$c n_steps 32:', round(d['value']/1e6,3), d['timing_s'], [ (r['iteration'], round(r['ep_return_mean'] or 0,1), r['diverged_envs'], round(r['vf_loss'],2)) for r in d['trend']])"
done
if [ -n "$N2048" ]; then
  timeout -k 10 400 python -u tools/bench_ppo.py --collect chained --n-steps 2048 --iters 1 > gpurun_out/${TAG}_ppo2048_chained.json 2> gpurun_out/${TAG}_ppo2048_chained.err || { tail -5 gpurun_out/${TAG}_ppo2048_chained.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_ppo2048_chained.json').read().strip().splitlines()[-1]);print('chained n_steps 2048:', round(d['value']/1e6,3), d['timing_s'], d['losses'], d['diverged_envs_reset'])"
fi
