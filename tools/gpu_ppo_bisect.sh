#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_gae_ppo.py tests/test_gpu_parity.py -x -q -k "sorted or order" --timeout 200 --timeout-method thread 2>&1 | tail -15
for m in 0 1; do
  timeout -k 10 300 python -u tools/bench_ppo.py --n-steps 32 --iters 1 --trend-iters 4 --lockstep-order $m > gpurun_out/bis_$m.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/bis_$m.json').read().strip().splitlines()[-1]);print('order $m', [ (r['iteration'], r['vf_loss'], r['diverged_envs']) for r in d['trend']])"
done
