#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
set -o pipefail
for r in 1 2; do for q in 336 360 384 408; do
  SALP_STEADY_Q8=$q timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-lockstep > gpurun_out/q2_$q$r.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/q2_$q$r.log').read().strip().splitlines()[-1]);print('q',$q,$r,round(d['value']/1e6,2),round(d['kernel_ms_per_launch'],3))"
done; done
