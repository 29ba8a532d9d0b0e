#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
set -o pipefail
for r in 1 2; do for c in 96 128 160 192; do
  timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-lockstep --chunk $c > gpurun_out/c2_$c$r.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/c2_$c$r.log').read().strip().splitlines()[-1]);print('chunk',$c,$r,round(d['value']/1e6,2),round(d['kernel_ms_per_launch'],3))"
done; done
