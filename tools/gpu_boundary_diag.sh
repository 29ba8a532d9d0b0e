#!/bin/bash
# Where the rollout's time goes besides the tick: tick-only kernel with PMC
# issue counters, then a chunk sweep of the rollout (boundary cost vs idle).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_tick_pmc.sh || exit 1
for c in 32 64 96 128 192 256; do
    timeout -k 10 200 python bench.py --steps 8 --warmup 1 --no-cpu-baseline --no-lockstep --chunk $c > gpurun_out/sweep_$c.log 2>&1 || { tail -3 gpurun_out/sweep_$c.log; exit 1; }
    python3 -c "import json;d=json.loads(open('gpurun_out/sweep_$c.log').read().strip().splitlines()[-1]);print('chunk $c', round(d['value']/1e6,3), round(d['kernel_ms_per_launch'],3))"
done
