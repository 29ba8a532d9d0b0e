#!/bin/bash
# A/B: tick-only and rollout bench for the product build and exp_build variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
for v in base ${VARIANTS}; do
    lib=""
    [ "$v" != base ] && lib="exp_build/libsalp_$v.so"
    SALP_LIB=$lib timeout -k 10 120 python tools/tick_bench.py > gpurun_out/var_${v}_tick.log 2>&1 || { echo "$v tick failed"; tail -3 gpurun_out/var_${v}_tick.log; exit 1; }
    SALP_LIB=$lib timeout -k 10 180 python bench.py --steps 8 --warmup 1 --no-cpu-baseline --no-lockstep ${BENCH_ARGS} > gpurun_out/var_${v}_bench.log 2>&1 || { echo "$v bench failed"; tail -3 gpurun_out/var_${v}_bench.log; exit 1; }
    python - "$v" <<'PY'
import json, sys
v = sys.argv[1]
t = json.loads(open(f"gpurun_out/var_{v}_tick.log").read().strip().splitlines()[-1])
b = json.loads(open(f"gpurun_out/var_{v}_bench.log").read().strip().splitlines()[-1])
print(f"{v:12s} tick_us/wave {t['us_per_tick_per_wave']:.3f}  rollout {b['value']/1e6:.2f} M env-steps/s  kernel {b['kernel_ms_per_launch']:.2f} ms")
PY
done
