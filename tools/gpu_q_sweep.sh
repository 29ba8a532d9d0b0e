#!/bin/bash
# Steady-budget sweep of the product k_rollout and the NaN fix without re-seating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
T=${TAG:-r2o}
b() {  # label env...
    local label=$1; shift
    timeout -k 10 150 env "$@" python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-lockstep ${BENCH_ARGS} \
        > gpurun_out/${T}_b_$label.log 2>&1 || { echo "bench $label failed"; tail -5 gpurun_out/${T}_b_$label.log; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/${T}_b_$label.log').read().strip().splitlines()[-1]);print('$label',round(d['value']/1e6,2),round(d['kernel_ms_per_launch'],3))"
}
b nanonly SALP_LIB=exp_build/libsalp_nanonly.so
for q in ${QS:-288 320 352 384 416}; do b q$q SALP_STEADY_Q8=$q; done
b nanonly2 SALP_LIB=exp_build/libsalp_nanonly.so
b q320b SALP_STEADY_Q8=320
