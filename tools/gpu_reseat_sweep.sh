#!/bin/bash
# k_rollout re-seating: steady-budget (SALP_STEADY_Q8) x chunk sweep, bench only.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
T=${TAG:-r2m}
b() {  # label chunk env...
    local label=$1 chunk=$2; shift 2
    timeout -k 10 150 env "$@" python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-lockstep --chunk $chunk \
        > gpurun_out/${T}_b_$label.log 2>&1 || { echo "bench $label failed"; tail -5 gpurun_out/${T}_b_$label.log; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/${T}_b_$label.log').read().strip().splitlines()[-1]);print('$label',round(d['value']/1e6,2),round(d.get('kernel_ms_per_launch'),3))"
}
b old128 128 SALP_LIB=exp_build/libsalp_noreseat.so
for q in ${QS:-128 192 256 288 320}; do b q${q}_c128 128 SALP_STEADY_Q8=$q; done
for c in ${CS:-64 96 192 256}; do b q${Q:-288}_c$c $c SALP_STEADY_Q8=${Q:-288}; done
b old128b 128 SALP_LIB=exp_build/libsalp_noreseat.so
