#!/bin/bash
# Re-seating k_rollout: rollout parity tests, then bench A/B against the
# previous kernel (exp_build/libsalp_noreseat.so) and a steady-budget sweep.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r2l}
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_randomization.py \
    -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; tail -4 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
b() {  # label env... -- bench args
    local label=$1; shift
    timeout -k 10 150 env "$@" python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-lockstep \
        > gpurun_out/${T}_b_$label.log 2>&1 || { echo "bench $label failed"; tail -5 gpurun_out/${T}_b_$label.log; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/${T}_b_$label.log').read().strip().splitlines()[-1]);print('$label',round(d['value']/1e6,2),d.get('kernel_ms_per_launch'))"
}
b old SALP_LIB=exp_build/libsalp_noreseat.so
b new SALP_STEADY_Q8=448
b old2 SALP_LIB=exp_build/libsalp_noreseat.so
b new2 SALP_STEADY_Q8=448
for q in 320 384 512 576; do b q$q SALP_STEADY_Q8=$q; done
