#!/bin/bash
# A/B: round-1 rollout (noreseat) / re-seating only (nonan) / product
# (re-seating + NaN angles on the small sin/cos path).  Tests first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r2n}
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_randomization.py \
    -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || exit $rc
b() {  # label env...
    local label=$1; shift
    timeout -k 10 150 env SALP_STEADY_Q8=320 "$@" python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline \
        > gpurun_out/${T}_b_$label.log 2>&1 || { echo "bench $label failed"; tail -5 gpurun_out/${T}_b_$label.log; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/${T}_b_$label.log').read().strip().splitlines()[-1]);print('$label',round(d['value']/1e6,2),round(d['kernel_ms_per_launch'],3),'lock',round(d['lockstep_env_steps_per_sec']/1e6,2),'div',d['divergence']['diverged_envs_at_end'])"
}
for r in 1 2; do
  b old$r SALP_LIB=exp_build/libsalp_noreseat.so
  b nonan$r SALP_LIB=exp_build/libsalp_nonan.so
  b prod$r
done
