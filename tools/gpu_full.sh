#!/bin/bash
# Full GPU session: parity tests, smoke, bench, rocprofv3 stats, PMC passes
# and their summary, PPO/GAE bench.  TAG names the outputs; every GPU step has
# its own time limit and a failure stops the script there.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r1}
step() {  # name seconds command...
    local name=$1 secs=$2
    shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc $(date +%T)"
    grep -v amdgpu.ids "gpurun_out/${TAG}_$name.log" | tail -n 4
    if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
if [ -z "$SKIP_TESTS" ]; then
    step pytest_gpu 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
    step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
fi
step bench 400 python -u bench.py
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/${TAG}_prof" -o run \
    -- python3 bench.py --no-cpu-baseline --steps 10
if [ -z "$SKIP_PMC" ]; then
    TAG=$TAG bash tools/gpu_pmc.sh || exit 1
    step pmc_summary 60 python tools/pmc_summary.py "$TAG"
fi
if [ -z "$SKIP_PPO" ]; then
    step bench_ppo 400 python -u tools/bench_ppo.py
fi
