#!/bin/bash
# One GPU session: parity tests, smoke, bench (JSON line), rocprofv3 kernel
# trace + stats of the bench.  Every GPU step has its own time limit; a crash
# or timeout stops the script there.  Outputs under gpurun_out/<TAG>_*.
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
    grep -v amdgpu.ids "gpurun_out/${TAG}_$name.log" | tail -n 6
    if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
if [ -z "$SKIP_TESTS" ]; then
    step pytest_gpu 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS}
    step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
fi
step bench 400 python -u bench.py ${BENCH_ARGS}
if [ -z "$SKIP_PROF" ]; then
    step prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/${TAG}_prof" -o run \
        -- python3 bench.py --no-cpu-baseline ${PROF_ARGS:---no-lockstep}
fi
