#!/bin/bash
# Round-3 GPU session: selected GPU tests (PYTEST_SEL), then the bench line.
# Every GPU step has its own time limit; a failure stops the script there.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r3}
step() {  # name seconds command...
    local name=$1 secs=$2
    shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc $(date +%T)"
    grep -v amdgpu.ids "gpurun_out/${TAG}_$name.log" | tail -n 8
    if [ $rc -ne 0 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
if [ -n "$PYTEST_SEL" ]; then
    step pytest 900 python -u -m pytest $PYTEST_SEL -x -v -s --timeout 300 --timeout-method thread
fi
if [ -z "$SKIP_BENCH" ]; then
    step bench 400 python -u bench.py ${BENCH_ARGS}
fi
