#!/bin/bash
# One GPU session: parity tests, smoke, short bench.  Every GPU step has its
# own time limit; a crash or timeout (rc >= 2) stops the script there.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name seconds command...
    local name=$1 secs=$2
    shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc $(date +%T)"
    tail -n 8 "gpurun_out/$name.log"
    if [ $rc -ge 2 ]; then
        echo "stopping after $name (rc=$rc)"
        exit $rc
    fi
    return 0
}
step pytest_gpu 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python bench.py --steps "${BENCH_STEPS:-10}" --warmup 2
