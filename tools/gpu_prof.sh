#!/bin/bash
# Parity tests + rocprofv3 kernel trace of the bench + counter listing.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 secs=$2
    shift 2
    echo "== $name $(date +%T)"
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc $(date +%T)"
    tail -n 12 "gpurun_out/$name.log"
    if [ $rc -ge 2 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
step pytest_gpu 900 python -m pytest tests -m gpu -q ${PYTEST_ARGS}
step counters 120 rocprofv3 -L
step prof_trace 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline
