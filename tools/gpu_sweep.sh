#!/bin/bash
# GPU parity tests, then bench sweeps over rollout knobs (no CPU baseline).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
    local name=$1 secs=$2
    shift 2
    timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    grep -v amdgpu.ids "gpurun_out/$name.log" | tail -n 4
    if [ $rc -ge 2 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
if [ -z "$SKIP_TESTS" ]; then run pytest_gpu 900 python -m pytest tests -m gpu -q -x; fi
for c in ${CHUNKS:-16 32 64}; do
    run "bench_chunk$c" 300 python bench.py --steps 6 --warmup 1 --no-cpu-baseline --chunk "$c" ${BENCH_EXTRA}
done
