#!/bin/bash
# rocprofv3 kernel stats + FETCH_SIZE / WRITE_SIZE passes of the GAE scan
# (tools/gae_bench.py: three shapes, 21 launches each).  Outputs gpurun_out/gae_*.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gae_prof -o run \
    -- python3 tools/gae_bench.py > gpurun_out/gae_prof.log 2>&1 || { tail -3 gpurun_out/gae_prof.log; exit 1; }
grep '^{' gpurun_out/gae_prof.log
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/gae_pmc_$c -o run \
        -- python3 tools/gae_bench.py > gpurun_out/gae_pmc_$c.log 2>&1 || { tail -3 gpurun_out/gae_pmc_$c.log; exit 1; }
done
echo done
