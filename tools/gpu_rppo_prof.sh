#!/bin/bash
# RecurrentPPO config-5 rate and its rocprofv3 kernel stats (TAG=...).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-rppo}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o run -- \
    python3 -u tools/bench_ppo.py --recurrent --n-steps ${NSTEPS:-64} --iters 1 > gpurun_out/${T}.log 2> gpurun_out/${T}.err
rc=$?; echo "== rppo_prof rc=$rc"
find gpurun_out/${T}_prof -type f ! -name "*kernel_stats.csv" -delete   # the traces exceed the 64 MiB copy-back limit
du -ah gpurun_out | sort -h | tail -n 5; tail -c 600 gpurun_out/${T}.log; exit $rc
