#!/bin/bash
# k_rollout_pair steady budget (SALP_PAIR_STEADY_Q8) x salp_collect chunk sweep at
# 32 768 envs (tools/collect_bench.py, both legs); one line per setting.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
OUT=${OUT:-gpurun_out/pair_qsweep.txt}
for q in ${QS:-300 380 480}; do for ch in ${CHUNKS:-256 384 512}; do
  SALP_PAIR_STEADY_Q8=$q SALP_COLLECT_CHUNK=$ch SALP_ROLLOUT_KERNEL=1 N="32768" K=32 timeout -k 10 100 \
      python tools/collect_bench.py 2>/dev/null | grep n_envs | sed "s/^/q=$q ch=$ch /" >> "$OUT" || exit 1
done; done
