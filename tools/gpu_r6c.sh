#!/bin/bash
# Round-6 call c: split probes (r5ao variant, product), the update kernels' PMC
# (eager minibatch steps, summarised on the box), then the round-5 profiler
# crash reproduced: one PMC pass over the whole bench (PPO leg included, graphed
# update) -- the last step, nothing runs after it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
T=r6c
SALP_LIB=exp_build/libsalp_r5ao.so ORACLE_LIB=exp_build/r5ao/oracle/libsalp_oracle.so timeout -k 10 400 \
    python -u tools/split_probe.py > gpurun_out/${T}_split_r5ao.json 2> gpurun_out/${T}_split_r5ao.err || exit 1
timeout -k 10 400 python -u tools/split_probe.py > gpurun_out/${T}_split_product.json 2> gpurun_out/${T}_split_product.err || exit 1
echo split probes done
TAG=$T GRAPHS=0 GROUPS_="mix lds fetch write flops" bash tools/gpu_pmc_update.sh || exit 1
echo "== whole-bench PMC pass (last step) $(date +%T)"
PYTHONFAULTHANDLER=1 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv \
    -d gpurun_out/pmcb_${T} -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-lockstep \
    --no-parity-check > gpurun_out/pmcb_${T}.log 2>&1
rc=$?
echo "whole-bench rc=$rc"
python3 tools/pmc_kernels_summary.py pmcb_${T} > gpurun_out/pmcb_${T}_summary.json
rm -rf gpurun_out/pmcb_${T}/
grep -v "^W2026\|amdgpu.ids" gpurun_out/pmcb_${T}.log | tail -60
