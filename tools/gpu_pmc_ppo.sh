#!/bin/bash
# PMC passes over a short config-5 PPO run (tools/bench_ppo.py, n_steps 32): one
# counter group per pass, kernel trace only.  Outputs gpurun_out/pmc_<tag>_ppo_*.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r3}
pass() {  # name counters...
    local name=$1
    shift
    echo "== pmc $name $(date +%T)"
    timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv \
        -d "gpurun_out/pmc_${TAG}_ppo_${name}" -o run -- python3 tools/bench_ppo.py --n-steps 32 --iters 1 \
        > "gpurun_out/pmc_${TAG}_ppo_${name}.log" 2>&1
    local rc=$?
    echo "== pmc $name rc=$rc"
    if [ $rc -ne 0 ]; then tail -n 3 "gpurun_out/pmc_${TAG}_ppo_${name}.log"; echo "stopping (rc=$rc)"; exit $rc; fi
}
pass lds SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY
pass mix SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE
python3 - <<'PY'
import csv, glob, collections, os, re
tag = os.environ.get("TAG", "r3")
for path in sorted(glob.glob(f"gpurun_out/pmc_{tag}_ppo_*/run_counter_collection.csv")):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        mm = re.search(r"(k_\w+)", r["Kernel_Name"])
        k = mm.group(1) if mm else r["Kernel_Name"][:40]
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k in ("k_mlp_fwd_bwd", "k_mlp_apply", "k_mlp_reduce"):
        if k in agg:
            print(k, {c: round(sum(v) / len(v)) for c, v in agg[k].items()})
PY
rm -f gpurun_out/pmc_${TAG}_ppo_*/run_kernel_trace.csv gpurun_out/pmc_${TAG}_ppo_*/run_counter_collection.csv
