#!/bin/bash
# PMC passes over tools/pair_pmc_probe.py (k_rollout vs k_rollout_pair).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-pp}
pass() {
    local name=$1
    shift
    timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-trace --output-format csv \
        -d "gpurun_out/pmc_${TAG}_${name}" -o run -- python3 tools/pair_pmc_probe.py > "gpurun_out/pmc_${TAG}_${name}.log" 2>&1
    local rc=$?
    echo "== pmc $name rc=$rc"
    if [ $rc -ne 0 ]; then tail -n 3 "gpurun_out/pmc_${TAG}_${name}.log"; exit $rc; fi
}
pass waves SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE
pass mix SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY
