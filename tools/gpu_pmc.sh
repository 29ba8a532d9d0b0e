#!/bin/bash
# PMC passes over a short bench run (one counter group per pass, kernel trace
# only; no sys/runtime trace domains).  Outputs under gpurun_out/pmc_<tag>_*.
# Each pass is SIGKILLed after 90 s (a counter request the hardware cannot
# serve hangs rocprofv3, SIGTERM included).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r1}
ARGS=${BENCH_ARGS:---steps 2 --warmup 1 --no-cpu-baseline --no-lockstep --no-parity-check --no-ppo}
PASSES=${PASSES:-fetch write waves mix}
pass() {  # name counters...
    local name=$1
    shift
    echo "== pmc $name $(date +%T)"
    timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-trace --output-format csv \
        -d "gpurun_out/pmc_${TAG}_${name}" -o run -- python3 bench.py $ARGS \
        > "gpurun_out/pmc_${TAG}_${name}.log" 2>&1
    local rc=$?
    echo "== pmc $name rc=$rc"
    tail -n 3 "gpurun_out/pmc_${TAG}_${name}.log"
    if [ $rc -ne 0 ]; then echo "stopping (rc=$rc)"; exit $rc; fi
}
for p in $PASSES; do
    case $p in
        fetch) pass fetch FETCH_SIZE ;;
        write) pass write WRITE_SIZE ;;
        waves) pass waves SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE ;;
        mix) pass mix SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 ;;
        stall) pass stall SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS_SMEM SQ_INST_CYCLES_SMEM SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES ;;
        salu) pass salu SQ_INSTS_SALU SQ_INST_CYCLES_SALU SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY ;;
    esac
done
