#!/bin/bash
# PMC passes over the bench's PPO leg (config 5: salp_collect on
# the auto two-wave kernel, k_rollout_split<true> from round 6, at 32 768 envs, n_steps 256), one counter group per
# pass, kernel trace only; summarise with
#   python tools/pmc_summary.py TAG --kernel 'k_rollout_split<true>' --symbol k_rollout_splitILb1EE \
#       --config-json '{"n_envs": 32768, "n_steps": 256}' --suffix pmc_collect_summary
# (the PPO leg runs two collections: warm-up and timed; the summary keeps the timed one).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r5c}
ARGS="--steps 1 --warmup 0 --no-cpu-baseline --no-lockstep --no-parity-check"
# PROBE=1: profile tools/collect_pmc_probe.py (salp_collect alone) instead of the bench
CMD="bench.py $ARGS"
[ "${PROBE:-0}" = 1 ] && CMD="tools/collect_pmc_probe.py"
pass() {  # name counters...
    local name=$1
    shift
    echo "== pmc $name $(date +%T)"
    SALP_BENCH_PPO_GRAPHS=0 timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-trace --output-format csv \
        -d "gpurun_out/pmc_${TAG}_${name}" -o run -- python3 $CMD \
        > "gpurun_out/pmc_${TAG}_${name}.log" 2>&1
    local rc=$?
    echo "== pmc $name rc=$rc"
    if [ $rc -ne 0 ]; then tail -n 3 "gpurun_out/pmc_${TAG}_${name}.log"; exit $rc; fi
}
for p in ${PASSES:-fetch write waves mix}; do
    case $p in
        fetch) pass fetch FETCH_SIZE ;;
        write) pass write WRITE_SIZE ;;
        waves) pass waves SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE ;;
        mix) pass mix SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 ;;
    esac
done
