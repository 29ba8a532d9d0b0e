#!/bin/bash
# PMC of the PPO update kernels (k_mlp_fwd_bwd / k_mlp_reduce / k_mlp_adam)
# over a short config-5 run (tools/bench_ppo.py, n_steps 32, one iteration),
# one counter group per pass, kernel trace only.  GRAPHS=0 runs the minibatch
# steps eagerly (PPO(use_graphs=False)); the kernels are the same.
# Outputs gpurun_out/pmcu_<TAG>_<group>/ and a summary on stdout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-r6}
EXTRA=""
[ "${GRAPHS:-0}" = "0" ] && EXTRA="--no-graphs"
pass() {  # name counters...
    local name=$1
    shift
    echo "== pmc $name $(date +%T)"
    timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-trace --output-format csv \
        -d "gpurun_out/pmcu_${TAG}_${name}" -o run -- python3 tools/bench_ppo.py --n-steps 32 --iters 1 $EXTRA \
        > "gpurun_out/pmcu_${TAG}_${name}.log" 2>&1
    local rc=$?
    echo "== pmc $name rc=$rc"
    if [ $rc -ne 0 ]; then tail -n 30 "gpurun_out/pmcu_${TAG}_${name}.log"; echo "stopping (rc=$rc)"; exit $rc; fi
}
for g in ${GROUPS_:-mix lds fetch write}; do
    case $g in
        mix) pass mix SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE ;;
        lds) pass lds SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY ;;
        fetch) pass fetch FETCH_SIZE ;;
        write) pass write WRITE_SIZE ;;
        flops) pass flops SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_TRANS_F32 ;;
    esac
done
python3 tools/pmc_kernels_summary.py pmcu_${TAG} k_mlp_fwd_bwd k_mlp_reduce k_mlp_adam k_mlp_apply k_mlp_adv_sums \
    k_rollout_split k_rollout_pair k_rollout k_gae > gpurun_out/pmcu_${TAG}_summary.json || exit 1
# the raw per-dispatch CSVs are too large to come back (gpurun_out <= 64 MiB)
rm -rf gpurun_out/pmcu_${TAG}_*/
echo "== done $(date +%T)"
