#!/bin/bash
# Executed-instruction attribution of k_rollout by ablation: for every library
# in LIBS ("product" = grasp_lab_salp_amd/libsalp.so, else a path built by
# tools/build_variant.py), one headline bench run (rollout leg only) and one
# PMC pass of the instruction counters on the same command.  Outputs under
# gpurun_out/ablate_<TAG>/; summarise with tools/ablate_summary.py TAG.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
TAG=${TAG:-r5a}
OUT=gpurun_out/ablate_$TAG
mkdir -p "$OUT"
ARGS="--steps ${STEPS:-6} --warmup 2 --no-cpu-baseline --no-lockstep --no-parity-check --no-ppo"
COUNTERS="SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64"
for lib in ${LIBS:-product}; do
    name=$(basename "$lib" .so); name=${name#libsalp_}
    l=$lib; [ "$lib" = product ] && l=""
    echo "== $name bench $(date +%T)"
    SALP_LIB=$l timeout -k 10 240 python bench.py $ARGS > "$OUT/${name}_bench.log" 2>&1 || { echo "bench rc=$?"; tail -n 5 "$OUT/${name}_bench.log"; exit 1; }
    grep '^{' "$OUT/${name}_bench.log" > "$OUT/${name}_bench.json"
    echo "== $name pmc $(date +%T)"
    SALP_LIB=$l timeout -s KILL 120 rocprofv3 --pmc $COUNTERS --kernel-trace --output-format csv \
        -d "$OUT/${name}_pmc" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-lockstep \
        --no-parity-check --no-ppo > "$OUT/${name}_pmc.log" 2>&1 || { echo "pmc rc=$?"; tail -n 5 "$OUT/${name}_pmc.log"; exit 1; }
done
echo "== done $(date +%T)"
