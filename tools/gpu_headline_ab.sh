#!/bin/bash
# Headline A/B of libsalp builds: ROUNDS alternations of bench.py's rollout leg
# (no cpu baseline, lock-step paths, parity replay or PPO leg) per library.
# LIBS="product exp_build/libsalp_x.so ..."; one line per run in $OUT.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
OUT=${OUT:-gpurun_out/headline_ab.txt}
for r in $(seq ${ROUNDS:-2}); do
    for lib in ${LIBS:-product}; do
        l=$lib; [ "$lib" = product ] && l=""
        v=$(SALP_AB_OLD_ABI=1 SALP_LIB=$l timeout -k 10 300 python bench.py --no-cpu-baseline --no-lockstep --no-parity-check --no-ppo \
            2>/dev/null | grep '^{' | python -c "import json,sys; d=json.load(sys.stdin); print(round(d['value']/1e6,2), round(d['kernel_ms_per_launch'],3))") || exit 1
        echo "$lib $v" >> "$OUT"
    done
done
