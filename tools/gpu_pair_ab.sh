#!/bin/bash
# Pair-kernel variants: parity (tests/test_gpu_pair.py + test_gpu_collect.py) per
# variant, then ROUNDS alternations of tools/collect_bench.py at 32 768 envs.
# LIBS="product exp_build/libsalp_x.so ..."; one line per run in $OUT.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
OUT=${OUT:-gpurun_out/pair_ab.txt}
for lib in ${LIBS:-product}; do
    l=$lib; [ "$lib" = product ] && l=""
    SALP_LIB=$l timeout -k 10 300 python -u -m pytest tests/test_gpu_pair.py tests/test_gpu_collect.py -x -q \
        --timeout 200 --timeout-method thread > gpurun_out/pair_ab_tests.log 2>&1
    rc=$?
    echo "$lib tests rc=$rc $(tail -n 1 gpurun_out/pair_ab_tests.log)" >> "$OUT"
    [ $rc -eq 0 ] || exit $rc
done
for r in $(seq ${ROUNDS:-2}); do
    for lib in ${LIBS:-product}; do
        l=$lib; [ "$lib" = product ] && l=""
        SALP_LIB=$l SALP_ROLLOUT_KERNEL=1 N=32768 timeout -k 10 200 python tools/collect_bench.py 2>/dev/null \
            | grep n_envs | sed "s|^|$lib |" >> "$OUT" || exit 1
    done
done
