#!/bin/bash
# Experiments: (1) does a wave with 32 of 64 lanes active run the tick in half
# the time (k_tick_bench, 1024 waves either way); (2) jet-rate float32 arm
# gated vs not (bench A/B).  Outputs under gpurun_out/lanes_*.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { echo "== $*"; timeout -k 10 120 "$@" || exit 1; }
for r in 1 2; do
  N=65536 TICKS=4096 run python tools/tick_bench.py
  SALP_LIB=exp_build/libsalp_lpw32.so N=32768 TICKS=4096 run python tools/tick_bench.py
  SALP_LIB=exp_build/libsalp_nogate.so N=65536 TICKS=4096 run python tools/tick_bench.py
done
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -n 3
LIBS="product exp_build/libsalp_nogate.so" ROUNDS=2 STEPS=8 bash tools/gpu_libab.sh
