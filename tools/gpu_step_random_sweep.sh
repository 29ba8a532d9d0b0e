#!/bin/bash
# salp_step_random(k): chained kernel (chunk 128 / 64 / 32) vs lock-step kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
set -o pipefail
run() { timeout -k 10 120 env "$@" python -u tools/step_random_sweep.py >> gpurun_out/step_random_sweep.jsonl 2>> gpurun_out/step_random_sweep.err; }
run SALP_STEP_RANDOM_LOCKSTEP=1 && run SALP_STEP_RANDOM_CHUNK=128 && run SALP_STEP_RANDOM_CHUNK=64 \
  && run SALP_STEP_RANDOM_CHUNK=32 && run N=32768 SALP_STEP_RANDOM_LOCKSTEP=1 && run N=32768 SALP_STEP_RANDOM_CHUNK=64
cat gpurun_out/step_random_sweep.jsonl
