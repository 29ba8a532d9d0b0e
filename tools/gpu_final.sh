#!/bin/bash
# Round artefacts: GPU parity suite, smoke, bench (JSON), rocprofv3 kernel
# stats of the bench, PMC passes (traffic / instruction mix / waves) and the
# host-sanitizer run.  TAG names the outputs (gpurun_out/<TAG>_*).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
TAG=${TAG:-r2h}
TAG=$TAG PROF_ARGS="--steps 5 --warmup 1 --no-lockstep --no-cpu-baseline" bash tools/gpu_round.sh || exit $?
TAG=$TAG PASSES="fetch write waves mix" bash tools/gpu_pmc.sh || exit $?
python3 tools/pmc_summary.py $TAG > /dev/null || exit 1
bash tools/gpu_sanitize.sh || exit $?
