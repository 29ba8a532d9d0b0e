#!/bin/bash
# Cold-block layout check: GPU parity suite, smoke, bench (its lock-step leg
# runs k_step_random on the state left by 23 rollout launches: the round-1
# fault scenario), then the PMC traffic and instruction passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
TAG=${TAG:-r2d} SKIP_PROF=1 bash tools/gpu_round.sh || exit $?
TAG=${TAG:-r2d} PASSES="fetch write waves mix" bash tools/gpu_pmc.sh || exit $?
python3 tools/pmc_summary.py ${TAG:-r2d}
