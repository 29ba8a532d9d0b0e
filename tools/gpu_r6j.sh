#!/bin/bash
# Round-6 call j: k_mlp_fwd_bwd's phase profile (tools/mlp_phase_prof.py) on
# the 8-wave two-network block (base) and the 4-wave one-network blocks (new).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base new; do
    SALP_LIB=exp_build/libsalp_mlpprof_$v.so timeout -k 10 300 python tools/mlp_phase_prof.py \
        > gpurun_out/r6j_mlpprof_$v.json 2> gpurun_out/r6j_mlpprof_$v.err || { tail -20 gpurun_out/r6j_mlpprof_$v.err; exit 1; }
    echo "== $v"; cat gpurun_out/r6j_mlpprof_$v.json
done
