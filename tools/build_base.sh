#!/bin/bash
# Build libsalp.so from a git revision (default HEAD) into exp_build/libsalp_base.so,
# for A/B runs against the working tree (SALP_LIB=exp_build/libsalp_base.so).
set -e
cd "$(dirname "$0")/.."
REV=${1:-HEAD}
D=exp_build/basesrc
rm -rf "$D" && mkdir -p "$D"
git archive "$REV" grasp_lab_salp_amd/csrc include | tar -x -C "$D"
FLAGS=$(python -c "from grasp_lab_salp_amd import build as B; print(' '.join(B.FLAGS))")
SRCS=$(python -c "from grasp_lab_salp_amd import build as B; import os; print(' '.join('$D/grasp_lab_salp_amd/csrc/' + os.path.basename(s) for s in B.SRCS))")
/opt/rocm/bin/hipcc $FLAGS -o exp_build/libsalp_base.so $SRCS
rm -rf "$D"
echo exp_build/libsalp_base.so
