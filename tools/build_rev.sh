#!/bin/bash
# Build libsalp.so of a git revision into exp_build/libsalp_<name>.so (A/B runs
# against the working tree: SALP_LIB=exp_build/libsalp_<name>.so).
#   tools/build_rev.sh REV NAME
set -e
cd "$(dirname "$0")/.."
REV=$1; NAME=${2:-$1}
D=exp_build/rev_$NAME
rm -rf "$D" && mkdir -p "$D"
git archive "$REV" grasp_lab_salp_amd/csrc include | tar -x -C "$D"
python - "$D" "exp_build/libsalp_$NAME.so" <<'PY'
import subprocess, sys, os
sys.path.insert(0, os.getcwd())
from grasp_lab_salp_amd import build as B
d, out = sys.argv[1], sys.argv[2]
srcs = [os.path.join(d, "grasp_lab_salp_amd", "csrc", f) for f in ("salp_kernels.hip", "salp_gae.hip", "salp_ppo.hip",
        "salp_ppo_mlp.hip", "salp_sort.hip", "salp_lstm.hip")]
subprocess.run([B.HIPCC, *B.FLAGS, "-o", out, *srcs], check=True)
print(out)
PY
