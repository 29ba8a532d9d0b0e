"""Build an experimental variant of libsalp.so from patched copies of csrc/
(A/B measurements; the product build is grasp_lab_salp_amd/build.py).

    python tools/build_variant.py NAME 'old1=>new1' ['old2=>new2' ...]

Each argument replaces one exact snippet in salp_kernels.hip or salp_device.h
(the file that contains it).  Output: exp_build/libsalp_NAME.so; run with
SALP_LIB=exp_build/libsalp_NAME.so.
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from grasp_lab_salp_amd import build as B  # noqa: E402


def main():
    name, reps = sys.argv[1], sys.argv[2:]
    d = os.path.join(ROOT, "exp_build", name)
    if os.path.exists(d):
        shutil.rmtree(d)
    shutil.copytree(os.path.join(ROOT, "grasp_lab_salp_amd", "csrc"), os.path.join(d, "grasp_lab_salp_amd", "csrc"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(d, "include"))
    files = [os.path.join(d, "grasp_lab_salp_amd", "csrc", f) for f in ("salp_kernels.hip", "salp_device.h", "salp_pair.h", "salp_gae.hip", "salp_math.h",
                                                                          "salp_ppo.hip", "salp_ppo_mlp.hip")]
    for r in reps:
        old, new = r.split("=>", 1)
        old, new = old.replace("\\n", "\n"), new.replace("\\n", "\n")
        hit = [f for f in files if old in open(f).read()]
        if len(hit) != 1 or open(hit[0]).read().count(old) != 1:
            raise SystemExit(f"snippet must occur exactly once: {old!r}")
        s = open(hit[0]).read().replace(old, new)
        open(hit[0], "w").write(s)
    out = os.path.join(ROOT, "exp_build", f"libsalp_{name}.so")
    srcs = [os.path.join(d, "grasp_lab_salp_amd", "csrc", f) for f in ("salp_kernels.hip", "salp_gae.hip", "salp_ppo.hip", "salp_ppo_mlp.hip", "salp_sort.hip",
                                                                     "salp_lstm.hip")]
    extra = os.environ.get("EXTRA_FLAGS", "").split()   # e.g. "-mllvm -amdgpu-sched-strategy=max-ilp"
    subprocess.run([B.HIPCC, *B.FLAGS, *extra, "-o", out, *srcs], check=True)
    print(out)


if __name__ == "__main__":
    main()
