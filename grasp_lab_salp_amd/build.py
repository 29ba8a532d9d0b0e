"""Build libsalp.so in-tree for gfx950 (hipcc cross-compiles without a GPU).

    python -m grasp_lab_salp_amd.build [--verbose]
"""
import argparse
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRCS = [os.path.join(HERE, "csrc", f) for f in ("salp_kernels.hip", "salp_gae.hip", "salp_ppo.hip", "salp_ppo_mlp.hip",
                                               "salp_sort.hip", "salp_lstm.hip")]
OUT = os.path.join(HERE, "libsalp.so")
ARCH = os.environ.get("SALP_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

# Strict IEEE fp64: no FP contraction (explicit fma() only), no fast-math, so
# device results are bit-identical to the CPU oracle built with gcc.
FLAGS = ["-O3", "-std=c++17", f"--offload-arch={ARCH}", "-ffp-contract=off", "-fno-fast-math",
         "-fPIC", "-shared", "-Wall", "-Wno-unused-function"]


def deps():
    c = os.path.join(HERE, "csrc")
    return SRCS + [os.path.join(c, f) for f in os.listdir(c) if f.endswith(".h")] + [
        os.path.join(HERE, "..", "include", "salp.h")]


def up_to_date():
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(d) <= t for d in deps())


# Per-source scheduler choice: the PPO update's kernels run faster under the
# max-ILP machine scheduler (update -2 %), the rollout kernels slower (-3 %:
# profiles/r6_experiments.md r6z), so each source is compiled on its own.
FILE_FLAGS = {"salp_ppo_mlp.hip": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]}


def build(force=False, verbose=False, extra=(), out=None, file_flags=None):
    """out / file_flags: another output path and per-source flags (A / B builds,
    tools/build_variant.py); the product build takes neither."""
    if out is None and not force and up_to_date():
        return OUT
    out = out or OUT
    file_flags = FILE_FLAGS if file_flags is None else file_flags
    import tempfile
    from concurrent.futures import ThreadPoolExecutor
    compile_flags = [f for f in FLAGS if f != "-shared"]
    with tempfile.TemporaryDirectory(prefix="salp_build_") as tmp:
        objs = [os.path.join(tmp, os.path.basename(src) + ".o") for src in SRCS]
        cmds = [[HIPCC, *compile_flags, *file_flags.get(os.path.basename(src), []), *extra, "-c", "-o", obj, src]
                for src, obj in zip(SRCS, objs)]
        link = [HIPCC, f"--offload-arch={ARCH}", "-fPIC", "-shared", "-o", out + ".tmp", *objs]
        if verbose:
            for c in cmds + [link]:
                print(" ".join(c), flush=True)
        with ThreadPoolExecutor(max_workers=min(len(cmds), os.cpu_count() or 1)) as ex:
            for r in list(ex.map(lambda c: subprocess.run(c, capture_output=True, text=True), cmds)):
                if r.returncode:
                    raise subprocess.CalledProcessError(r.returncode, r.args, r.stdout, r.stderr)
                if r.stderr and verbose:
                    print(r.stderr, end="", flush=True)
        subprocess.run(link, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--resource-usage", action="store_true")
    a = ap.parse_args()
    extra = ["-Rpass-analysis=kernel-resource-usage"] if a.resource_usage else []
    print(build(force=a.force or a.resource_usage, verbose=a.verbose, extra=extra))
    sys.exit(0)
