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


def build(force=False, verbose=False, extra=()):
    if not force and up_to_date():
        return OUT
    cmd = [HIPCC, *FLAGS, *extra, "-o", OUT + ".tmp", *SRCS]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--resource-usage", action="store_true")
    a = ap.parse_args()
    extra = ["-Rpass-analysis=kernel-resource-usage"] if a.resource_usage else []
    print(build(force=a.force or a.resource_usage, verbose=a.verbose, extra=extra))
    sys.exit(0)
