"""Build exp_build/libsalp_mlpprof.so: k_mlp_fwd_bwd with s_memtime marks
after every __syncthreads() of the kernel (phase i = the time up to barrier
i) and salp_debug_mlp_prof to read them (tools/mlp_phase_prof.py)."""
import os
import re
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from grasp_lab_salp_amd import build as B  # noqa: E402

NPH = 24


def main():
    d = os.path.join(ROOT, "exp_build", "mlpprof")
    if os.path.exists(d):
        shutil.rmtree(d)
    shutil.copytree(os.path.join(ROOT, "grasp_lab_salp_amd", "csrc"), os.path.join(d, "grasp_lab_salp_amd", "csrc"))
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(d, "include"))
    p = os.path.join(d, "grasp_lab_salp_amd", "csrc", "salp_ppo_mlp.hip")
    s = open(p).read()
    head = "void k_mlp_fwd_bwd(RowArgs a) {"
    a = s.index(head) + len(head)
    b = s.index("\n}\n", a)
    body = s[a:b]
    n = [0]

    def mark(m):
        i = n[0]
        n[0] += 1
        return m.group(0) + f" {{ const uint64_t t_ = clock64(); prof_[{i}] += t_ - tmark_; tmark_ = t_; }}"
    body = re.sub(r"__syncthreads\(\);", mark, body)
    assert n[0] < NPH, n[0]
    # the last two slots: the wave's start and end on the constant 100 MHz clock
    # (wall_clock64, one clock for the whole device): the launch skew and each wave's span
    assert n[0] + 1 < NPH - 2, n[0]
    body = (f"\n    uint64_t prof_[{NPH}] = {{}};\n    prof_[{NPH - 2}] = wall_clock64();\n"
            f"    uint64_t tmark_ = clock64();" + body +
            f"\n    {{ const uint64_t t_ = clock64(); prof_[{n[0]}] += t_ - tmark_; }}\n"
            f"    prof_[{NPH - 1}] = wall_clock64();\n"
            f"    if ((threadIdx.x & 63) == 0)\n        for (int q = 0; q < {NPH}; ++q) "
            f"g_mlp_dbg[((size_t)blockIdx.x * (NT / 64) + threadIdx.x / 64) * {NPH} + q] = prof_[q];")
    s = s[:a] + body + s[b:]
    s = s.replace("struct RowArgs {", f"__device__ uint64_t g_mlp_dbg[{NPH} * 8192];\nstruct RowArgs {{", 1)
    s += ("\nextern \"C\" int salp_debug_mlp_prof(uint64_t* out, int64_t n) {\n"
          f"    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mlp_dbg), sizeof(uint64_t) * {NPH} * n, 0,"
          " hipMemcpyDeviceToHost);\n}\n")
    open(p, "w").write(s)
    out = os.path.join(ROOT, "exp_build", "libsalp_mlpprof.so")
    srcs = [os.path.join(d, "grasp_lab_salp_amd", "csrc", os.path.basename(x)) for x in B.SRCS]
    subprocess.run([B.HIPCC, *B.FLAGS, "-o", out, *srcs], check=True)
    print(out, "phases:", n[0] + 1)


if __name__ == "__main__":
    main()
