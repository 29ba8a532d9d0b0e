"""Where the instructions of a kernel's loops come from (ISA attribution).

    python tools/isa_attr.py [--kernel 'k_rolloutILb0ELb0EE'] [--min-loop 300] [--top 40]

Builds salp_kernels.hip for gfx950 device-only with line tables
(-gline-tables-only; same optimisation flags as the product), disassembles
the kernel, finds its loops (backward branches), and attributes every
instruction of each large loop to the source of its full inline stack
(llvm-symbolizer --inlining): the innermost frame in salp_device.h /
salp_kernels.hip names the part of the tick, the innermost frame overall
(salp_math.h) the math routine.  Prints, per loop, the instruction count
split by class (fp64 VALU, other VALU, SALU, memory) and by source.
"""
import argparse
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
OUT = os.path.join(ROOT, "exp_build", "isa")
SRC = os.path.join(ROOT, "grasp_lab_salp_amd", "csrc", "salp_kernels.hip")
sys.path.insert(0, ROOT)
from grasp_lab_salp_amd.build import FLAGS  # noqa: E402

# parts of salp_device.h's tick by line range (kept in sync by the regexes below)
DEVICE_PARTS = [("newton", r"-+ Newton -+"), ("euler", r"-+ Euler -+"),
                ("integrate v,w", r"-+ integrate \(semi-implicit Euler\) -+"),
                ("euler-rate map", r"to_euler_angle_rate_jit"), ("world frame", r"to_world_frame_jit"),
                ("q,g + clocks/phase", r"h\.q0 = sm_mad\(h\.v0"), ("steady tail", r"if \(STEADY\) \{\s*$"),
                ("geometry", r"float64 geometry \(bitwise"), ("end", r"^/\* -+ Nozzle / Robot control")]


def build(force=False):
    os.makedirs(OUT, exist_ok=True)
    obj = os.path.join(OUT, "k.o")
    dev = os.path.join(OUT, "k.gfx950.o")
    if force or not os.path.exists(dev) or os.path.getmtime(dev) < max(
            os.path.getmtime(os.path.join(ROOT, "grasp_lab_salp_amd", "csrc", f))
            for f in os.listdir(os.path.join(ROOT, "grasp_lab_salp_amd", "csrc"))):
        flags = [f for f in FLAGS if f not in ("-shared", "-fPIC")]
        subprocess.run(["/opt/rocm/bin/hipcc", *flags, "-gline-tables-only", "--offload-device-only", "-c",
                        "-o", obj, SRC], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={obj}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={dev}"], check=True)
    return dev


def disasm(dev, kernel):
    txt = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", dev], check=True,
                         capture_output=True, text=True).stdout
    ins, on = [], False
    for line in txt.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.+)>:$", line)
        if m:
            on = kernel in m.group(2)
            continue
        if on:
            m = re.match(r"^\t(\S+)(.*?)\s*// ([0-9A-F]+):", line)
            if m:
                ins.append((int(m.group(3), 16), m.group(1), m.group(2).strip()))
    return ins


def loops(ins):
    """(start, end) address ranges of backward branches, innermost-first by size."""
    out = []
    for addr, op, args in ins:
        if op.startswith("s_cbranch") or op == "s_branch":
            m = re.match(r"(-?\d+)", args)
            if not m:
                continue
            off = int(m.group(1))
            if off >= 32768:
                off -= 65536
            tgt = addr + 4 + 4 * off
            if tgt <= addr:
                out.append((tgt, addr))
    return sorted(set(out), key=lambda r: r[1] - r[0])


def symbolize(dev, addrs):
    p = subprocess.run([f"{LLVM}/llvm-symbolizer", f"--obj={dev}", "--inlining", "--relative-address"],
                       input="\n".join(hex(a) for a in addrs), capture_output=True, text=True, check=True)
    frames, cur = [], []
    lines = p.stdout.split("\n")
    k = 0
    while k < len(lines):
        if lines[k] == "":
            frames.append(cur)
            cur = []
            k += 1
            continue
        cur.append((lines[k], lines[k + 1] if k + 1 < len(lines) else ""))
        k += 2
    return frames[:len(addrs)]


def device_part_table():
    src = open(os.path.join(ROOT, "grasp_lab_salp_amd", "csrc", "salp_device.h")).read().split("\n")
    marks = []
    for name, rx in DEVICE_PARTS:
        for i, line in enumerate(src, 1):
            if re.search(rx, line):
                marks.append((i, name))
                break
    return sorted(marks)


def classify(op):
    if op.endswith("_f64") or "_f64_" in op or op.startswith("v_div_fixup_f64") or op in ("v_rcp_f64",):
        return "fp64"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    return "mem"


def attribute(frames, marks):
    """(part, routine) of one instruction's inline stack."""
    part, routine = "other", None
    for fn, loc in frames:   # innermost first
        m = re.match(r"(.*):(\d+):\d+", loc)
        if not m:
            continue
        path, line = m.group(1), int(m.group(2))
        base = os.path.basename(path)
        if routine is None and base in ("salp_math.h",):
            routine = re.sub(r"\(.*", "", fn)
        if base == "salp_device.h":
            name = None
            for ln, nm in marks:
                if line >= ln:
                    name = nm
            if name and name != "end":
                f = re.sub(r"\(.*", "", fn).split("::")[-1]
                return (name if f.startswith("tick") else f"{name}/{f}"), routine
            return f"device:{re.sub(r'.*::', '', re.sub(r'[(<].*', '', fn))}", routine
        if base == "salp_kernels.hip":
            part = f"kernel:{line}"
    return part, routine


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", default="k_rolloutILb0ELb0EE")
    ap.add_argument("--min-loop", type=int, default=300, help="smallest loop (instructions) to report")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args()
    dev = build(a.force)
    ins = disasm(dev, a.kernel)
    marks = device_part_table()
    by_addr = {x[0]: x for x in ins}
    reported = []
    for lo, hi in loops(ins):
        body = [x for x in ins if lo <= x[0] <= hi]
        if len(body) < a.min_loop or any(lo <= r0 and r1 <= hi for r0, r1 in reported):
            continue
        reported.append((lo, hi))
        frames = symbolize(dev, [x[0] for x in body])
        cls = collections.Counter(classify(op) for _, op, _ in body)
        parts = collections.Counter()
        parts_f64 = collections.Counter()
        routines = collections.Counter()
        ops = collections.Counter(op for _, op, _ in body)
        for (addr, op, _), fr in zip(body, frames):
            part, routine = attribute(fr, marks)
            parts[part] += 1
            if classify(op) == "fp64":
                parts_f64[part] += 1
            if routine:
                routines[routine] += 1
        print(f"== loop {lo:#x}..{hi:#x}: {len(body)} instructions  " +
              "  ".join(f"{k} {v}" for k, v in sorted(cls.items())))
        print("   by part (all / fp64):")
        for k, v in parts.most_common(a.top):
            print(f"     {v:5d} {parts_f64[k]:5d}  {k}")
        print("   by math routine (innermost salp_math.h frame):")
        for k, v in routines.most_common(12):
            print(f"     {v:5d}  {k}")
        print("   top opcodes:", ", ".join(f"{k} {v}" for k, v in ops.most_common(16)))
    _ = by_addr


if __name__ == "__main__":
    main()
