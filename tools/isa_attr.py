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


def natural_loops(ins):
    """Natural loops of the kernel's control-flow graph: for every loop header
    (the target of a back edge: an edge to a block that dominates its source),
    the header plus every basic block that reaches one of its back edges
    without passing through it.  Unlike an
    address range, this includes the blocks the compiler laid out after the
    loop's back edge (cold paths, a branch's else side).  Returns
    [(header_addr, [instruction addresses])]."""
    addrs = [x[0] for x in ins]
    index = {a: k for k, a in enumerate(addrs)}
    def target(addr, op, args):
        m = re.match(r"(-?\d+)", args)
        if not (op.startswith("s_cbranch") or op == "s_branch") or not m:
            return None
        off = int(m.group(1))
        if off >= 32768:
            off -= 65536
        return addr + 4 + 4 * off
    # basic block leaders
    leaders = {addrs[0]}
    for k, (addr, op, args) in enumerate(ins):
        t = target(addr, op, args)
        if t is not None:
            leaders.add(t)
            if k + 1 < len(ins):
                leaders.add(addrs[k + 1])
        elif op in ("s_endpgm", "s_setpc_b64") and k + 1 < len(ins):
            leaders.add(addrs[k + 1])
    starts = sorted(a for a in leaders if a in index)
    blocks = {}
    for j, a in enumerate(starts):
        end = starts[j + 1] if j + 1 < len(starts) else addrs[-1] + 4
        blocks[a] = [x for x in addrs[index[a]:] if x < end]
    succ = {a: [] for a in blocks}
    for a, body in blocks.items():
        last = body[-1]
        _, op, args = ins[index[last]]
        t = target(last, op, args)
        nxt = addrs[index[last] + 1] if index[last] + 1 < len(addrs) else None
        if t is not None and t in blocks:
            succ[a].append(t)
        if op not in ("s_branch", "s_endpgm", "s_setpc_b64") and nxt is not None and nxt in blocks:
            succ[a].append(nxt)
    pred = {a: [] for a in blocks}
    for a, ss in succ.items():
        for b in ss:
            pred[b].append(a)
    # dominators (Cooper, Harvey & Kennedy's iterative algorithm) over the
    # blocks reachable from the entry, in reverse postorder
    entry = starts[0]
    order, seen, stack = [], {entry}, [(entry, iter(succ[entry]))]
    while stack:
        node, it = stack[-1]
        nxt = next(it, None)
        if nxt is None:
            order.append(node)
            stack.pop()
        elif nxt not in seen:
            seen.add(nxt)
            stack.append((nxt, iter(succ[nxt])))
    rpo = order[::-1]
    num = {b: k for k, b in enumerate(rpo)}
    idom = {entry: entry}
    changed = True
    while changed:
        changed = False
        for b in rpo[1:]:
            ps = [p for p in pred[b] if p in idom]
            if not ps:
                continue
            new_idom = ps[0]
            for p in ps[1:]:
                x, y = p, new_idom
                while x != y:
                    while num[x] > num[y]:
                        x = idom[x]
                    while num[y] > num[x]:
                        y = idom[y]
                new_idom = x
            if idom.get(b) != new_idom:
                idom[b] = new_idom
                changed = True

    def dominates(h, b):
        while True:
            if b == h:
                return True
            if b == entry or b not in idom:
                return False
            b = idom[b]

    loops_ = {}
    for a, ss in succ.items():
        for h in ss:
            if a in idom and dominates(h, a):   # back edge a -> h
                body = loops_.setdefault(h, {h})
                stack = [a]
                while stack:
                    x = stack.pop()
                    if x not in body:
                        body.add(x)
                        stack.extend(pred[x])
    return [(h, sorted(i for b in body for i in blocks[b])) for h, body in loops_.items()]


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
    ap.add_argument("--max-loop", type=int, default=2500, help="largest natural loop to report")
    a = ap.parse_args()
    dev = build(a.force)
    ins = disasm(dev, a.kernel)
    marks = device_part_table()
    by_addr = {x[0]: x for x in ins}
    for h, members in sorted(natural_loops(ins), key=lambda x: len(x[1])):
        if not a.min_loop <= len(members) <= a.max_loop:
            continue
        body = [by_addr[m] for m in members]
        lo, hi = members[0], members[-1]
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
        print(f"== natural loop, header {h:#x} (span {lo:#x}..{hi:#x}): {len(body)} instructions  " +
              "  ".join(f"{k} {v}" for k, v in sorted(cls.items())))
        print("   by part (all / fp64):")
        for k, v in parts.most_common(a.top):
            print(f"     {v:5d} {parts_f64[k]:5d}  {k}")
        print("   by math routine (innermost salp_math.h frame):")
        for k, v in routines.most_common(12):
            print(f"     {v:5d}  {k}")
        print("   top opcodes:", ", ".join(f"{k} {v}" for k, v in ops.most_common(16)))


if __name__ == "__main__":
    main()
