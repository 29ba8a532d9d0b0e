"""Compact per-kernel summary of rocprofv3 PMC passes (run on the GPU box,
right after the passes, so the raw per-dispatch CSVs can be deleted before
gpurun copies gpurun_out/ back; they exceed its 64 MiB limit).

    python tools/pmc_kernels_summary.py PREFIX k_mlp_fwd_bwd k_mlp_reduce ... > out.json

Reads gpurun_out/PREFIX_*/run_counter_collection.csv (and run_kernel_trace.csv
for durations): per kernel and counter the mean / min / max over dispatches and
the dispatch count; per kernel the mean duration (ns) of each pass.
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def short(name):
    m = re.search(r"(k_\w+?)(?:I|E|\(|<|$)", name)
    return m.group(1) if m else name[:60]


def main():
    prefix, kernels = sys.argv[1], sys.argv[2:]
    out = {"prefix": prefix, "kernels": {}}
    for d in sorted(glob.glob(os.path.join("gpurun_out", prefix + "_*"))):
        if not os.path.isdir(d):
            continue
        group = d[len(os.path.join("gpurun_out", prefix + "_")):]
        cc = os.path.join(d, "run_counter_collection.csv")
        if os.path.exists(cc):
            agg = collections.defaultdict(lambda: collections.defaultdict(list))
            for r in csv.DictReader(open(cc)):
                k = short(r["Kernel_Name"])
                if not kernels or k in kernels:
                    agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            for k, cs in agg.items():
                e = out["kernels"].setdefault(k, {"counters": {}, "duration_ns": {}})
                for c, v in cs.items():
                    e["counters"][c] = {"mean": sum(v) / len(v), "min": min(v), "max": max(v), "dispatches": len(v)}
        kt = os.path.join(d, "run_kernel_trace.csv")
        if os.path.exists(kt):
            dur = collections.defaultdict(list)
            for r in csv.DictReader(open(kt)):
                k = short(r["Kernel_Name"])
                if not kernels or k in kernels:
                    dur[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            for k, v in dur.items():
                e = out["kernels"].setdefault(k, {"counters": {}, "duration_ns": {}})
                e["duration_ns"][group] = {"mean": sum(v) / len(v), "dispatches": len(v)}
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
