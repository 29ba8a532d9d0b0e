"""Summarise tools/gpu_gae_prof.sh output (gpurun_out/gae_*) into
profiles/<tag>_gae_profile.json: per shape, rocprof average k_gae duration,
algorithmic bytes (20 B per (step, env) + 8 B per env), and PMC HBM bytes
(FETCH_SIZE KiB x1024 x2 gfx950 correction; WRITE_SIZE KiB x1024)."""
import collections
import csv
import json
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "r1k"
root = "gpurun_out"
shapes = {32768: 2048, 65536: 512, 524288: 256}   # n_envs -> n_steps (tools/gae_bench.py)
t = collections.defaultdict(list)
for r in csv.DictReader(open(f"{root}/gae_prof/run_kernel_trace.csv")):
    if "k_gae" in r["Kernel_Name"]:
        t[int(r["Grid_Size_X"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
pm = collections.defaultdict(lambda: collections.defaultdict(list))
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for r in csv.DictReader(open(f"{root}/gae_pmc_{c}/run_counter_collection.csv")):
        if "k_gae" in r["Kernel_Name"]:
            pm[int(r["Grid_Size"])][c].append(float(r["Counter_Value"]))
out = []
for n, ts in sorted(t.items()):
    T = shapes[n]
    ms = sum(ts[1:]) / (len(ts) - 1)                 # first launch is a warm-up
    alg = T * n * 20 + n * 8
    f = sum(pm[n]["FETCH_SIZE"][1:]) / (len(pm[n]["FETCH_SIZE"]) - 1) * 1024 * 2
    w = sum(pm[n]["WRITE_SIZE"][1:]) / (len(pm[n]["WRITE_SIZE"]) - 1) * 1024
    out.append({"n_steps": T, "n_envs": n, "launches": len(ts), "rocprof_avg_ms": round(ms, 4),
                "algorithmic_bytes": alg, "achieved_GBs": round(alg / ms / 1e6, 1),
                "frac_of_8TBs": round(alg / ms / 1e6 / 8000, 3), "pmc_fetch_bytes": f, "pmc_write_bytes": w,
                "traffic_over_algorithmic": round((f + w) / alg, 3)})
res = {"command": "tools/gpu_gae_prof.sh (rocprofv3 --kernel-trace --stats; --pmc FETCH_SIZE, --pmc WRITE_SIZE)",
       "kernel": "k_gae", "per_shape": out}
json.dump(res, open(f"profiles/{tag}_gae_profile.json", "w"), indent=1)
print(json.dumps(res, indent=1))
