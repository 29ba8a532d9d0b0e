"""Summarise tools/gpu_ablate.sh: per library, the headline rate, k_rollout's
time per launch and its PMC instruction counts per wave and per executed
tick, and the difference to the product build.

    python tools/ablate_summary.py TAG [--out profiles/TAG_ablation.json]

Env-ticks per launch = env-steps per launch x ticks per env-step (the
ablations leave the cycle lengths alone: they are set by the actions and the
nozzle angles, src/robot.py:589-592, 742); --ticks-per-step overrides the
oracle's 710.4.
"""
import argparse
import collections
import csv
import glob
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "k_rollout<false, false>"


def counters(path):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if KERNEL in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: (sum(v[1:]) / len(v[1:]) if len(v) > 1 else v[0]) for k, v in agg.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--out")
    ap.add_argument("--ticks-per-step", type=float, default=710.4)
    a = ap.parse_args()
    d = os.path.join(ROOT, "gpurun_out", f"ablate_{a.tag}")
    rows = {}
    for bj in sorted(glob.glob(os.path.join(d, "*_bench.json"))):
        name = os.path.basename(bj)[:-len("_bench.json")]
        b = json.loads(open(bj).read().strip().splitlines()[-1])
        steps_launch = b["value"] * b["ms_per_step"] / 1e3
        c = counters(os.path.join(d, f"{name}_pmc", "run_counter_collection.csv"))
        waves = c.get("SQ_WAVES", 1024.0)
        ticks = steps_launch * a.ticks_per_step
        wave_ticks = ticks / 64.0
        f64 = sum(c.get(k, 0.0) for k in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64",
                                          "SQ_INSTS_VALU_TRANS_F64"))
        flops = 64 * (f64 + c.get("SQ_INSTS_VALU_FMA_F64", 0.0))
        rows[name] = {
            "value_M": b["value"] / 1e6, "kernel_ms": b["kernel_ms_per_launch"], "env_steps_per_launch": steps_launch,
            "valu_per_wave": c.get("SQ_INSTS_VALU", 0.0) / waves, "salu_per_wave": c.get("SQ_INSTS_SALU", 0.0) / waves,
            "valu_per_wave_tick": c.get("SQ_INSTS_VALU", 0.0) / wave_ticks,
            "salu_per_wave_tick": c.get("SQ_INSTS_SALU", 0.0) / wave_ticks,
            "fp64_per_wave_tick": f64 / wave_ticks, "fp64_flops_per_env_tick": flops / ticks,
            "wave_cycles_per_wave": c.get("SQ_WAVE_CYCLES", 0.0) / waves, "counters": c}
    base = rows.get("product")
    for name, r in rows.items():
        if base and name != "product":
            r["delta_valu_per_wave_tick"] = r["valu_per_wave_tick"] - base["valu_per_wave_tick"]
            r["delta_salu_per_wave_tick"] = r["salu_per_wave_tick"] - base["salu_per_wave_tick"]
            r["speedup"] = base["kernel_ms"] / r["kernel_ms"] * r["env_steps_per_launch"] / base["env_steps_per_launch"]
        print(f"{name:12s} {r['value_M']:6.2f} M  {r['kernel_ms']:6.2f} ms  VALU/wave-tick {r['valu_per_wave_tick']:7.1f}"
              f"  SALU/wave-tick {r['salu_per_wave_tick']:6.1f}  fp64/wave-tick {r['fp64_per_wave_tick']:6.1f}"
              f"  flops/env-tick {r['fp64_flops_per_env_tick']:6.1f}"
              + (f"  dVALU {r['delta_valu_per_wave_tick']:+6.1f}  speedup {r['speedup']:.3f}" if "speedup" in r else ""))
    if a.out:
        json.dump({"tag": a.tag, "ticks_per_env_step": a.ticks_per_step, "rows": rows}, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
