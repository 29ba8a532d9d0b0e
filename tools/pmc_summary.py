"""Summarise the rocprofv3 PMC passes of tools/gpu_pmc.sh for one kernel.

    python tools/pmc_summary.py TAG [--kernel k_rollout] [--n-envs N --tick-budget T --chunk C]

Reads gpurun_out/pmc_<TAG>_<pass>/run_counter_collection.csv and writes
profiles/<TAG>_pmc_summary.json: per-dispatch means of every counter, the HBM
bytes per dispatch (FETCH_SIZE and WRITE_SIZE are KiB; FETCH_SIZE doubled, the
gfx950 correction of MI355X_MICROARCH.md §HBM) and fp64 VALU counts.  bench.py
reports `roofline.traffic` from the summary whose config matches its own and
whose `kernel_sha16` (the counted kernel's machine-code fingerprint,
grasp_lab_salp_amd/_codeobj.py) equals the one of the library it ran: run this
on the tree whose libsalp.so the passes profiled.
"""
import argparse
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from grasp_lab_salp_amd import _codeobj  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--kernel", default="k_rollout")
    ap.add_argument("--symbol", default=_codeobj.ROLLOUT_KERNEL,
                    help="mangled-name fragment of the counted instance (fingerprint)")
    ap.add_argument("--n-envs", type=int, default=65536)
    ap.add_argument("--tick-budget", type=int, default=8192)
    ap.add_argument("--chunk", type=int, default=64)
    ap.add_argument("--config-json", help="the run's config as JSON instead of n_envs / tick_budget / chunk "
                                         "(e.g. the PPO collection: {\"n_envs\": 32768, \"n_steps\": 256})")
    ap.add_argument("--suffix", default="pmc_summary", help="output profiles/<tag>_<suffix>.json")
    ap.add_argument("--command", help="the profiled command, for the record")
    ap.add_argument("--workload-json", help="a JSON file the profiled program wrote about its workload "
                                           "(tools/collect_pmc_probe.py: env-steps per dispatch, ticks per env-step)")
    a = ap.parse_args()
    per = {}
    for path in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", f"pmc_{a.tag}_*", "run_counter_collection.csv"))):
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(path)):
            if a.kernel in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, v in agg.items():
            # the first dispatch is the warm-up launch: keep the timed ones
            vv = v[1:] if len(v) > 1 else v
            per[k] = {"mean": sum(vv) / len(vv), "dispatches": len(vv)}
    if not per:
        raise SystemExit(f"no counters for {a.kernel} under gpurun_out/pmc_{a.tag}_*")
    g = lambda k: per[k]["mean"] if k in per else None  # noqa: E731
    config = (json.loads(a.config_json) if a.config_json else
              {"n_envs": a.n_envs, "tick_budget": a.tick_budget, "chunk": a.chunk})
    out = {"tag": a.tag, "kernel": a.kernel, "config": config,
           "command": a.command or ("tools/gpu_pmc.sh: rocprofv3 --pmc <group> --kernel-trace -- python3 bench.py "
                                    "--steps 2 --warmup 1 --no-cpu-baseline --no-lockstep --no-parity-check --no-ppo, "
                                    "one pass per group"),
           "kernel_symbol": a.symbol,
           "kernel_sha16": _codeobj.kernel_sha(os.path.join(ROOT, "grasp_lab_salp_amd", "libsalp.so"), a.symbol),
           "per_dispatch": per, "derived": {}}
    if a.workload_json:
        out["workload"] = json.load(open(a.workload_json))
    d = out["derived"]
    if g("FETCH_SIZE") is not None:
        d["fetch_bytes"] = g("FETCH_SIZE") * 1024 * 2
    if g("WRITE_SIZE") is not None:
        d["write_bytes"] = g("WRITE_SIZE") * 1024
    if "fetch_bytes" in d and "write_bytes" in d:
        d["hbm_bytes"] = d["fetch_bytes"] + d["write_bytes"]
    f64 = [g(k) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                          "SQ_INSTS_VALU_TRANS_F64")]
    if None not in f64:
        d["fp64_valu_insts"] = sum(f64)
        d["fp64_flops"] = 64 * (f64[0] + f64[1] + 2 * f64[2] + f64[3])
        if not a.config_json:
            # per budget tick (n_envs x tick_budget): round 4's normalisation; bench.py
            # reports flops per executed tick from the measured ticks per env-step
            d["fp64_flops_per_env_tick"] = d["fp64_flops"] / (a.n_envs * a.tick_budget)
    wl = out.get("workload", {})
    if "fp64_flops" in d and wl.get("env_steps_per_dispatch") and wl.get("ticks_per_env_step"):
        d["fp64_flops_per_executed_tick"] = d["fp64_flops"] / (wl["env_steps_per_dispatch"] * wl["ticks_per_env_step"])
    if g("SQ_WAVES"):
        d["valu_insts_per_wave"] = g("SQ_INSTS_VALU") / g("SQ_WAVES")
        d["wait_any_frac"] = g("SQ_WAIT_ANY") / g("SQ_WAVE_CYCLES")
        d["active_valu_frac"] = g("SQ_ACTIVE_INST_VALU") / g("SQ_WAVE_CYCLES")
    dst = os.path.join(ROOT, "profiles", f"{a.tag}_{a.suffix}.json")
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(d, indent=1))


if __name__ == "__main__":
    main()
