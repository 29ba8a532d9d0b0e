"""GAE kernel alone against the HBM roofline at a few shapes (HIP events)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.bench_ppo import gae_roofline  # noqa: E402

if __name__ == "__main__":
    for T, n in ((2048, 32768), (512, 65536), (256, 524288)):
        r = gae_roofline(T, n)
        print(json.dumps({"lib": os.environ.get("SALP_LIB", "product"), "T": T, "n": n, "ms": round(r["ms"], 4),
                          "GBs": round(r["roofline"]["achieved"], 1), "frac": round(r["roofline"]["frac"], 3)}))
