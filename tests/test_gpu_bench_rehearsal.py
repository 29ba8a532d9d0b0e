"""bench.py's N-rank code path on the GPU, every GPUTEST round.

The driver's 2/4/8-GPU scaling runs start `bench.py --gpus N`, which launches
N ranks under torch.distributed.run.  A one-GPU box cannot give each rank its
own device, so SALP_BENCH_REHEARSAL=1 lets two ranks share cuda:0 and carries
the reductions (and the PPO leg's gradient all-reduce) over gloo: every other
line of the N-rank run is the real one - env-id sharding, the kernels, the
max-over-ranks timing, rank 0's sampled oracle replay and its CPU baseline.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_two_rank_bench_rehearsal_on_one_gpu():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["SALP_BENCH_REHEARSAL"] = "1"
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--cpu-baseline-seconds", "1.5", "--ppo-envs", "4096"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=540, env=env, cwd=ROOT)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["world_size"] == 2
    assert res["value"] > 0 and res["steps"] == 2
    assert res["parity_sampled"]["ok"], res["parity_sampled"]
    cb = res["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] >= 1 and cb["kind"] == "port"
    assert res["ppo"]["value"] > 0
