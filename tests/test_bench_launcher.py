"""bench.py's multi-rank launcher on the CPU (gloo, no GPU kernels).

`python bench.py --gpus N` starts N ranks itself (torch.distributed.run as a
child process) and every rank owns the global env ids [rank * n, (rank+1) * n);
the driver's 2/4/8-GPU scaling runs go through exactly this path.  --dry-run
swaps RCCL for gloo and skips the kernels, so the rank layout, offsets and the
end-of-run reductions are checked here.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True, timeout=timeout,
                          env=env, cwd=ROOT)


def _json_line(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_gpus_2_launches_two_ranks():
    r = _run(["--gpus", "2", "--dry-run", "--n-envs", "1024"])
    assert r.returncode == 0, r.stderr[-3000:]
    res = _json_line(r.stdout)
    assert res["dry_run"] is True
    assert res["n_gpus"] == 2 and res["world_size"] == 2
    assert res["env_id_offsets"] == [0, 1024]
    # max of per-rank times (1.0 + rank), sum of per-rank env counts
    assert res["max_elapsed"] == 2.0 and res["env_steps_sum"] == 2048


def test_gpus_1_runs_in_process():
    r = _run(["--gpus", "1", "--dry-run", "--n-envs", "64"])
    assert r.returncode == 0, r.stderr[-3000:]
    res = _json_line(r.stdout)
    assert res["n_gpus"] == 1 and res["world_size"] == 1 and res["env_id_offsets"] == [0]


def test_world_size_mismatch_is_an_error():
    r = _run(["--gpus", "2", "--dry-run"], env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "--gpus 2" in r.stderr
