"""The RCCL ("nccl") backend on the GPU box (VERDICT r5 missing #3: the nccl
branch had only run under gloo).  One GPU allows one RCCL rank, so this is a
world-size-1 group in a child process: the collectives bench.py's N-rank run
and the multi-rank PPO learner issue (a broadcast of the policy, the flat
gradient's all-reduce as ppo._allreduce_flat_grads does it, the max-over-ranks
of the timed region, a barrier) run through RCCL on device tensors and leave
them as they were.  The N-rank arithmetic itself is covered by the gloo tests
(test_ppo_ddp_gloo.py, test_bench_launcher.py) and the two-rank GPU test
(test_gpu_ppo_multirank.py)."""
import os
import socket
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent("""
    import sys, torch, torch.distributed as dist
    sys.path.insert(0, sys.argv[2])
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:" + sys.argv[1], rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    from grasp_lab_salp_amd.ppo import PPO
    from grasp_lab_salp_amd.vec_env import SalpVecEnv
    env = SalpVecEnv(1024, seed=0, infos=False)
    m = PPO("MlpPolicy", env, n_steps=8, batch_size=4096, n_epochs=1, seed=0, use_graphs=False)
    assert not m._multi and m.fused_update
    m.learn(8 * 1024)                                   # one iteration: the fused minibatch steps
    g = m._f_grads.clone()
    assert bool(torch.isfinite(g).all()) and float(g.abs().sum()) > 0
    dist.all_reduce(m._f_grads)                          # ppo._allreduce_flat_grads with one rank
    m._f_grads /= dist.get_world_size()
    assert torch.equal(m._f_grads, g)
    w = [p.detach().clone() for p in m.policy.parameters()]
    for p in m.policy.parameters():
        dist.broadcast(p.data, 0)
    assert all(torch.equal(a, p) for a, p in zip(w, m.policy.parameters()))
    t = torch.tensor([1.25], device="cuda", dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)            # bench.py's max over ranks
    dist.barrier()
    torch.cuda.synchronize()
    assert float(t) == 1.25
    print("RCCL_OK", dist.get_backend())
    dist.destroy_process_group()
""")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_collectives_on_device_tensors():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    out = subprocess.run([sys.executable, "-c", CHILD, str(_free_port()), REPO], env=env, capture_output=True,
                         text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "RCCL_OK nccl" in out.stdout, out.stdout[-2000:]
