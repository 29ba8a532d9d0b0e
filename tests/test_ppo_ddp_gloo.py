"""PPO's gradient averaging across ranks (gloo, world size 2, CPU): ranks that
see different minibatches end every optimizer step with identical weights,
equal to a single-process step on the averaged gradient."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from grasp_lab_salp_amd.ppo import ActorCritic, allreduce_gradients, sampling_generator


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _loss(pol, obs, act):
    v, lp, ent = pol.evaluate(obs, act)
    return (v ** 2).mean() - lp.mean() - 0.01 * ent.mean()


def _data(rank):
    g = torch.Generator().manual_seed(100 + rank)
    return torch.randn(32, 10, generator=g), torch.randn(32, 3, generator=g)


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(rank)                       # different init per rank ...
    pol = ActorCritic(10, 3)
    for p in pol.parameters():                    # ... made identical as PPO.__init__ does
        dist.broadcast(p.data, 0)
    opt = torch.optim.SGD(pol.parameters(), lr=0.1)
    for _ in range(3):
        opt.zero_grad()
        obs, act = _data(rank)
        _loss(pol, obs, act).backward()
        allreduce_gradients(list(pol.parameters()))
        opt.step()
    flat = torch.cat([p.detach().reshape(-1) for p in pol.parameters()])
    parts = [torch.empty_like(flat) for _ in range(world)]
    dist.all_gather(parts, flat)
    # exploration noise: PPO seeds every rank with the same seed (identical
    # policies), the sampling generator must still differ per rank
    torch.manual_seed(0)
    a, _, _ = pol.act(torch.zeros(16, 10), generator=sampling_generator(0, "cpu"))
    acts = [torch.empty_like(a) for _ in range(world)]
    dist.all_gather(acts, a)
    if rank == 0:
        q.put((torch.stack(parts).numpy(), torch.stack(acts).numpy()))
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_stay_identical_and_match_averaged_step():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got, acts = q.get(timeout=300)
    for p in ps:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in ps)
    assert (got[0] == got[1]).all()
    assert not (acts[0] == acts[1]).any(), "ranks drew the same exploration noise"
    # single process: same init (rank 0's), gradient = mean of both ranks' grads
    torch.manual_seed(0)
    pol = ActorCritic(10, 3)
    opt = torch.optim.SGD(pol.parameters(), lr=0.1)
    for _ in range(3):
        opt.zero_grad()
        for r in range(2):
            obs, act = _data(r)
            (_loss(pol, obs, act) / 2).backward()
        opt.step()
    ref = torch.cat([p.detach().reshape(-1) for p in pol.parameters()]).numpy()
    assert abs(got[0] - ref).max() < 1e-5
