"""Multi-rank path on the CPU (gloo, world size 2).

Each rank simulates its shard of global env ids with the oracle (the GPU path
shards the same way, tests/test_gpu_parity.py::test_sharding_by_env_id_offset
checks the device), the shards are gathered and must equal an unsharded run;
then the bench's end-of-run reduction (grasp_lab_salp_amd.shard.reduce_run)
must take the MAX of times and the SUM of env-steps over ranks.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from grasp_lab_salp_amd._abi import default_params
from grasp_lab_salp_amd.shard import env_id_offset, reduce_run, reduce_sums

N_PER_RANK = 48
STEPS = 3
SEED = 11


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from oracle.oracle import Oracle
        o = Oracle(default_params(), N_PER_RANK, seed=SEED, env_offset=env_id_offset(rank, N_PER_RANK))
        o.reset()
        rs, ticks = o.step_random(STEPS, threads=1)
        st = torch.from_numpy(o.state.copy())
        parts = [torch.empty_like(st) for _ in range(world)]
        dist.all_gather(parts, st)
        rsum = [torch.empty(N_PER_RANK, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(rsum, torch.from_numpy(rs))
        red = reduce_run(1.0 + rank, 100 * (rank + 1), 10.0 * (rank + 1), 5.0)
        sums = reduce_sums([3 + rank, 1.25e7 + 0.5 * rank, 2 ** 40 + rank])
        if rank == 0:
            q.put(("ok", torch.cat(parts, 1).numpy(), torch.cat(rsum).numpy(), (red, sums)))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put(("err", repr(e), None, None))
        raise


def test_env_id_offset():
    assert env_id_offset(0, 65536) == 0
    assert env_id_offset(3, 65536) == 3 * 65536
    with pytest.raises(ValueError):
        env_id_offset(-1, 4)


def test_reduce_run_without_process_group():
    assert reduce_run(2.0, 10, 3.0, None) == (2.0, 10.0, 3.0, 0.0)
    assert reduce_sums([3, 2.5]) == [3, 2.5]


def test_two_rank_shards_equal_unsharded_run():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    status, state, rsum, red = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
    assert status == "ok", state
    assert all(p.exitcode == 0 for p in procs)
    red, sums = red
    # counters summed exactly as ints, rates as floats (not truncated)
    assert sums == [7, 2.5e7 + 0.5, 2 ** 41 + 1]
    assert isinstance(sums[0], int) and isinstance(sums[1], float)

    from oracle.oracle import Oracle
    ref = Oracle(default_params(), world * N_PER_RANK, seed=SEED, env_offset=0)
    ref.reset()
    rs_ref, _ = ref.step_random(STEPS, threads=1)
    assert np.array_equal(state, ref.state)
    assert np.array_equal(rsum, rs_ref)
    # MAX of wall / kernel time, SUM of env-steps and lock-step rates
    assert red == (2.0, 300.0, 20.0, 10.0)
