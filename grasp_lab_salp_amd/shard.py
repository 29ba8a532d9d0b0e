"""Env sharding across ranks (one process per GPU).

Envs are independent (the reference has no cross-env state),
so rank r simulates the contiguous global env ids [r * n, (r + 1) * n).  The
device RNG is keyed by global env id, so an env's trajectory does not depend on
the world size.  Nothing is exchanged on the data path; the only collectives
are these end-of-run reductions of counters and timings (RCCL on GPUs, gloo in
the CPU tests).
"""
import torch
import torch.distributed as dist

__all__ = ["env_id_offset", "reduce_run", "reduce_sums"]


def env_id_offset(rank, n_envs_per_rank):
    """Global id of this rank's env 0."""
    if rank < 0 or n_envs_per_rank <= 0:
        raise ValueError("rank must be >= 0 and n_envs_per_rank > 0")
    return int(rank) * int(n_envs_per_rank)


def reduce_run(elapsed_s, env_steps, kernel_ms, lockstep_rate, device=None):
    """Combine per-rank bench results: wall time and kernel time are the MAX
    over ranks (the job ends with its slowest rank), env-steps and lock-step
    rates are SUMS.  Returns python floats; without an initialised process
    group it returns the inputs."""
    vals = [float(elapsed_s), float(env_steps), float(kernel_ms), float(lockstep_rate or 0.0)]
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return tuple(vals)
    t = torch.tensor(vals, dtype=torch.float64, device=device)
    mx, sm = t.clone(), t.clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    dist.all_reduce(sm, op=dist.ReduceOp.SUM)
    return mx[0].item(), sm[1].item(), mx[2].item(), sm[3].item()


def reduce_sums(values, device=None):
    """SUM of per-rank counters (e.g. diverged envs) or rates over ranks; the
    inputs themselves without an initialised process group.  Python ints stay
    ints (summed exactly as int64), anything else is summed as float64."""
    ints = [isinstance(v, int) and not isinstance(v, bool) for v in values]
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [int(v) if k else float(v) for v, k in zip(values, ints)]
    ti = torch.tensor([int(v) if k else 0 for v, k in zip(values, ints)], dtype=torch.int64, device=device)
    tf = torch.tensor([0.0 if k else float(v) for v, k in zip(values, ints)], dtype=torch.float64, device=device)
    dist.all_reduce(ti, op=dist.ReduceOp.SUM)
    dist.all_reduce(tf, op=dist.ReduceOp.SUM)
    return [int(a) if k else float(b) for a, b, k in zip(ti.tolist(), tf.tolist(), ints)]
