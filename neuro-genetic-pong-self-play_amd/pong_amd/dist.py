"""Population sharding over ranks and the one collective of a generation.

The reference farms individuals out to SCOOP workers (ga.py:83
``futures.map``).  Here rank r of N evaluates the contiguous rows
``shard_range(P, r, N)`` of a replicated population, and the fitness vector is
all-gathered once per generation (RCCL over xGMI with the "nccl" backend on
MI355X; gloo in the CPU tests).  Nothing else crosses ranks: the GA state is
replicated and updated identically from the same counter-based RNG keys.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(n: int, rank: int, world: int):
    """Rows [lo, hi) of rank ``rank``: contiguous, sizes differ by at most one."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of world {world}")
    base, rem = divmod(int(n), int(world))
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def gather_fitness(local: torch.Tensor, n_total: int, group=None) -> torch.Tensor:
    """All-gather each rank's fitness shard into the full [n_total] vector, in
    row order (a [rows, c] shard: the full [n_total, c] table, e.g. fitness
    beside each row's longest game)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    lo, hi = shard_range(n_total, rank, world)
    if local.shape[0] != hi - lo:
        raise ValueError(f"rank {rank} holds {local.shape[0]} fitness values, expected {hi - lo}")
    width = -(-n_total // world)  # ceil: all_gather needs equal sizes
    # gloo (the CPU test backend, also used for several ranks on one GPU) moves
    # host tensors; RCCL ("nccl") gathers device memory over xGMI directly
    stage = local.is_cuda and dist.get_backend(group) == "gloo"
    dev = torch.device("cpu") if stage else local.device
    tail = tuple(local.shape[1:])
    buf = torch.zeros((width,) + tail, dtype=local.dtype, device=dev)
    buf[: hi - lo] = local.to(dev)
    out = torch.empty((width * world,) + tail, dtype=local.dtype, device=dev)
    if stage:
        dist.all_gather(list(out.split(width)), buf, group=group)
    else:
        dist.all_gather_into_tensor(out, buf, group=group)
    parts = []
    for r in range(world):
        a, b = shard_range(n_total, r, world)
        parts.append(out[r * width: r * width + (b - a)])
    return torch.cat(parts).to(local.device)


def gather_equal(local: torch.Tensor, group=None) -> torch.Tensor:
    """All-gather equal-sized per-rank tables ([n, ...] each) into [world * n, ...],
    rank-major: the length-balanced shards' (row, fitness, longest game) entries
    (evolve.DeviceGA.balance_shards), whose rows are dealt, not contiguous."""
    world = dist.get_world_size(group)
    stage = local.is_cuda and dist.get_backend(group) == "gloo"
    dev = torch.device("cpu") if stage else local.device
    buf = local.to(dev).contiguous()
    out = torch.empty((local.shape[0] * world,) + tuple(local.shape[1:]), dtype=local.dtype, device=dev)
    if stage:
        dist.all_gather(list(out.split(local.shape[0])), buf, group=group)
    else:
        dist.all_gather_into_tensor(out, buf, group=group)
    return out.to(local.device)


def deal_positions(n_buf: int, rank: int, world: int, device=None) -> torch.Tensor:
    """Positions of rank ``rank`` in a snake deal of a length-ordered list over
    ``world`` ranks: round k gives position k * world + (rank if k is even else
    world - 1 - rank), so each rank's k-th game is as long as the others' (the
    longest first) and the per-rank totals stay within one game's length."""
    k = torch.arange(n_buf, device=device, dtype=torch.int64)
    off = torch.where(k % 2 == 0, torch.full_like(k, rank), torch.full_like(k, world - 1 - rank))
    return k * world + off


def gather_rows(local: torch.Tensor, n_total: int, group=None) -> torch.Tensor:
    """All-gather each rank's shard rows ([rows, ...]) into the full table in
    row order (gather_fitness for any row width: genomes, hashes)."""
    return gather_fitness(local, n_total, group)


def evaluate_sharded(evaluate_rows, n_total: int, group=None):
    """Evaluate this rank's rows with ``evaluate_rows(lo, hi) -> fitness tensor``
    and return the full fitness vector on every rank."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    lo, hi = shard_range(n_total, rank, world)
    local = evaluate_rows(lo, hi)
    if world == 1:
        return local
    return gather_fitness(local, n_total, group)
