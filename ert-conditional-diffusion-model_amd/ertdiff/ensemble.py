"""Sharded ensemble sampling across the GPUs of a node.

The reference draws realisations in an outer Python loop
(ERT_Conditional_Diffusion.py:398-410 and :1052-1069): members are independent,
so the ensemble shards with no exchange on the data path.  One process per GPU
(torchrun / torch.distributed, backend "nccl" = RCCL):

  1. rank 0 holds the ERT condition; ONE broadcast (RCCL over xGMI) gives it
     to every rank -- the only collective before sampling;
  2. rank r samples the contiguous member range member_range(n, world, r),
     reading the shared condition in place (stride 0) with Philox noise keyed
     by the GLOBAL member id, so the ensemble is bitwise identical for any
     world size;
  3. each rank returns its own shard (hi-lo, P) on its device; the caller
     copies it to the host (per-device D2H) and concatenates by member_range
     -- no gather collective.  ``gather=True`` is an opt-in
     convenience that adds one all_gather AFTER sampling, for callers that
     want the whole ensemble on every rank.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import torch
import torch.distributed as dist


def member_range(n_members: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous balanced split: the first n % world ranks get one extra member."""
    if n_members < 0 or world < 1 or not 0 <= rank < world:
        raise ValueError("bad ensemble partition arguments")
    base, rem = divmod(n_members, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def _dist_info(group=None) -> Tuple[int, int]:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def broadcast_condition(condition: Optional[torch.Tensor], shape, device, src: int = 0,
                        group=None) -> torch.Tensor:
    """Give every rank rank-`src`'s condition (14, L) / (1, 14, L)."""
    rank, world = _dist_info(group)
    if rank == src:
        if condition is None:
            raise ValueError("the source rank must provide the condition")
        buf = condition.to(device=device, dtype=torch.float32).contiguous()
    else:
        buf = torch.empty(tuple(shape), dtype=torch.float32, device=device)
    if world > 1:
        dist.broadcast(buf, src=src, group=group)
    return buf


def gather_members(local: torch.Tensor, n_members: int, group=None) -> torch.Tensor:
    """All ranks' shards, concatenated in global member order."""
    rank, world = _dist_info(group)
    if world == 1:
        return local
    P = local.shape[1]
    width = max(hi - lo for lo, hi in (member_range(n_members, world, r) for r in range(world)))
    pad = torch.zeros(width, P, dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    out = torch.empty(world * width, P, dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, pad, group=group)
    parts = []
    for r in range(world):
        lo, hi = member_range(n_members, world, r)
        parts.append(out[r * width: r * width + (hi - lo)])
    return torch.cat(parts)


@torch.no_grad()
def sample_ensemble(model, condition: Optional[torch.Tensor], n_members: int, T: int, betas,
                    alphas, alpha_bar, *, seed: int, num_steps=None, temperature: float = 1.0,
                    mode: str = "hoisted", L: Optional[int] = None, device=None, group=None,
                    gather: bool,
                    _sampler: Optional[Callable] = None) -> torch.Tensor:
    """n_members realisations x_0 (unconstrained space) for ONE condition.

    condition: (14, L) or (1, 14, L) on the source rank (others may pass None
    and give L).  ``gather`` has no default (round 2 changed the old
    gather-by-default behaviour; a caller must now say which result it
    wants): False returns this rank's (hi-lo, P) shard (global members
    member_range(n_members, world, rank)), True adds one all_gather after
    sampling and returns the whole (n_members, P) ensemble on every rank.
    With one rank both are the whole ensemble.  ``_sampler`` replaces the device sampler in the
    CPU (gloo) tests of this host logic; the product always uses
    ertdiff.sample_model.
    """
    rank, world = _dist_info(group)
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    if condition is not None:
        L = condition.shape[-1]
    if L is None:
        raise ValueError("non-source ranks must pass L")
    cond = broadcast_condition(condition.reshape(1, 14, L) if condition is not None else None,
                               (1, 14, L), device, group=group)
    lo, hi = member_range(n_members, world, rank)
    if _sampler is None:
        from .sampler import sample_model
        _sampler = sample_model
    P = model.param_dim
    if hi > lo:
        local = _sampler(model, cond, T, betas, alphas, alpha_bar, P, device, num_steps=num_steps,
                         temperature=temperature, mode=mode, noise="philox", seed=seed,
                         member_offset=lo, shared_condition=True, n_members=hi - lo)
    else:
        local = torch.empty(0, P, dtype=torch.float32, device=device)
    return gather_members(local, n_members, group) if gather else local


@torch.no_grad()
def sample_conditions_sharded(model, conditions, n_samples: int, T: int, betas, alphas, alpha_bar,
                              *, seed: int, num_steps=None, temperature: float = 1.0,
                              mode: str = "hoisted", device=None, group=None,
                              _sampler: Optional[Callable] = None) -> Tuple[torch.Tensor, int, int]:
    """The test-set evaluation (ERT_Conditional_Diffusion.py:1042-1069) sharded
    over the ranks of one node: rank r takes the condition slice
    [c0, c1) = member_range(N, world, r) of the HOST array `conditions`
    (N, 14, L) -- a host-side scatter, no collective -- copies
    only that slice to its device and runs every realisation of it as one
    sampler launch (ertdiff.sample_conditions) with condition offset c0 and
    id period N, so every member keeps its global Philox id r * N + c.

    Returns (local, c0, c1): this rank's (n_samples, c1 - c0, P) block of the
    (n_samples, N, P) `Uncertainty_params` array; the caller concatenates the
    blocks along dim 1 (per-device D2H).  ``_sampler`` replaces the device
    sampler in the CPU (gloo) tests of this host logic."""
    rank, world = _dist_info(group)
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    N = conditions.shape[0]
    c0, c1 = member_range(N, world, rank)
    if _sampler is None:
        from .sampler import sample_conditions
        _sampler = sample_conditions
    P = model.param_dim
    if c1 == c0:
        return torch.empty(n_samples, 0, P, dtype=torch.float32, device=device), c0, c1
    local_cond = torch.as_tensor(conditions[c0:c1], dtype=torch.float32).to(device).contiguous()
    local = _sampler(model, local_cond, n_samples, T, betas, alphas, alpha_bar, P, device,
                     num_steps=num_steps, temperature=temperature, mode=mode, seed=seed,
                     cond_offset=c0, n_conditions_total=N)
    return local, c0, c1
