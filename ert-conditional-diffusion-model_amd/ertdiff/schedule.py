"""Diffusion schedule and per-step scalar tables.

These are host-side setup values (a few hundred floats, computed once per
sampler call) formed with exactly the reference's expressions so the device
receives bit-identical inputs:

  get_diffusion_schedule   ERT_Conditional_Diffusion.py:90-94 (float32 linspace /
                           cumprod, evaluated with CPU semantics -- the
                           reference's documented devices are CPU/MPS, :282)
  step_tables              the scalars sample_model forms per step (:111-118):
                           c2 = (1-a_t)/(sqrt(1-ab_t)+1e-8) is a float32 tensor,
                           c1 = 1/sqrt(a_t) and sigma = sqrt(b_t)*temperature are
                           Python doubles that torch rounds to float32 when it
                           multiplies them into a float32 tensor
  timestep_frequencies     exp(arange(half) * -ln(1e4)/(half-1)) in float32 (:81-83)
"""
from __future__ import annotations

import math
from functools import lru_cache
from typing import Tuple

import torch


def get_diffusion_schedule(T: int, beta_start: float = 1e-4, beta_end: float = 0.02,
                           device="cpu") -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Linear beta schedule (ERT_Conditional_Diffusion.py:90-94)."""
    betas = torch.linspace(beta_start, beta_end, T)
    alphas = 1 - betas
    alpha_bar = torch.cumprod(alphas, dim=0)
    return betas.to(device), alphas.to(device), alpha_bar.to(device)


def step_tables(betas: torch.Tensor, alphas: torch.Tensor, alpha_bar: torch.Tensor,
                num_steps: int, temperature: float = 1.0) -> torch.Tensor:
    """(3, num_steps) float32 CPU tensor: rows c1, c2, sigma, indexed by t."""
    b = betas.detach().to("cpu", torch.float32)
    a = alphas.detach().to("cpu", torch.float32)
    ab = alpha_bar.detach().to("cpu", torch.float32)
    if num_steps > a.shape[0]:
        raise RuntimeError(f"num_steps={num_steps} exceeds the schedule length {a.shape[0]}")
    out = torch.empty(3, num_steps, dtype=torch.float32)
    for t in range(num_steps):
        a_t, ab_t = a[t], ab[t]
        out[1, t] = (1 - a_t) / (math.sqrt(1 - ab_t) + 1e-8)
        out[0, t] = 1.0 / math.sqrt(a_t)
        out[2, t] = math.sqrt(b[t]) * temperature
    return out


@lru_cache(maxsize=16)
def _freq_cpu(dim: int) -> torch.Tensor:
    half = dim // 2
    scale = math.log(10000.0) / (half - 1)
    return torch.exp(torch.arange(half, dtype=torch.float32) * -scale)


_freq_dev = {}


def timestep_frequencies(dim: int, device: torch.device) -> torch.Tensor:
    key = (dim, str(device))
    f = _freq_dev.get(key)
    if f is None:
        f = _freq_cpu(dim).to(device)
        _freq_dev[key] = f
    return f
