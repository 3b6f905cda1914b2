"""ORACLE (test infrastructure only) -- PyTorch-CPU restatement of the
reference denoising path of pnnl/ERT-Conditional-Diffusion-Model.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module, and only as the checker / the timed CPU baseline.  The product
(ert-conditional-diffusion-model_amd/ertdiff) never imports it.

Pinning: tests/test_oracle.py checks every function here BIT-EXACTLY against
the golden vectors that tests/golden/make_golden.py produced by executing the
reference's own definitions (ERT_Conditional_Diffusion.py:26-218).

The restatement is functional (weights passed as a dict keyed like the
reference's state_dict, ERT_Conditional_Diffusion.py:133-153) and issues the
same ATen ops in the same order as the reference, which is what makes it
bit-identical on CPU.
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import torch
import torch.nn.functional as F

Weights = Dict[str, torch.Tensor]


def timestep_embedding(timesteps: torch.Tensor, dim: int) -> torch.Tensor:
    """ERT_Conditional_Diffusion.py:80-88 (sinusoid, always float32)."""
    half = dim // 2
    scale = math.log(10000.0) / (half - 1)
    freqs = torch.exp(torch.arange(half, dtype=torch.float32) * -scale)
    arg = timesteps.float().unsqueeze(1) * freqs.unsqueeze(0)
    out = torch.cat([torch.sin(arg), torch.cos(arg)], dim=1)
    if dim % 2 == 1:
        out = torch.cat([out, torch.zeros(timesteps.size(0), 1)], dim=1)
    return out


def diffusion_schedule(T: int, beta_start: float = 1e-4, beta_end: float = 0.02):
    """ERT_Conditional_Diffusion.py:90-94."""
    betas = torch.linspace(beta_start, beta_end, T)
    alphas = 1 - betas
    return betas, alphas, torch.cumprod(alphas, dim=0)


def q_sample(x0, t, noise, alpha_bar):
    """ERT_Conditional_Diffusion.py:96-99."""
    a = torch.sqrt(alpha_bar[t]).unsqueeze(1)
    b = torch.sqrt(1 - alpha_bar[t]).unsqueeze(1)
    return a * x0 + b * noise


def encoder(cond: torch.Tensor, W: Weights) -> torch.Tensor:
    """condition_encoder, ERT_Conditional_Diffusion.py:133-142."""
    h = F.relu(F.conv1d(cond, W["condition_encoder.0.weight"], W["condition_encoder.0.bias"],
                        stride=2, padding=1))
    h = F.relu(F.conv1d(h, W["condition_encoder.2.weight"], W["condition_encoder.2.bias"],
                        stride=2, padding=1))
    m = torch.flatten(F.adaptive_avg_pool1d(h, 1), 1)
    return F.relu(F.linear(m, W["condition_encoder.6.weight"], W["condition_encoder.6.bias"]))


def time_mlp(timesteps: torch.Tensor, W: Weights) -> torch.Tensor:
    """time_embed applied to the sinusoid, ERT_Conditional_Diffusion.py:144-147, :159-160."""
    e = timestep_embedding(timesteps, W["time_embed.0.weight"].shape[1])
    return F.relu(F.linear(e, W["time_embed.0.weight"], W["time_embed.0.bias"]))


def forward(x, t, cond, W: Weights) -> torch.Tensor:
    """ConditionalDiffusionModel.forward, ERT_Conditional_Diffusion.py:155-164."""
    h = torch.cat([x, time_mlp(t, W), encoder(cond, W)], dim=1)
    h = F.relu(F.linear(h, W["mlp.0.weight"], W["mlp.0.bias"]))
    return F.linear(h, W["mlp.2.weight"], W["mlp.2.bias"])


def step_tables(betas, alphas, alpha_bar, temperature: float = 1.0):
    """Per-step scalars exactly as sample_model forms them
    (ERT_Conditional_Diffusion.py:111-118): c1 = 1/sqrt(alpha_t) and
    sigma = sqrt(beta_t)*temperature are Python doubles, c2 is a float32 tensor."""
    T = betas.shape[0]
    c1, c2, sg = [], [], []
    for t_ in range(T):
        a_t = alphas[t_]
        ab_t = alpha_bar[t_]
        c2.append(float((1 - a_t) / (math.sqrt(1 - ab_t) + 1e-8)))
        c1.append(1.0 / math.sqrt(a_t))
        sg.append(math.sqrt(betas[t_]) * temperature)
    return c1, c2, sg


@torch.no_grad()
def sample(cond, W: Weights, T: int, noise: torch.Tensor, num_steps: Optional[int] = None,
           temperature: float = 1.0, encoder_every_step: bool = True, max_steps: Optional[int] = None):
    """sample_model (ERT_Conditional_Diffusion.py:102-119) with injected noise.

    noise[0] is x_T and noise[k] is the z drawn for t = n-k (reference draw
    order).  ``encoder_every_step=False`` hoists the t-invariant condition
    encoder (bit-identical on CPU; used only for the hoisted CPU baseline).
    ``max_steps`` stops early (bounded CPU-baseline samples).
    """
    betas, alphas, alpha_bar = diffusion_schedule(T)
    n = T if num_steps is None else num_steps
    B = cond.shape[0]
    x = noise[0].clone()
    cemb = None if encoder_every_step else encoder(cond, W)
    done = 0
    for t_ in reversed(range(n)):
        tt = torch.full((B,), t_, dtype=torch.long)
        if cemb is None:
            pred = forward(x, tt, cond, W)
        else:
            h = torch.cat([x, time_mlp(tt, W), cemb], dim=1)
            h = F.relu(F.linear(h, W["mlp.0.weight"], W["mlp.0.bias"]))
            pred = F.linear(h, W["mlp.2.weight"], W["mlp.2.bias"])
        a_t = alphas[t_]
        ab_t = alpha_bar[t_]
        coef = (1 - a_t) / (math.sqrt(1 - ab_t) + 1e-8)
        x = (1.0 / math.sqrt(a_t)) * (x - coef * pred)
        if t_ > 0:
            x = x + math.sqrt(betas[t_]) * temperature * noise[n - t_]
        done += 1
        if max_steps is not None and done >= max_steps:
            break
    return x


def train_steps(W0: Weights, x0, cond, T: int, ts, noises, lr: float = 1e-4):
    """The reference train step (ERT_Conditional_Diffusion.py:309-319) with
    injected t / noise, repeated len(ts) times with torch.optim.Adam."""
    names = list(W0.keys())
    params = {k: W0[k].clone().requires_grad_(True) for k in names}
    opt = torch.optim.Adam([params[k] for k in names], lr=lr)
    _, _, alpha_bar = diffusion_schedule(T)
    losses, grads0 = [], None
    for i, (t, noise) in enumerate(zip(ts, noises)):
        x_noisy = q_sample(x0, t, noise, alpha_bar)
        pred = forward(x_noisy, t, cond, params)
        loss = F.mse_loss(pred, noise)
        opt.zero_grad()
        loss.backward()
        if i == 0:
            grads0 = {k: params[k].grad.detach().clone() for k in names}
        opt.step()
        losses.append(loss.item())
    return losses, grads0, {k: v.detach() for k, v in params.items()}
