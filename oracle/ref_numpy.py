"""ORACLE (test infrastructure only) -- float64 numpy restatement of the
reference denoising path, written independently of PyTorch so it can serve as
the "truth" against which both the reference's fp32 CPU arithmetic and the HIP
kernels are measured.  Includes the hand-derived backward pass and Adam, which
pin the GPU train step.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module.  tests/test_oracle.py pins it against the golden vectors generated
from the reference (tolerances there, ~1e-6 relative: fp64 vs the reference's
fp32 arithmetic).

Reference anchors (ERT_Conditional_Diffusion.py):
  get_timestep_embedding :80-88, get_diffusion_schedule :90-94,
  q_sample :96-99, sample_model :102-119, ConditionalDiffusionModel :122-164,
  train step :308-320 (MSELoss :295, Adam lr=1e-4 :294),
  transform_to_unconstrained :26-40, inverse_transform :42-53,
  check_param_bounds :183-218.
"""
from __future__ import annotations

import math
from typing import Dict

import numpy as np

Weights = Dict[str, np.ndarray]
KEYS = ["condition_encoder.0.weight", "condition_encoder.0.bias",
        "condition_encoder.2.weight", "condition_encoder.2.bias",
        "condition_encoder.6.weight", "condition_encoder.6.bias",
        "time_embed.0.weight", "time_embed.0.bias",
        "mlp.0.weight", "mlp.0.bias", "mlp.2.weight", "mlp.2.bias"]


def conv_out_len(L: int) -> int:
    """Conv1d(k=3, s=2, p=1) output length."""
    return (L + 2 - 3) // 2 + 1


def timestep_embedding(t, dim: int) -> np.ndarray:
    """:80-88 in float64."""
    t = np.asarray(t, dtype=np.float64)
    half = dim // 2
    freqs = np.exp(np.arange(half, dtype=np.float64) * -(math.log(10000.0) / (half - 1)))
    arg = t[:, None] * freqs[None, :]
    out = np.concatenate([np.sin(arg), np.cos(arg)], axis=1)
    if dim % 2 == 1:
        out = np.concatenate([out, np.zeros((t.shape[0], 1))], axis=1)
    return out


def diffusion_schedule(T: int, beta_start=1e-4, beta_end=0.02):
    """:90-94 (float64 here; the reference is float32)."""
    betas = np.linspace(beta_start, beta_end, T, dtype=np.float64)
    alphas = 1.0 - betas
    return betas, alphas, np.cumprod(alphas)


def q_sample(x0, t, noise, alpha_bar):
    """:96-99."""
    ab = np.asarray(alpha_bar, np.float64)[np.asarray(t)]
    return np.sqrt(ab)[:, None] * x0 + np.sqrt(1.0 - ab)[:, None] * noise


def _im2col(x: np.ndarray) -> np.ndarray:
    """x (B,C,L) -> cols (B, C*3, Lout) for k=3, stride 2, zero pad 1."""
    B, C, L = x.shape
    Lo = conv_out_len(L)
    xp = np.zeros((B, C, 2 * Lo + 1), dtype=x.dtype)
    xp[:, :, 1:1 + L] = x[:, :, : 2 * Lo]
    cols = np.stack([xp[:, :, k: k + 2 * Lo: 2] for k in range(3)], axis=2)  # B,C,3,Lo
    return cols.reshape(B, C * 3, Lo)


def _col2im(dcols: np.ndarray, C: int, L: int) -> np.ndarray:
    B, _, Lo = dcols.shape
    d = dcols.reshape(B, C, 3, Lo)
    dxp = np.zeros((B, C, 2 * Lo + 1), dtype=dcols.dtype)
    for k in range(3):
        dxp[:, :, k: k + 2 * Lo: 2] += d[:, :, k, :]
    dx = np.zeros((B, C, L), dtype=dcols.dtype)
    n = min(L, 2 * Lo)
    dx[:, :, :n] = dxp[:, :, 1:1 + n]
    return dx


def conv1d_s2(x, w, b):
    cols = _im2col(x)
    return np.einsum("ok,bki->boi", w.reshape(w.shape[0], -1), cols, optimize=True) + b[None, :, None], cols


def _w(W, k):
    return np.asarray(W[k], dtype=np.float64)


def forward_full(x, t, cond, W: Weights) -> dict:
    """Forward with every intermediate kept (for backward and for per-op checks)."""
    x = np.asarray(x, np.float64)
    cond = np.asarray(cond, np.float64)
    z1, cols1 = conv1d_s2(cond, _w(W, "condition_encoder.0.weight"), _w(W, "condition_encoder.0.bias"))
    a1 = np.maximum(z1, 0.0)
    z2, cols2 = conv1d_s2(a1, _w(W, "condition_encoder.2.weight"), _w(W, "condition_encoder.2.bias"))
    a2 = np.maximum(z2, 0.0)
    m = a2.mean(axis=2)
    z3 = m @ _w(W, "condition_encoder.6.weight").T + _w(W, "condition_encoder.6.bias")
    c = np.maximum(z3, 0.0)
    H = W["time_embed.0.weight"].shape[1]
    e = timestep_embedding(t, H)
    z4 = e @ _w(W, "time_embed.0.weight").T + _w(W, "time_embed.0.bias")
    te = np.maximum(z4, 0.0)
    hcat = np.concatenate([x, te, c], axis=1)
    z5 = hcat @ _w(W, "mlp.0.weight").T + _w(W, "mlp.0.bias")
    h = np.maximum(z5, 0.0)
    out = h @ _w(W, "mlp.2.weight").T + _w(W, "mlp.2.bias")
    return dict(cond=cond, z1=z1, a1=a1, cols1=cols1, z2=z2, a2=a2, cols2=cols2, m=m, z3=z3,
                cond_emb=c, e=e, z4=z4, t_emb=te, hcat=hcat, z5=z5, h=h, out=out)


def encoder(cond, W: Weights) -> np.ndarray:
    cond = np.asarray(cond, np.float64)
    z1, _ = conv1d_s2(cond, _w(W, "condition_encoder.0.weight"), _w(W, "condition_encoder.0.bias"))
    z2, _ = conv1d_s2(np.maximum(z1, 0), _w(W, "condition_encoder.2.weight"), _w(W, "condition_encoder.2.bias"))
    m = np.maximum(z2, 0).mean(axis=2)
    return np.maximum(m @ _w(W, "condition_encoder.6.weight").T + _w(W, "condition_encoder.6.bias"), 0)


def forward(x, t, cond, W: Weights) -> np.ndarray:
    return forward_full(x, t, cond, W)["out"]


def backward(f: dict, noise, W: Weights) -> tuple:
    """MSE(mean) loss and gradients of every state_dict entry (hand-derived)."""
    noise = np.asarray(noise, np.float64)
    out = f["out"]
    B, P = out.shape
    diff = out - noise
    loss = float(np.mean(diff * diff))
    g = {}
    dout = 2.0 * diff / (B * P)
    g["mlp.2.weight"] = dout.T @ f["h"]
    g["mlp.2.bias"] = dout.sum(0)
    dz5 = (dout @ _w(W, "mlp.2.weight")) * (f["z5"] > 0)
    g["mlp.0.weight"] = dz5.T @ f["hcat"]
    g["mlp.0.bias"] = dz5.sum(0)
    dh = dz5 @ _w(W, "mlp.0.weight")
    H = f["t_emb"].shape[1]
    dte = dh[:, P:P + H]
    dc = dh[:, P + H:]
    dz4 = dte * (f["z4"] > 0)
    g["time_embed.0.weight"] = dz4.T @ f["e"]
    g["time_embed.0.bias"] = dz4.sum(0)
    dz3 = dc * (f["z3"] > 0)
    g["condition_encoder.6.weight"] = dz3.T @ f["m"]
    g["condition_encoder.6.bias"] = dz3.sum(0)
    dm = dz3 @ _w(W, "condition_encoder.6.weight")
    L2 = f["a2"].shape[2]
    dz2 = np.repeat(dm[:, :, None] / L2, L2, axis=2) * (f["z2"] > 0)
    w2 = _w(W, "condition_encoder.2.weight")
    g["condition_encoder.2.weight"] = np.einsum("boi,bki->ok", dz2, f["cols2"], optimize=True).reshape(w2.shape)
    g["condition_encoder.2.bias"] = dz2.sum((0, 2))
    dcols2 = np.einsum("ok,boi->bki", w2.reshape(w2.shape[0], -1), dz2, optimize=True)
    da1 = _col2im(dcols2, f["a1"].shape[1], f["a1"].shape[2])
    dz1 = da1 * (f["z1"] > 0)
    w1 = _w(W, "condition_encoder.0.weight")
    g["condition_encoder.0.weight"] = np.einsum("boi,bki->ok", dz1, f["cols1"], optimize=True).reshape(w1.shape)
    g["condition_encoder.0.bias"] = dz1.sum((0, 2))
    return loss, g


def adam_update(params: Weights, grads: Weights, state: dict, lr=1e-4, b1=0.9, b2=0.999, eps=1e-8):
    """torch.optim.Adam default semantics (no weight decay, no amsgrad)."""
    state["step"] = state.get("step", 0) + 1
    s = state["step"]
    out = {}
    for k, p in params.items():
        m = state.setdefault("m", {}).get(k, np.zeros_like(p, dtype=np.float64))
        v = state.setdefault("v", {}).get(k, np.zeros_like(p, dtype=np.float64))
        gk = grads[k]
        m = b1 * m + (1 - b1) * gk
        v = b2 * v + (1 - b2) * gk * gk
        bc1 = 1 - b1 ** s
        bc2 = 1 - b2 ** s
        denom = np.sqrt(v) / math.sqrt(bc2) + eps
        out[k] = np.asarray(p, np.float64) - (lr / bc1) * m / denom
        state["m"][k], state["v"][k] = m, v
    return out


def train_steps(W0: Weights, x0, cond, T, ts, noises, lr=1e-4):
    params = {k: np.asarray(W0[k], np.float64) for k in KEYS}
    _, _, ab = diffusion_schedule(T)
    ab32 = np.cumprod(1.0 - np.linspace(1e-4, 0.02, T, dtype=np.float32), dtype=np.float32)
    state, losses, grads0 = {}, [], None
    for i, (t, noise) in enumerate(zip(ts, noises)):
        xn = q_sample(x0, t, noise, ab32.astype(np.float64))
        f = forward_full(xn, t, cond, params)
        loss, g = backward(f, noise, params)
        if i == 0:
            grads0 = g
        params = adam_update(params, g, state, lr=lr)
        losses.append(loss)
    return losses, grads0, params


def sample(cond, W: Weights, T: int, noise, num_steps=None, temperature=1.0, alphas32=True,
           max_steps=None):
    """sample_model :102-119 with injected noise in float64.  ``alphas32`` uses
    the reference's float32 schedule values (so only arithmetic differs);
    ``max_steps`` stops after that many reverse steps (first steps of a chain)."""
    if alphas32:
        betas = np.linspace(1e-4, 0.02, T, dtype=np.float32).astype(np.float64)
        betas32 = np.linspace(1e-4, 0.02, T, dtype=np.float32)
        alphas = (np.float32(1) - betas32).astype(np.float64)
        alpha_bar = np.cumprod((np.float32(1) - betas32), dtype=np.float32).astype(np.float64)
    else:
        betas, alphas, alpha_bar = diffusion_schedule(T)
    n = T if num_steps is None else num_steps
    noise = np.asarray(noise, np.float64)
    cond = np.asarray(cond, np.float64)
    B = cond.shape[0]
    x = noise[0].copy()
    for i, t_ in enumerate(reversed(range(n))):
        if max_steps is not None and i >= max_steps:
            break
        pred = forward_full(x, np.full(B, t_), cond, W)["out"]
        coef = (1 - alphas[t_]) / (math.sqrt(1 - alpha_bar[t_]) + 1e-8)
        x = (1.0 / math.sqrt(alphas[t_])) * (x - coef * pred)
        if t_ > 0:
            x = x + math.sqrt(betas[t_]) * temperature * noise[n - t_]
    return x


def transform_to_unconstrained(x, a, b):
    """:26-40."""
    eps = 1e-6
    xn = np.clip((x - a) / (b - a), eps, 1 - eps)
    return np.log(xn / (1 - xn))


def inverse_transform(u, a, b):
    """:42-53."""
    return a + (b - a) * (1.0 / (1.0 + np.exp(-u)))


def bounds_mask(params, limits) -> np.ndarray:
    """check_param_bounds :183-218 as a per-row validity mask: a row is rejected
    when some value is < min or > max (so a NaN passes, as in the reference)."""
    lo = limits[:, 0]
    hi = limits[:, 1]
    return ~np.any((params < lo) | (params > hi), axis=1)


def postprocess_chain(u, min_, scale_, limits, a=0.0, b=1.0):
    """The post-sampling chain of :400-406 / :1054-1060 on a float32 (rows, P)
    array: sigmoid inverse_transform in float32 (torch op on a float32 tensor:
    (b-a) and a enter as float32 scalars), then sklearn MinMaxScaler's
    in-place ``x -= min_; x /= scale_`` (float64 operands, result stored back
    into the float32 array), then check_param_bounds as a mask."""
    u = np.asarray(u, np.float32)
    # torch.sigmoid on float32 = 1/(1+exp(-u)) with float32 rounding per op
    e = np.exp(-u.astype(np.float64)).astype(np.float32)
    s = (np.float32(1.0) / (np.float32(1.0) + e)).astype(np.float32)
    x = (np.float32(a) + np.float32(b - a) * s).astype(np.float32)
    x = (x.astype(np.float64) - min_).astype(np.float32)
    x = (x.astype(np.float64) / scale_).astype(np.float32)
    return x, bounds_mask(x, limits)


def rel_l2(a, b) -> float:
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))
