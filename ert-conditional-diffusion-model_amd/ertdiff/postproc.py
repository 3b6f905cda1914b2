"""Ensemble post-processing on the device.

After every realisation the reference copies the sampler output to the host
and runs inverse_transform -> param_scaler.inverse_transform ->
check_param_bounds in numpy (ERT_Conditional_Diffusion.py:398-410 for one
test batch, :1052-1069 for the whole test set), then stacks the realisations
into the (n_samples, N_test, 29) `Uncertainty_params` layout.  Here one kernel
(`ertd_postprocess`, csrc/postproc.hip) does the three steps on the samples
while they are still in HBM; the host only receives the finished array and a
validity mask.

    postprocess(u, scaler, limits)          -> params (rows, P) f32, valid (rows,) bool
    sample_realisations(model, cond, n, ...) -> params (n, B, P), valid (n, B), u (n, B, P)
        (batched=True: the n x B members as ONE sampler launch, sample_conditions)
    compact(params, valid)                  -> check_param_bounds' output per realisation
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import numpy as np
import torch

from . import _lib
from .sampler import sample_conditions, sample_model


def _scaler_vectors(scaler, P: int, dev) -> Tuple[torch.Tensor, torch.Tensor]:
    """(min_, scale_) of a fitted sklearn MinMaxScaler (or a (min_, scale_) pair)."""
    if isinstance(scaler, (tuple, list)):
        mn, sc = scaler
    else:
        mn, sc = scaler.min_, scaler.scale_
    mn = torch.as_tensor(np.asarray(mn, np.float64).reshape(-1), device=dev)
    sc = torch.as_tensor(np.asarray(sc, np.float64).reshape(-1), device=dev)
    if mn.numel() != P or sc.numel() != P:
        raise RuntimeError(f"ertdiff: scaler has {mn.numel()} features, samples have {P}")
    return mn.contiguous(), sc.contiguous()


def _limits(limits, P: int, dev) -> torch.Tensor:
    lim = torch.as_tensor(np.asarray(limits, np.float64), device=dev).contiguous()
    if tuple(lim.shape) != (P, 2):
        raise RuntimeError(f"ertdiff: limits must be ({P}, 2), got {tuple(lim.shape)}")
    return lim


def postprocess(u: torch.Tensor, scaler, limits, a: float = 0.0, b: float = 1.0,
                out: Optional[torch.Tensor] = None,
                valid: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """inverse_transform + MinMaxScaler.inverse_transform + check_param_bounds
    on device.  u: (..., P) float32 samples (unconstrained space).  Returns the
    physical-unit parameters (same shape, float32) and a bool mask over the
    leading dims (True = the row check_param_bounds keeps)."""
    dev = _lib.require_device(u)
    u = _lib.f32c(u, "u")
    P = u.shape[-1]
    rows = u.numel() // P
    mn, sc = _scaler_vectors(scaler, P, dev)
    lim = _limits(limits, P, dev)
    if out is None:
        out = torch.empty_like(u)
    if valid is None:
        valid = torch.empty(u.shape[:-1], dtype=torch.uint8, device=dev)
    if out.shape != u.shape or not out.is_contiguous() or out.dtype != torch.float32:
        raise RuntimeError("ertdiff: out must be a contiguous float32 tensor shaped like u")
    if valid.numel() != rows or not valid.is_contiguous() or valid.dtype not in (torch.uint8, torch.bool):
        raise RuntimeError("ertdiff: valid must be a contiguous uint8/bool tensor with one entry per row")
    with torch.cuda.device(dev):
        _lib.check(_lib.lib().ertd_postprocess(u.data_ptr(), rows, P, float(a), float(b),
                                                mn.data_ptr(), sc.data_ptr(), lim.data_ptr(),
                                                out.data_ptr(), valid.data_ptr(),
                                                _lib.stream_of(dev)), "postprocess")
    return out, valid.view(torch.bool) if valid.dtype == torch.uint8 else valid


@torch.no_grad()
def sample_realisations(model, condition, n_samples: int, T, betas, alphas, alpha_bar,
                        param_dim: int, device, scaler, limits, a: float = 0.0, b: float = 1.0,
                        *, batched: bool = False, **sample_kw):
    """The reference's uncertainty loop (:398-410 / :1052-1064) with the
    post-processing on device.

    batched=False: n_samples calls of sample_model, each followed by
    ertd_postprocess into slice r of an (n_samples, B, P) buffer (the
    reference's loop shape).  batched=True (noise="philox", one condition per
    member): ONE sampler launch over all n_samples x B members
    (sample_conditions) and one ertd_postprocess over the whole array.

    Returns (params, valid, unconstrained): physical-unit parameters
    (n_samples, B, P), the bounds mask (n_samples, B) and the raw sampler
    outputs (the reference's params_realizations_norm).  With noise="philox"
    realisation r's members are Philox member ids r*B .. r*B+B-1 under the one
    seed -- the ids of the batched launch, so both forms return the same bits.
    All three stay on the device."""
    dev = _lib.require_device(condition)
    B = sample_kw.get("n_members") or condition.shape[0]
    seed = int(sample_kw.pop("seed", 0))
    if sample_kw.get("noise") == "philox" and sample_kw.get("member_offset"):
        raise RuntimeError("ertdiff: sample_realisations assigns the member ids itself (realisation r, "
                           "member b -> id r * B + b under one seed); to offset the ids of a slice "
                           "of conditions use sample_conditions(..., cond_offset=...)")
    if batched:
        if sample_kw.get("noise") != "philox" or sample_kw.get("shared_condition"):
            raise RuntimeError("ertdiff: batched realisations need noise='philox' and (B, 14, L) conditions")
        kw = {k: v for k, v in sample_kw.items() if k in ("num_steps", "temperature", "mode", "precision")}
        unc = sample_conditions(model, condition, n_samples, T, betas, alphas, alpha_bar, param_dim,
                                device, seed=seed, **kw)
        params, valid = postprocess(unc, scaler, limits, a, b)
        return params, valid, unc
    unc = torch.empty(n_samples, B, param_dim, dtype=torch.float32, device=dev)
    params = torch.empty_like(unc)
    valid = torch.empty(n_samples, B, dtype=torch.uint8, device=dev)
    for r in range(n_samples):
        kw = dict(sample_kw)
        if kw.get("noise") == "philox":
            kw["seed"] = seed
            kw["member_offset"] = r * B
        unc[r] = sample_model(model, condition, T, betas, alphas, alpha_bar, param_dim, device,
                              **kw)
        postprocess(unc[r], scaler, limits, a, b, out=params[r], valid=valid[r])
    return params, valid.view(torch.bool), unc


def compact(params, valid) -> List[Optional[np.ndarray]]:
    """check_param_bounds' return value per realisation: the kept rows as an
    (n_valid, P) array, or None when no row is kept (:211-218)."""
    p = params.cpu().numpy() if isinstance(params, torch.Tensor) else np.asarray(params)
    m = valid.cpu().numpy() if isinstance(valid, torch.Tensor) else np.asarray(valid)
    p = p.reshape(-1, p.shape[-2], p.shape[-1]) if p.ndim == 3 else p[None]
    m = m.reshape(-1, m.shape[-1]) if m.ndim == 2 else m[None]
    return [np.stack(list(pr[mr])) if mr.any() else None for pr, mr in zip(p, m)]
