"""Training path on the GPU (ERT_Conditional_Diffusion.py:294-320).

  DiffusionForwardFn   autograd.Function: model(x, t, cond) under autograd runs
                       the HIP training forward (activations kept in a per-call
                       workspace) and, on backward, the HIP backward: gradients
                       of all 12 parameters (and of x).  So the reference's own
                       loop -- MSELoss, loss.backward(), optimizer.step() --
                       works unchanged on an ertdiff model.
  train_step           the reference's train-step body (:309-320) fused into one
                       library call: q_sample -> forward -> MSELoss -> backward
                       -> Adam, updating the torch.optim.Adam state in place so
                       optimizer.state_dict() stays valid (:348).
  validation_loss      the no-grad validation pass body (:327-336).
"""
from __future__ import annotations

import ctypes

import torch
import torch.nn.functional as F

from . import _lib
from .schedule import timestep_frequencies


def _train_ws(dev, B, L, P):
    n = _lib.lib().ertd_workspace_bytes(B, L, P, 0, _lib.OP_TRAIN)
    return torch.empty(max(n, 256), dtype=torch.uint8, device=dev)


class DiffusionForwardFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, model, x, t, cond, *params):
        dev = x.device
        x = _lib.f32c(x, "x")
        cond = _lib.f32c(cond, "condition")
        tt = t.to(torch.int64).contiguous()
        B, L, P = x.shape[0], cond.shape[2], model.param_dim
        ws = _train_ws(dev, B, L, P)
        packed = torch.empty(_lib.lib().ertd_packed_floats(), dtype=torch.float32, device=dev)
        eps = torch.empty(B, P, dtype=torch.float32, device=dev)
        freq = timestep_frequencies(_lib.HIDDEN, dev)
        w = model.weights_struct()
        with torch.cuda.device(dev):
            _lib.check(_lib.lib().ertd_train_forward(
                ctypes.byref(w), packed.data_ptr(), x.data_ptr(), None, None, None, tt.data_ptr(),
                cond.data_ptr(), B, L, freq.data_ptr(), eps.data_ptr(), ws.data_ptr(), ws.numel(),
                _lib.stream_of(dev)), "train_forward")
        ctx.model = model
        ctx.ws, ctx.packed, ctx.cond, ctx.B, ctx.L = ws, packed, cond, B, L
        ctx.save_for_backward(*params)
        return eps

    @staticmethod
    def backward(ctx, grad_eps):
        params = ctx.saved_tensors
        dev = grad_eps.device
        dout = _lib.f32c(grad_eps, "grad")
        grads = [torch.empty_like(p) for p in params]
        dx = (torch.empty(ctx.B, ctx.model.param_dim, dtype=torch.float32, device=dev)
              if ctx.needs_input_grad[1] else None)
        w = ctx.model.weights_struct()
        with torch.cuda.device(dev):
            _lib.check(_lib.lib().ertd_train_backward(
                ctypes.byref(w), ctx.packed.data_ptr(), dout.data_ptr(), None, ctx.cond.data_ptr(),
                ctx.B, ctx.L, _lib.ptr_array(grads), None, _lib.ptr(dx), ctx.ws.data_ptr(),
                ctx.ws.numel(), _lib.stream_of(dev)), "train_backward")
        return (None, dx, None, None, *grads)


def _adam_hparams(optimizer, params):
    if not isinstance(optimizer, torch.optim.Adam):
        raise RuntimeError("ertdiff.train_step drives torch.optim.Adam (the reference optimizer, :294)")
    if len(optimizer.param_groups) != 1:
        raise RuntimeError("ertdiff.train_step expects one parameter group")
    g = optimizer.param_groups[0]
    gp = g["params"]
    if len(gp) != len(params) or any(a is not b for a, b in zip(gp, params)):
        raise RuntimeError("optimizer parameters must be model.parameters() in module order")
    if g.get("weight_decay", 0) != 0 or g.get("amsgrad", False) or g.get("maximize", False):
        raise RuntimeError("ertdiff Adam supports weight_decay=0, amsgrad=False, maximize=False")
    lr = g["lr"]
    if isinstance(lr, torch.Tensor):
        lr = float(lr)
    return float(lr), float(g["betas"][0]), float(g["betas"][1]), float(g["eps"])


def train_step(model, optimizer, x0, cond, T, alpha_bar, *, t=None, noise=None,
               return_tensor: bool = False):
    """One reference train step (:309-320); returns loss.item() (or the device
    scalar if ``return_tensor``).  t / noise default to the reference's draws
    (torch.randint then torch.randn_like, :312-313)."""
    from .unet import ConditionalUNet
    if isinstance(model, ConditionalUNet):   # the same call surface over the U-Net denoiser
        from .unet_train import unet_train_step
        return unet_train_step(model, optimizer, x0, cond, T, alpha_bar, t=t, noise=noise,
                               return_tensor=return_tensor)
    model._check_supported()
    params = model._params()
    dev = _lib.require_device(x0, cond, alpha_bar, params[0])
    B = x0.size(0)
    if t is None:
        t = torch.randint(0, T, (B,), device=dev).long()
    if noise is None:
        noise = torch.randn_like(x0)
    x0 = _lib.f32c(x0, "x0")
    noise = _lib.f32c(noise, "noise")
    cond = _lib.f32c(cond, "condition")
    ab = _lib.f32c(alpha_bar, "alpha_bar")
    tt = t.to(device=dev, dtype=torch.int64).contiguous()
    model._check_inputs(x0, tt, cond)
    lr, b1, b2, eps = _adam_hparams(optimizer, params)
    exp_avg, exp_avg_sq = [], []
    for p in params:
        st = optimizer.state[p]
        if len(st) == 0:
            st["step"] = torch.tensor(0.0, dtype=torch.float32)
            st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
            st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
        st["step"] += 1
        exp_avg.append(st["exp_avg"])
        exp_avg_sq.append(st["exp_avg_sq"])
        if p.grad is None:
            p.grad = torch.empty_like(p)
    step = int(optimizer.state[params[0]]["step"].item())
    grads = [p.grad for p in params]
    L = cond.shape[2]
    ws = model.workspace(dev, B, L, 0, _lib.OP_TRAIN)
    packed = model.packed_weights(dev)
    loss = torch.empty((), dtype=torch.float32, device=dev)
    freq = timestep_frequencies(_lib.HIDDEN, dev)
    w = model.weights_struct()
    with torch.cuda.device(dev):
        _lib.check(_lib.lib().ertd_train_step(
            ctypes.byref(w), packed.data_ptr(), x0.data_ptr(), tt.data_ptr(), noise.data_ptr(),
            cond.data_ptr(), ab.data_ptr(), B, L, freq.data_ptr(), _lib.ptr_array(grads),
            _lib.ptr_array(exp_avg), _lib.ptr_array(exp_avg_sq), step, lr, b1, b2, eps,
            loss.data_ptr(), ws.data_ptr(), ws.numel(), _lib.stream_of(dev)), "train_step")
    model._packed_key = None  # parameters changed in place behind autograd's back: re-pack
    return loss if return_tensor else loss.item()


@torch.no_grad()
def validation_loss(model, x0, cond, T, alpha_bar, *, t=None, noise=None) -> float:
    """Validation pass body (:327-336): forward on q_sample'd inputs, MSE."""
    from .model import q_sample
    B = x0.size(0)
    dev = x0.device
    if t is None:
        t = torch.randint(0, T, (B,), device=dev).long()
    if noise is None:
        noise = torch.randn_like(x0)
    x_noisy = q_sample(x0, t, noise, alpha_bar)
    pred = model(x_noisy, t, cond)
    return F.mse_loss(pred, noise).item()
