"""ConditionalDiffusionModel drop-in (ERT_Conditional_Diffusion.py:121-164).

The module keeps the reference's exact submodule tree, so its state_dict keys,
shapes, parameter order (what Adam's state_dict indexes) and default
initialisation under a given torch seed are identical to the reference's
(checked against the seed-42 golden weights).  Only forward() differs: on a
gfx950 device it runs the fused HIP encoder + head (libertdiff_hip.so); on any
other device it raises -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import torch
import torch.nn as nn

from . import _lib
from .schedule import timestep_frequencies

STATE_KEYS = [
    "condition_encoder.0.weight", "condition_encoder.0.bias",
    "condition_encoder.2.weight", "condition_encoder.2.bias",
    "condition_encoder.6.weight", "condition_encoder.6.bias",
    "time_embed.0.weight", "time_embed.0.bias",
    "mlp.0.weight", "mlp.0.bias", "mlp.2.weight", "mlp.2.bias",
]
_PREC = {"fp32": _lib.PREC_FP32, "bf16": _lib.PREC_BF16}


def get_timestep_embedding(timesteps: torch.Tensor, embedding_dim: int) -> torch.Tensor:
    """Sinusoidal embedding (ERT_Conditional_Diffusion.py:80-88), float32, on device."""
    dev = _lib.require_device(timesteps)
    if embedding_dim < 4:
        raise RuntimeError("ertdiff: embedding_dim must be >= 4")
    t = timesteps.to(torch.int64).contiguous()
    B = t.shape[0]
    out = torch.empty(B, embedding_dim, dtype=torch.float32, device=dev)
    freq = timestep_frequencies(embedding_dim, dev)
    with torch.cuda.device(dev):
        _lib.check(_lib.lib().ertd_timestep_embedding(
            t.data_ptr(), B, embedding_dim, freq.data_ptr(), out.data_ptr(),
            _lib.stream_of(dev)), "timestep_embedding")
    return out


def q_sample(x0: torch.Tensor, t: torch.Tensor, noise: torch.Tensor,
             alpha_bar: torch.Tensor) -> torch.Tensor:
    """Forward noising (ERT_Conditional_Diffusion.py:96-99) on device."""
    dev = _lib.require_device(x0, t, noise, alpha_bar)
    x0 = _lib.f32c(x0, "x0")
    noise = _lib.f32c(noise, "noise")
    ab = _lib.f32c(alpha_bar, "alpha_bar")
    if x0.dim() != 2 or noise.shape != x0.shape or t.shape != (x0.shape[0],):
        raise RuntimeError(f"ertdiff.q_sample: bad shapes x0={tuple(x0.shape)} "
                           f"t={tuple(t.shape)} noise={tuple(noise.shape)}")
    t = t.to(torch.int64).contiguous()
    out = torch.empty_like(x0)
    B, P = x0.shape
    with torch.cuda.device(dev):
        _lib.check(_lib.lib().ertd_q_sample(x0.data_ptr(), t.data_ptr(), noise.data_ptr(),
                                            ab.data_ptr(), B, P, out.data_ptr(),
                                            _lib.stream_of(dev)), "q_sample")
    return out


class ConditionalDiffusionModel(nn.Module):
    """Noise predictor eps(x, t, condition) with a 1-D CNN condition encoder.

    Submodules mirror ERT_Conditional_Diffusion.py:133-153 one for one.
    ``precision``: "fp32" (default, the reference arithmetic) or "bf16"
    (bf16 conv operands with fp32 accumulation; SURVEY.md 7 "bf16").
    """

    def __init__(self, param_dim: int, hidden_dim: int = 128):
        super().__init__()
        self.param_dim = param_dim
        self.condition_encoder = nn.Sequential(
            nn.Conv1d(in_channels=14, out_channels=32, kernel_size=3, stride=2, padding=1),
            nn.ReLU(),
            nn.Conv1d(32, 64, kernel_size=3, stride=2, padding=1),
            nn.ReLU(),
            nn.AdaptiveAvgPool1d(1),
            nn.Flatten(),
            nn.Linear(64, hidden_dim),
            nn.ReLU(),
        )
        self.time_embed = nn.Sequential(nn.Linear(hidden_dim, hidden_dim), nn.ReLU())
        self.mlp = nn.Sequential(
            nn.Linear(param_dim + 2 * hidden_dim, hidden_dim),
            nn.ReLU(),
            nn.Linear(hidden_dim, param_dim),
        )
        self.precision = "fp32"
        self._packed: Optional[torch.Tensor] = None
        self._packed_key = None
        self._ws = {}

    # ---- device plumbing -------------------------------------------------------
    def _check_supported(self):
        hid = self.time_embed[0].in_features
        if hid != _lib.HIDDEN:
            raise RuntimeError(f"ertdiff kernels support hidden_dim={_lib.HIDDEN} only (got {hid})")
        if not 1 <= self.param_dim <= _lib.PMAX:
            raise RuntimeError(f"ertdiff kernels support 1 <= param_dim <= {_lib.PMAX}")

    def _params(self):
        sd = dict(self.named_parameters())
        return [sd[k] for k in STATE_KEYS]

    def weights_struct(self) -> _lib.ErtdWeights:
        ps = self._params()
        for k, p in zip(STATE_KEYS, ps):
            if p.dtype != torch.float32 or not p.is_contiguous():
                raise RuntimeError(f"ertdiff: parameter {k} must be contiguous float32")
        w = _lib.ErtdWeights(*[p.data_ptr() for p in ps], self.param_dim, _lib.HIDDEN)
        return w

    def packed_weights(self, dev: torch.device) -> torch.Tensor:
        """Fragment-order / k-major copies of the weights, re-packed whenever a
        parameter is modified in place (tracked by tensor version counters)."""
        ps = self._params()
        key = tuple((p.data_ptr(), p._version) for p in ps)
        if self._packed is None or self._packed_key != key or self._packed.device != dev:
            n = _lib.lib().ertd_packed_floats()
            if self._packed is None or self._packed.device != dev:
                self._packed = torch.empty(n, dtype=torch.float32, device=dev)
            w = self.weights_struct()
            with torch.cuda.device(dev):
                _lib.check(_lib.lib().ertd_pack_weights(ctypes.byref(w), self._packed.data_ptr(),
                                                        _lib.stream_of(dev)), "pack_weights")
            self._packed_key = key
        return self._packed

    def workspace(self, dev: torch.device, B: int, L: int, T: int, op: int) -> torch.Tensor:
        n = _lib.lib().ertd_workspace_bytes(B, L, self.param_dim, T, op)
        ws = self._ws.get((dev, op))
        if ws is None or ws.numel() < n:
            ws = torch.empty(max(n, 256), dtype=torch.uint8, device=dev)
            self._ws[(dev, op)] = ws
        return ws

    def _check_inputs(self, x, t, condition):
        if x.dim() != 2 or x.shape[1] != self.param_dim:
            raise RuntimeError(f"ertdiff: x must be (B, {self.param_dim}), got {tuple(x.shape)}")
        B = x.shape[0]
        if condition.dim() != 3 or condition.shape[0] != B or condition.shape[1] != _lib.CIN:
            raise RuntimeError(f"ertdiff: condition must be (B, 14, L), got {tuple(condition.shape)}")
        if t.dim() != 1 or t.shape[0] != B:
            raise RuntimeError(f"ertdiff: t must be (B,), got {tuple(t.shape)}")

    # ---- forward --------------------------------------------------------------------
    def forward(self, x: torch.Tensor, t: torch.Tensor, condition: torch.Tensor,
                return_intermediates: bool = False):
        """eps = model(x (B,P), t (B,) int, condition (B,14,L)) -- :155-164."""
        self._check_supported()
        dev = _lib.require_device(x, t, condition, self.mlp[0].weight)
        self._check_inputs(x, t, condition)
        if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in self.parameters())):
            from .train import DiffusionForwardFn
            return DiffusionForwardFn.apply(self, x, t, condition, *self._params())
        return self._forward_nograd(x, t, condition, dev, return_intermediates)

    def _forward_nograd(self, x, t, condition, dev, return_intermediates=False):
        x = _lib.f32c(x, "x")
        cond = _lib.f32c(condition, "condition")
        tt = t.to(torch.int64).contiguous()
        B, L = x.shape[0], cond.shape[2]
        out = torch.empty(B, self.param_dim, dtype=torch.float32, device=dev)
        cemb = temb = None
        if return_intermediates:
            cemb = torch.empty(B, _lib.HIDDEN, dtype=torch.float32, device=dev)
            temb = torch.empty(B, _lib.HIDDEN, dtype=torch.float32, device=dev)
        packed = self.packed_weights(dev)
        ws = self.workspace(dev, B, L, 0, _lib.OP_FORWARD)
        freq = timestep_frequencies(_lib.HIDDEN, dev)
        w = self.weights_struct()
        with torch.cuda.device(dev):
            _lib.check(_lib.lib().ertd_forward(
                ctypes.byref(w), packed.data_ptr(), x.data_ptr(), tt.data_ptr(), cond.data_ptr(),
                B, L, freq.data_ptr(), _PREC[self.precision], out.data_ptr(), _lib.ptr(cemb),
                _lib.ptr(temb), ws.data_ptr(), ws.numel(), _lib.stream_of(dev)), "forward")
        if return_intermediates:
            return out, cemb, temb
        return out

    @torch.no_grad()
    def encode_condition(self, condition: torch.Tensor) -> torch.Tensor:
        """condition_encoder(condition) -> (B,128) (:133-142)."""
        self._check_supported()
        dev = _lib.require_device(condition, self.mlp[0].weight)
        cond = _lib.f32c(condition, "condition")
        if cond.dim() != 3 or cond.shape[1] != _lib.CIN:
            raise RuntimeError(f"ertdiff: condition must be (B, 14, L), got {tuple(cond.shape)}")
        B, L = cond.shape[0], cond.shape[2]
        out = torch.empty(B, _lib.HIDDEN, dtype=torch.float32, device=dev)
        packed = self.packed_weights(dev)
        ws = self.workspace(dev, B, L, 1, _lib.OP_SAMPLE)
        w = self.weights_struct()
        with torch.cuda.device(dev):
            _lib.check(_lib.lib().ertd_encoder_fwd(
                ctypes.byref(w), packed.data_ptr(), cond.data_ptr(), B, L, _PREC[self.precision],
                out.data_ptr(), ws.data_ptr(), ws.numel(), _lib.stream_of(dev)), "encoder_fwd")
        return out
