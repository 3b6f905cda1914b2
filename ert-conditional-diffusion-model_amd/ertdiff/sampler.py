"""Reverse-diffusion sampler drop-in (ERT_Conditional_Diffusion.py:102-119).

``sample_model`` keeps the reference signature.  The T-step loop runs inside
libertdiff_hip.so:

  mode="hoisted"  (default) condition encoder once per call, then one
                  persistent kernel runs all steps with x in registers.
  mode="faithful" encoder re-evaluated every step exactly like the reference:
                  one persistent launch per chain (encoder strips streamed
                  ahead of per-member step chains), or the per-step schedule
                  when the grid cannot be resident;
  mode="faithful_steps"  faithful, forced per-step schedule (an encoder and a
                  head launch per step).

All modes are bit-identical: the encoder is deterministic (fixed-order
reductions) and every schedule runs the same fma chains in the same order.

Noise sources (keyword ``noise``):
  "torch"   (default) x_T and every z_t drawn with torch.randn on ``device``
            in the reference's order (:107, :116), so the RNG stream consumed
            is the one the reference would consume under the same seed;
  "philox"  counter-based Philox in-kernel, keyed by (seed, member id, t):
            no host work, and results are independent of how members are
            split across calls or GPUs;
  tensor    (num_steps, B, P) injected draws in reference order (parity tests).
"""
from __future__ import annotations

import ctypes
from typing import Optional, Union

import torch

from . import _lib
from .model import _PREC, ConditionalDiffusionModel, STATE_KEYS
from .schedule import step_tables, timestep_frequencies

_MODES = {"hoisted": _lib.MODE_HOISTED, "faithful": _lib.MODE_FAITHFUL,
          "faithful_steps": _lib.MODE_FAITHFUL_STEPS}


def sample_status(ws: torch.Tensor, B: int, L: int, num_steps: int) -> int:
    """Status word of the last faithful run on ``ws`` (synchronizes): 0 = ok,
    else the code of the persistent-chain wait that timed out."""
    st = ctypes.c_int(0)
    with torch.cuda.device(ws.device):
        rc = _lib.lib().ertd_sample_status(ws.data_ptr(), B, L, num_steps, ctypes.byref(st),
                                           _lib.stream_of(ws.device))
    if rc not in (_lib.ERTD_OK, _lib.ERTD_ETIMEOUT):
        _lib.check(rc, "sample_status")
    return st.value


def as_ertdiff_model(model, device) -> ConditionalDiffusionModel:
    """Accept any module with the reference's state_dict (e.g. the reference's
    own ConditionalDiffusionModel) by loading its weights into an ertdiff one."""
    if isinstance(model, ConditionalDiffusionModel):
        return model
    sd = model.state_dict()
    missing = [k for k in STATE_KEYS if k not in sd]
    if missing:
        raise RuntimeError(f"ertdiff: model lacks reference parameters {missing}")
    P = sd["mlp.2.weight"].shape[0]
    H = sd["time_embed.0.weight"].shape[0]
    m = ConditionalDiffusionModel(P, H)
    m.load_state_dict(sd)
    return m.to(device).eval()


def draw_reference_noise(B: int, P: int, num_steps: int, device) -> torch.Tensor:
    """(num_steps, B, P): x_T then z for t = num_steps-1 .. 1, one torch.randn
    call per draw exactly as sample_model issues them."""
    x = torch.randn(B, P, device=device)
    buf = torch.empty(num_steps, B, P, dtype=torch.float32, device=x.device)
    buf[0] = x
    for k in range(1, num_steps):
        buf[k] = torch.randn_like(x)
    return buf


class _Prepared:
    """Device-side inputs of one sampler call (kept alive for plan replays)."""

    def __init__(self, model, condition, T, betas, alphas, alpha_bar, num_steps, temperature,
                 precision, shared_condition):
        self.model = model
        dev = _lib.require_device(condition, model.mlp[0].weight)
        self.dev = dev
        model._check_supported()
        cond = _lib.f32c(condition, "condition")
        if cond.dim() == 2:
            cond = cond.unsqueeze(0)
        if cond.dim() != 3 or cond.shape[1] != _lib.CIN:
            raise RuntimeError(f"ertdiff: condition must be (B, 14, L), got {tuple(condition.shape)}")
        self.cond = cond
        self.L = cond.shape[2]
        self.stride = 0 if shared_condition else _lib.CIN * self.L
        self.num_steps = T if num_steps is None else int(num_steps)
        if not 1 <= self.num_steps <= T:
            raise RuntimeError(f"ertdiff: num_steps={self.num_steps} must be in [1, T={T}]")
        self.tables = step_tables(betas, alphas, alpha_bar, self.num_steps, temperature).to(dev)
        self.freq = timestep_frequencies(_lib.HIDDEN, dev)
        self.packed = model.packed_weights(dev)
        self.prec = _PREC[precision]
        self.w = model.weights_struct()

    def workspace(self, B):
        return self.model.workspace(self.dev, B, self.L, self.num_steps, _lib.OP_SAMPLE)

    def args(self, B, x, noise, seed, member_offset, mode, t_first, n_run, ws):
        tb = self.tables
        return (ctypes.byref(self.w), self.packed.data_ptr(), self.cond.data_ptr(), self.stride,
                B, self.L, self.num_steps, t_first, n_run, tb[0].data_ptr(), tb[1].data_ptr(),
                tb[2].data_ptr(), self.freq.data_ptr(), _lib.ptr(noise), int(seed) & (2**64 - 1),
                int(member_offset) & 0xFFFFFFFF, _MODES[mode], self.prec, x.data_ptr(),
                ws.data_ptr(), ws.numel())


def philox_normal(B: int, P: int, t: int, tag: int, seed: int, member_offset: int,
                  device) -> torch.Tensor:
    """Draws of the in-kernel Philox stream (tag 1 = x_T, tag 0 = z_t)."""
    dev = torch.device(device)
    out = torch.empty(B, P, dtype=torch.float32, device=dev)
    _lib.require_device(out)
    with torch.cuda.device(dev):
        _lib.check(_lib.lib().ertd_philox_normal(int(seed) & (2**64 - 1), member_offset, B, P, t,
                                                 tag, out.data_ptr(), _lib.stream_of(dev)),
                   "philox_normal")
    return out


@torch.no_grad()
def sample_model(model, condition, T, betas, alphas, alpha_bar, param_dim, device,
                 num_steps=None, temperature=1.0, *, mode: str = "hoisted",
                 noise: Union[str, torch.Tensor] = "torch", seed: int = 0,
                 member_offset: int = 0, precision: Optional[str] = None,
                 shared_condition: bool = False, n_members: Optional[int] = None):
    """Drop-in for sample_model (ERT_Conditional_Diffusion.py:102-119).

    Returns x_0 (B, param_dim) in the unconstrained space.  Extra keywords:
    mode ("hoisted"|"faithful"|"faithful_steps"), noise ("torch"|"philox"|tensor), seed and
    member_offset (philox), precision ("fp32"|"bf16", default: the model's),
    shared_condition + n_members: one (1,14,L) / (14,L) condition shared by
    n_members ensemble members (read in place, never replicated).
    """
    from .unet import ConditionalUNet, sample_unet
    if isinstance(model, ConditionalUNet):
        return sample_unet(model, condition, T, betas, alphas, alpha_bar, param_dim, device,
                           num_steps, temperature, noise=noise, seed=seed,
                           member_offset=member_offset, shared_condition=shared_condition,
                           n_members=n_members, precision=precision,
                           mode=None if mode == "hoisted" else mode)
    if mode not in _MODES:
        raise ValueError(f"mode must be one of {list(_MODES)}")
    dev = _lib.require_device(condition)
    model = as_ertdiff_model(model, dev)
    if model.param_dim != param_dim:
        raise RuntimeError(f"ertdiff: param_dim={param_dim} but the model predicts {model.param_dim}")
    prec = precision or model.precision
    prep = _Prepared(model, condition, T, betas, alphas, alpha_bar, num_steps, temperature, prec,
                     shared_condition)
    n = prep.num_steps
    if shared_condition:
        B = n_members if n_members is not None else (
            noise.shape[1] if isinstance(noise, torch.Tensor) else None)
        if B is None:
            raise RuntimeError("ertdiff: shared_condition needs n_members (or a noise tensor)")
    else:
        B = condition.shape[0]
    inj = None
    if isinstance(noise, torch.Tensor):
        inj = _lib.f32c(noise, "noise")
        if inj.shape != (n, inj.shape[1], param_dim):
            raise RuntimeError(f"ertdiff: noise must be (num_steps={n}, B, {param_dim}), got {tuple(noise.shape)}")
        B = inj.shape[1]
        _lib.require_device(inj, condition)
        x = inj[0].clone()
    elif noise == "torch":
        inj = draw_reference_noise(B, param_dim, n, device)
        if inj.device != dev:
            inj = inj.to(dev)
        x = inj[0].clone()
    elif noise == "philox":
        x = philox_normal(B, param_dim, n, 1, seed, member_offset, dev)
    else:
        raise ValueError("noise must be 'torch', 'philox' or a tensor")
    if not shared_condition and prep.cond.shape[0] != B:
        raise RuntimeError(f"ertdiff: condition batch {prep.cond.shape[0]} != noise batch {B}")
    ws = prep.workspace(B)
    with torch.cuda.device(dev):
        _lib.check(_lib.lib().ertd_sample(*prep.args(B, x, inj, seed, member_offset, mode,
                                                     n - 1, n, ws), _lib.stream_of(dev)), "sample")
    if mode != "hoisted" and sample_status(ws, B, prep.L, n) != 0:
        raise RuntimeError("ertdiff: the persistent faithful sampler timed out (GPU shared with "
                           "other work?); x is not valid")
    return x


def conditions_x_T(n_cond: int, n_samples: int, P: int, n: int, seed: int, cond_offset: int,
                   id_period: int, device) -> torch.Tensor:
    """x_T of a many-condition launch: realisation r's rows are the Philox
    draws of members cond_offset + r * id_period + (0 .. n_cond-1)."""
    x = torch.empty(n_samples * n_cond, P, dtype=torch.float32, device=device)
    for r in range(n_samples):
        x[r * n_cond:(r + 1) * n_cond] = philox_normal(n_cond, P, n, 1, seed, cond_offset + r * id_period,
                                                       device)
    return x


class _Conditions:
    """Geometry of a many-condition launch (ertd_sample_conditions)."""

    def __init__(self, prep, n_samples, cond_offset, n_conditions_total):
        self.n_cond = prep.cond.shape[0]
        self.n_samples = int(n_samples)
        self.cond_offset = int(cond_offset)
        self.period = self.n_cond if n_conditions_total is None else int(n_conditions_total)
        if self.n_samples < 1 or self.cond_offset < 0 or self.period < self.cond_offset + self.n_cond:
            raise RuntimeError("ertdiff: need n_samples >= 1 and cond_offset + n_cond <= n_conditions_total")
        if prep.stride == 0:
            raise RuntimeError("ertdiff: a many-condition launch reads (n_cond, 14, L) conditions")
        self.B = self.n_cond * self.n_samples

    def args(self, prep, x, noise, seed, mode, t_first, n_run, ws):
        tb = prep.tables
        return (ctypes.byref(prep.w), prep.packed.data_ptr(), prep.cond.data_ptr(), self.n_cond,
                self.n_samples, self.period, prep.L, prep.num_steps, t_first, n_run, tb[0].data_ptr(),
                tb[1].data_ptr(), tb[2].data_ptr(), prep.freq.data_ptr(), _lib.ptr(noise),
                int(seed) & (2**64 - 1), self.cond_offset & 0xFFFFFFFF, _MODES[mode], prep.prec,
                x.data_ptr(), ws.data_ptr(), ws.numel())


@torch.no_grad()
def sample_conditions(model, conditions, n_samples: int, T, betas, alphas, alpha_bar, param_dim,
                      device, num_steps=None, temperature=1.0, *, mode: str = "hoisted",
                      seed: int = 0, cond_offset: int = 0,
                      n_conditions_total: Optional[int] = None,
                      noise: Union[str, torch.Tensor] = "philox",
                      precision: Optional[str] = None) -> torch.Tensor:
    """The reference's test-set uncertainty evaluation (ERT_Conditional_Diffusion.py
    :1042-1069: `uncertainty_samples` calls of sample_model per test batch) as
    ONE sampler launch over every (realisation, condition) pair.

    conditions: (n_cond, 14, L).  Returns x_0 as (n_samples, n_cond, P) -- the
    reference's `Uncertainty_params` layout (:1073), unconstrained space.
    Member (r, c) is Philox member id cond_offset + r * n_conditions_total + c
    (n_conditions_total defaults to n_cond), i.e. realisation r draws exactly
    what sample_model(..., noise="philox", seed=seed, member_offset=
    r * n_conditions_total + cond_offset) draws for these conditions -- so a
    rank holding the condition slice [cond_offset, cond_offset + n_cond) of N
    computes exactly its columns of the whole evaluation.  mode="hoisted" runs
    the condition encoder once per condition; "faithful" re-runs it per member
    and step as the reference does.  noise: "philox", or an injected
    (num_steps, n_samples * n_cond, P) tensor."""
    if mode not in _MODES:
        raise ValueError(f"mode must be one of {list(_MODES)}")
    dev = _lib.require_device(conditions)
    model = as_ertdiff_model(model, dev)
    if model.param_dim != param_dim:
        raise RuntimeError(f"ertdiff: param_dim={param_dim} but the model predicts {model.param_dim}")
    prep = _Prepared(model, conditions, T, betas, alphas, alpha_bar, num_steps, temperature,
                     precision or model.precision, False)
    geo = _Conditions(prep, n_samples, cond_offset, n_conditions_total)
    n = prep.num_steps
    inj = None
    if isinstance(noise, torch.Tensor):
        inj = _lib.f32c(noise, "noise")
        if tuple(inj.shape) != (n, geo.B, param_dim):
            raise RuntimeError(f"ertdiff: noise must be (num_steps={n}, {geo.B}, {param_dim})")
        x = inj[0].clone()
    elif noise == "philox":
        x = conditions_x_T(geo.n_cond, geo.n_samples, param_dim, n, seed, geo.cond_offset, geo.period,
                           dev)
    else:
        raise ValueError("noise must be 'philox' or a tensor")
    ws = prep.workspace(geo.B)
    with torch.cuda.device(dev):
        _lib.check(_lib.lib().ertd_sample_conditions(*geo.args(prep, x, inj, seed, mode, n - 1, n, ws),
                                                     _lib.stream_of(dev)), "sample_conditions")
    if mode != "hoisted" and sample_status(ws, geo.B, prep.L, n) != 0:
        raise RuntimeError("ertdiff: the persistent faithful sampler timed out; x is not valid")
    return x.view(geo.n_samples, geo.n_cond, param_dim)


class SamplerPlan:
    """A captured hipGraph of ``n_run`` sampler steps starting at ``t_first``.

    All buffers are bound at construction; ``launch()`` replays every kernel of
    every step with one host call.  ``x`` holds the state in/out (set it to
    x_T before the first segment of a chain).  Used by bench.py and by the
    ensemble driver for long chains.
    """

    def __init__(self, model, condition, T, betas, alphas, alpha_bar, *, num_steps=None,
                 t_first=None, n_run=None, temperature=1.0, mode="faithful", seed=0,
                 member_offset=0, B=None, precision=None, shared_condition=False,
                 noise: Optional[torch.Tensor] = None, n_samples: Optional[int] = None,
                 n_conditions_total: Optional[int] = None):
        """n_samples: a many-condition plan (ertd_sample_conditions_plan_create):
        condition (n_cond, 14, L), B = n_samples * n_cond members in the
        sample_conditions layout, member_offset = the condition offset."""
        dev = _lib.require_device(condition)
        model = as_ertdiff_model(model, dev)
        self.prep = _Prepared(model, condition, T, betas, alphas, alpha_bar, num_steps,
                              temperature, precision or model.precision, shared_condition)
        n = self.prep.num_steps
        self.t_first = n - 1 if t_first is None else int(t_first)
        self.n_run = (self.t_first + 1) if n_run is None else int(n_run)
        self.geo = None if n_samples is None else _Conditions(self.prep, n_samples, member_offset,
                                                              n_conditions_total)
        self.B = self.geo.B if self.geo else (B if B is not None else self.prep.cond.shape[0])
        self.noise = None if noise is None else _lib.f32c(noise, "noise")
        self.x = torch.zeros(self.B, model.param_dim, dtype=torch.float32, device=dev)
        self.ws = self.prep.workspace(self.B)
        self.mode = mode
        self.seed = seed
        self.member_offset = member_offset
        self.dev = dev
        self._plan = ctypes.c_void_p()
        with torch.cuda.device(dev):
            if self.geo:
                _lib.check(_lib.lib().ertd_sample_conditions_plan_create(
                    *self.geo.args(self.prep, self.x, self.noise, seed, mode, self.t_first, self.n_run,
                                   self.ws), ctypes.byref(self._plan)), "sample_conditions_plan_create")
            else:
                _lib.check(_lib.lib().ertd_sample_plan_create(
                    *self.prep.args(self.B, self.x, self.noise, seed, member_offset, mode,
                                    self.t_first, self.n_run, self.ws), ctypes.byref(self._plan)),
                    "sample_plan_create")

    def launch(self, stream: Optional[torch.cuda.Stream] = None):
        s = (stream or torch.cuda.current_stream(self.dev)).cuda_stream
        with torch.cuda.device(self.dev):
            _lib.check(_lib.lib().ertd_plan_launch(self._plan, s), "plan_launch")

    def enqueue_direct(self, stream: Optional[torch.cuda.Stream] = None):
        """Same work as launch() but as eager launches (no graph), for comparison."""
        s = (stream or torch.cuda.current_stream(self.dev)).cuda_stream
        with torch.cuda.device(self.dev):
            if self.geo:
                _lib.check(_lib.lib().ertd_sample_conditions(
                    *self.geo.args(self.prep, self.x, self.noise, self.seed, self.mode, self.t_first,
                                   self.n_run, self.ws), s), "sample_conditions")
            else:
                _lib.check(_lib.lib().ertd_sample(
                    *self.prep.args(self.B, self.x, self.noise, self.seed, self.member_offset,
                                    self.mode, self.t_first, self.n_run, self.ws), s), "sample")

    def status(self) -> int:
        """0, or the timeout code of the last faithful replay (synchronizes)."""
        return sample_status(self.ws, self.B, self.prep.L, self.prep.num_steps)

    def close(self):
        if self._plan:
            _lib.lib().ertd_plan_destroy(self._plan)
            self._plan = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
