"""Build-defined conditional U-Net denoiser (SURVEY.md 8a', BASELINE north_star).

PARITY UNPINNED vs the reference: ERT_Conditional_Diffusion.py has no U-Net
(SURVEY.md 0.3).  The specification is oracle/unet_torch.py; the kernels are
in csrc/unet_conv.hip (3x3 / 1x1 convs as implicit GEMMs on fp32 MFMA, with
GroupNorm+SiLU fused into the input staging and bias / embedding / residual
adds fused into the epilogue), csrc/unet_ops.hip (GroupNorm statistics,
embedding-path dense layers, mid-block attention, DDPM update) and
csrc/unet_capi.hip (the layer walk and the sampler step graph).

The call surface is the reference's: ``ConditionalUNet`` is an ``nn.Module``
whose forward is ``model(x (B, image^2), t (B,), condition (B,14,L))`` like
ConditionalDiffusionModel.forward (:155-164), so ``x`` keeps the (B,
param_dim) contract of sample_model (:107); ``sample_model`` dispatches to
``sample_unet`` when handed a ConditionalUNet.
"""
from __future__ import annotations

import ctypes
import math
from typing import Dict, List, Optional, Sequence, Tuple, Union

import torch
import torch.nn as nn

from . import _lib
from .schedule import step_tables, timestep_frequencies


class ErtdUnetConfig(ctypes.Structure):
    _fields_ = [("image", ctypes.c_int), ("ch", ctypes.c_int), ("n_levels", ctypes.c_int),
                ("ch_mult", ctypes.c_int * 4), ("num_res", ctypes.c_int), ("attn", ctypes.c_int),
                ("groups", ctypes.c_int), ("precision", ctypes.c_int)]


# SURVEY.md 8a' table (U4 = U2's network on the 1024-member ensemble)
CONFIGS: Dict[str, dict] = {
    "U1": dict(image=32, ch=32, ch_mult=(1, 2), num_res=2, attn=False),
    "U2": dict(image=64, ch=64, ch_mult=(1, 2, 4), num_res=2, attn=False),
    "U3": dict(image=64, ch=64, ch_mult=(1, 2, 4), num_res=2, attn=True),
    "U5": dict(image=128, ch=128, ch_mult=(1, 1, 2, 2), num_res=2, attn=True),
}


# "bf16x3": split-bf16 conv operands (hi + lo bf16 planes, 3 bf16 MFMAs per
# product, fp32 accumulate) -- the bf16 configs' MFMA path at ~2^-16 relative
# per product, inside the north star's 1e-4 rel-L2
_PRECISIONS = {"fp32": 0, "bf16": 1, "bf16x3": 2}
_PRECISION_NAMES = {v: k for k, v in _PRECISIONS.items()}


def make_config(image=64, ch=64, ch_mult: Sequence[int] = (1, 2, 4), num_res=2, attn=False,
                groups=32, precision: str = "fp32") -> ErtdUnetConfig:
    m = list(ch_mult) + [0] * (4 - len(ch_mult))
    return ErtdUnetConfig(int(image), int(ch), len(ch_mult), (ctypes.c_int * 4)(*m), int(num_res),
                          int(bool(attn)), int(groups), _PRECISIONS[precision])


def param_layout(cfg: ErtdUnetConfig) -> List[Tuple[str, Tuple[int, ...]]]:
    """(name, shape) of every parameter, in state_dict order, from the library."""
    lib = _lib.lib()
    n = lib.ertd_unet_n_params(ctypes.byref(cfg))
    if n < 0:
        raise RuntimeError("ertdiff: unsupported U-Net configuration")
    out = []
    name = ctypes.create_string_buffer(128)
    shape = (ctypes.c_int64 * 4)()
    nd = ctypes.c_int()
    for i in range(n):
        _lib.check(lib.ertd_unet_param_info(ctypes.byref(cfg), i, name, 128, shape,
                                            ctypes.byref(nd)), "unet_param_info")
        out.append((name.value.decode(), tuple(int(shape[j]) for j in range(nd.value))))
    return out


def unet_flops(image=64, ch=64, ch_mult: Sequence[int] = (1, 2, 4), num_res=2, attn=False,
               groups=32, batch: Optional[int] = None, cus: int = 256) -> Dict[str, int]:
    """Algorithmic FLOP per sample-step (multiply-add = 2) of the U-Net forward:
    convs, attention core (QK^T and PV) and the dense layers; elementwise work
    (GroupNorm, SiLU, adds) is not counted.  `conv_executed_fp32` is the MFMA
    work the fp32 kernels execute at batch `batch` on `cus` CUs (the 16x16
    level's kernel depends on the batch; None = the F(2x2) count there)."""
    cfg = make_config(image, ch, ch_mult, num_res, attn, groups)
    layout = param_layout(cfg)
    conv = dense = ups = ups4 = wino = wino4 = 0
    # spatial size per conv: walk the layout names
    res_of = {}
    r = image
    nl = len(ch_mult)
    for i in range(nl):
        res_of[f"down.{i}"] = r
        if i != nl - 1:
            r //= 2
    res_of["mid"] = r
    for i in reversed(range(nl)):
        res_of[f"up.{i}"] = image >> i

    def f4_items_fill(hw, cout):   # csrc/unet_conv_wino.hip wino4s_ok at W = 16
        return batch is not None and (hw // 4) ** 2 // 16 * batch * (cout // 64) >= cus

    for name, shape in layout:
        if not name.endswith(".weight") or name.startswith("condition_encoder"):
            continue
        parts = name.split(".")
        if len(shape) == 4:
            if parts[0] in ("conv_in", "conv_out"):
                hw = image
            elif parts[0] == "mid":
                hw = res_of["mid"]
            else:
                hw = res_of[f"{parts[0]}.{parts[1]}"]
                if parts[2] == "downsample":
                    hw //= 2
                elif parts[2] == "upsample":     # runs at the doubled resolution
                    hw *= 2
            f = 2 * shape[0] * shape[1] * shape[2] * shape[3] * hw * hw
            conv += f
            if len(parts) > 2 and parts[2] == "upsample":
                # F(4x4) on the nearest-x2 source (unet_conv_wino4s.hip, UP) where
                # wino4s_up_ok, else 4 sub-pixel 2x2 convs (4 of the 9 taps)
                if shape[1] % 8 == 0 and shape[0] % 64 == 0 and hw in (32, 64) or \
                        (hw == 16 and shape[1] % 8 == 0 and shape[0] % 64 == 0 and f4_items_fill(hw, shape[0])):
                    ups4 += f
                else:
                    ups += f
            # ResBlock 3x3 convs the fp32 Winograd kernels take: F(4x4,3x3) at
            # W >= 32 (unet_conv_wino4s.hip / unet_conv_wino4.hip) and at W = 16
            # where its tile items fill the CUs, else F(2x2,3x3) (unet_conv_wino.hip)
            if parts[-2] in ("conv1", "conv2") and shape[2] == 3 and shape[0] % 64 == 0:
                if (hw >= 32 and shape[1] % 4 == 0) or (hw == 16 and shape[1] % 8 == 0 and
                                                        f4_items_fill(hw, shape[0])):
                    wino4 += f
                elif shape[1] % 8 == 0:
                    wino += f
        elif len(shape) == 2:
            dense += 2 * shape[0] * shape[1]
    attn_f = 0
    if attn:
        C = ch * ch_mult[-1]
        N = res_of["mid"] ** 2
        attn_f = 2 * 2 * N * N * C
    enc = 6_308_736 + 14_426_112 + 2 * 64 * 128   # the reference's condition encoder
    # executed MFMA work: F(4x4,3x3) 36 multiplies per 4x4 outputs instead of
    # 144, F(2x2,3x3) 16 per 2x2 instead of 36, sub-pixel Upsample 4 of 9 taps
    return {"conv": conv, "attention": attn_f, "dense": dense, "condition_encoder": enc,
            "total": conv + attn_f + dense + enc,
            "conv_winograd": wino + wino4 + ups4,
            "conv_winograd_f4": wino4 + ups4,
            "conv_executed_fp32": conv - ups * 5 // 9 - wino * 5 // 9 - (wino4 + ups4) * 3 // 4}


class ConditionalUNet(nn.Module):
    """eps(x, t, condition) with a 2-D U-Net over x viewed as (B,1,image,image).

    Parameters are registered as nested modules so the state_dict keys and
    order are those of oracle/unet_torch.layer_shapes (and of the library's
    enumeration).  Init: uniform(+-1/sqrt(fan_in)) for conv/linear weights and
    biases (PyTorch's default bound), GroupNorm weight 1 / bias 0.
    """

    def __init__(self, image=64, ch=64, ch_mult: Sequence[int] = (1, 2, 4), num_res=2, attn=False,
                 groups=32, seed: Optional[int] = None, precision: str = "fp32"):
        super().__init__()
        self.spec = dict(image=image, ch=ch, ch_mult=tuple(ch_mult), num_res=num_res, attn=attn,
                         groups=groups)
        self.cfg = make_config(image, ch, ch_mult, num_res, attn, groups, precision)
        self.image = image
        self.param_dim = image * image
        self.layout = param_layout(self.cfg)
        g = torch.Generator().manual_seed(seed) if seed is not None else None
        shapes = dict(self.layout)
        for name, shape in self.layout:
            parts = name.split(".")
            mod = self
            for p in parts[:-1]:
                if not hasattr(mod, p) or not isinstance(getattr(mod, p), nn.Module):
                    mod.add_module(p, nn.Module())
                mod = getattr(mod, p)
            if ".norm" in name or name.startswith("norm_out"):
                val = torch.ones(shape) if parts[-1] == "weight" else torch.zeros(shape)
            else:
                wshape = shape if parts[-1] == "weight" else shapes[name[:-4] + "weight"]
                fan_in = int(math.prod(wshape[1:]))
                bound = 1.0 / math.sqrt(fan_in)
                val = (torch.rand(shape, generator=g) * 2 - 1) * bound
            mod.register_parameter(parts[-1], nn.Parameter(val))
        keys = list(self.state_dict().keys())
        if keys != [n for n, _ in self.layout]:
            raise RuntimeError("ertdiff: U-Net state_dict order differs from the library's")
        self._packed: Optional[torch.Tensor] = None
        self._packed_key = None
        self._ws: Dict = {}

    @classmethod
    def from_config(cls, name: str, seed: Optional[int] = None,
                    precision: str = "fp32") -> "ConditionalUNet":
        return cls(**CONFIGS[name], seed=seed, precision=precision)

    @property
    def precision(self) -> str:
        return _PRECISION_NAMES[self.cfg.precision]

    def set_precision(self, precision: str) -> None:
        """fp32 convs (default), bf16 conv operands with fp32 accumulation, or
        "bf16x3" split-bf16 operands; the packed weights are rebuilt on the
        next call."""
        self.cfg.precision = _PRECISIONS[precision]
        self._packed = None
        self._packed_key = None
        self._ws = {}

    def _params(self) -> List[torch.Tensor]:
        sd = dict(self.named_parameters())
        return [sd[n] for n, _ in self.layout]

    def packed_weights(self, dev: torch.device) -> torch.Tensor:
        ps = self._params()
        key = tuple((p.data_ptr(), p._version) for p in ps)
        if self._packed is None or self._packed_key != key or self._packed.device != dev:
            for (n, _), p in zip(self.layout, ps):
                if p.dtype != torch.float32 or not p.is_contiguous() or p.device != dev:
                    raise RuntimeError(f"ertdiff: parameter {n} must be contiguous float32 on {dev}")
            lib = _lib.lib()
            nf = lib.ertd_unet_packed_floats(ctypes.byref(self.cfg))
            if self._packed is None or self._packed.device != dev:
                self._packed = torch.empty(nf, dtype=torch.float32, device=dev)
            arr = (ctypes.c_void_p * len(ps))(*[p.data_ptr() for p in ps])
            freq = timestep_frequencies(self.spec["ch"], dev)
            with torch.cuda.device(dev):
                _lib.check(lib.ertd_unet_pack(ctypes.byref(self.cfg), arr, freq.data_ptr(),
                                              self._packed.data_ptr(), _lib.stream_of(dev)),
                           "unet_pack")
            self._packed_key = key
        return self._packed

    def workspace(self, dev: torch.device, B: int, L: int) -> torch.Tensor:
        n = _lib.lib().ertd_unet_workspace_bytes(ctypes.byref(self.cfg), B, L)
        if n == 0:
            raise RuntimeError("ertdiff: unsupported U-Net configuration")
        ws = self._ws.get(dev)
        if ws is None or ws.numel() < n:
            self._ws.pop(dev, None)
            ws = torch.empty(n, dtype=torch.uint8, device=dev)
            self._ws[dev] = ws
        return ws

    def forward(self, x: torch.Tensor, t: torch.Tensor, condition: torch.Tensor,
                return_cond_emb: bool = False):
        """eps (B, image^2).  With autograd recording and x or any parameter
        requiring grad (the reference train loop, ERT_Conditional_Diffusion.py:
        314-318), the call runs the train-mode forward (saved activations) and
        loss.backward() runs the HIP backward (ertdiff.unet_train.UNetForwardFn);
        otherwise (no_grad, return_cond_emb) the inference forward
        (ertd_unet_forward).  The bf16-operand precision has no backward: under
        autograd it raises instead of returning a tensor that silently does
        not require grad."""
        if (torch.is_grad_enabled() and not return_cond_emb and
                (x.requires_grad or any(p.requires_grad for p in self.parameters()))):
            if self.precision != "fp32":
                raise RuntimeError(
                    "ertdiff: the bf16-operand U-Net has no backward; call it under torch.no_grad() "
                    "for inference (sample_model does) or model.set_precision('fp32') to train")
            from .unet_train import UNetForwardFn
            dev = _lib.require_device(x, t, condition, self.conv_in.weight)
            self._check_call(x, t, condition)
            return UNetForwardFn.apply(self, _lib.f32c(x, "x"), t.to(device=dev, dtype=torch.int64)
                                       .contiguous(), _lib.f32c(condition, "condition"),
                                       *self._params())
        return self._infer(x, t, condition, return_cond_emb)

    def _check_call(self, x, t, cond):
        B = x.shape[0]
        if x.dim() != 2 or x.shape[1] != self.param_dim:
            raise RuntimeError(f"ertdiff: x must be (B, {self.param_dim}), got {tuple(x.shape)}")
        if cond.dim() != 3 or cond.shape[0] != B or cond.shape[1] != _lib.CIN:
            raise RuntimeError(f"ertdiff: condition must be (B, 14, L), got {tuple(cond.shape)}")
        if t.shape != (B,):
            raise RuntimeError(f"ertdiff: t must be (B,), got {tuple(t.shape)}")

    @torch.no_grad()
    def _infer(self, x: torch.Tensor, t: torch.Tensor, condition: torch.Tensor,
               return_cond_emb: bool = False):
        dev = _lib.require_device(x, t, condition, self.conv_in.weight)
        x = _lib.f32c(x, "x")
        cond = _lib.f32c(condition, "condition")
        B = x.shape[0]
        if x.dim() != 2 or x.shape[1] != self.param_dim:
            raise RuntimeError(f"ertdiff: x must be (B, {self.param_dim}), got {tuple(x.shape)}")
        if cond.dim() != 3 or cond.shape[0] != B or cond.shape[1] != _lib.CIN:
            raise RuntimeError(f"ertdiff: condition must be (B, 14, L), got {tuple(cond.shape)}")
        tt = t.to(torch.int64).contiguous()
        if tt.shape != (B,):
            raise RuntimeError(f"ertdiff: t must be (B,), got {tuple(t.shape)}")
        L = cond.shape[2]
        out = torch.empty(B, self.param_dim, dtype=torch.float32, device=dev)
        cemb = torch.empty(B, _lib.HIDDEN, dtype=torch.float32, device=dev) if return_cond_emb else None
        packed = self.packed_weights(dev)
        ws = self.workspace(dev, B, L)
        with torch.cuda.device(dev):
            _lib.check(_lib.lib().ertd_unet_forward(
                ctypes.byref(self.cfg), packed.data_ptr(), x.data_ptr(), tt.data_ptr(),
                cond.data_ptr(), _lib.CIN * L, L, B, out.data_ptr(), _lib.ptr(cemb), ws.data_ptr(),
                ws.numel(), _lib.stream_of(dev)), "unet_forward")
        return (out, cemb) if return_cond_emb else out


class _UPrepared:
    def __init__(self, model: ConditionalUNet, condition, T, betas, alphas, alpha_bar, num_steps,
                 temperature, shared_condition):
        dev = _lib.require_device(condition, model.conv_in.weight)
        self.dev = dev
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
        self.model = model
        self.packed = model.packed_weights(dev)

    def args(self, B, x, noise, seed, member_offset, t_first, n_run, ws):
        tb = self.tables
        return (ctypes.byref(self.model.cfg), self.packed.data_ptr(), self.cond.data_ptr(),
                self.stride, self.L, B, self.num_steps, t_first, n_run, tb[0].data_ptr(),
                tb[1].data_ptr(), tb[2].data_ptr(), _lib.ptr(noise), int(seed) & (2**64 - 1),
                int(member_offset) & 0xFFFFFFFF, x.data_ptr(), ws.data_ptr(), ws.numel())


@torch.no_grad()
def sample_unet(model: ConditionalUNet, condition, T, betas, alphas, alpha_bar, param_dim, device,
                num_steps=None, temperature=1.0, *, noise: Union[str, torch.Tensor] = "torch",
                seed: int = 0, member_offset: int = 0, shared_condition: bool = False,
                n_members: Optional[int] = None, precision: Optional[str] = None,
                mode: Optional[str] = None):
    """sample_model (ERT_Conditional_Diffusion.py:102-119) with the U-Net
    denoiser: same signature, same noise options as ertdiff.sample_model.
    ``precision`` must be None or the model's own (ConditionalUNet.set_precision
    changes it); ``mode`` is a reference-model option: the U-Net has a single
    schedule, so anything but None raises instead of being ignored."""
    from .sampler import draw_reference_noise, philox_normal
    if precision is not None and precision != model.precision:
        raise RuntimeError(f"ertdiff: precision={precision!r} but the U-Net runs {model.precision!r}; "
                           "call model.set_precision() first")
    if mode is not None:
        raise RuntimeError(f"ertdiff: mode={mode!r} applies to ConditionalDiffusionModel only")
    if model.param_dim != param_dim:
        raise RuntimeError(f"ertdiff: param_dim={param_dim} but the U-Net predicts {model.param_dim}")
    prep = _UPrepared(model, condition, T, betas, alphas, alpha_bar, num_steps, temperature,
                      shared_condition)
    n = prep.num_steps
    dev = prep.dev
    B = n_members if shared_condition else prep.cond.shape[0]
    inj = None
    if isinstance(noise, torch.Tensor):
        inj = _lib.f32c(noise, "noise")
        if inj.dim() != 3 or inj.shape[0] != n or inj.shape[2] != param_dim:
            raise RuntimeError(f"ertdiff: noise must be (num_steps={n}, B, {param_dim})")
        B = inj.shape[1]
        x = inj[0].clone()
    elif noise == "torch":
        if B is None:
            raise RuntimeError("ertdiff: shared_condition needs n_members")
        inj = draw_reference_noise(B, param_dim, n, device).to(dev)
        x = inj[0].clone()
    elif noise == "philox":
        x = philox_normal(B, param_dim, n, 1, seed, member_offset, dev)
    else:
        raise ValueError("noise must be 'torch', 'philox' or a tensor")
    if not shared_condition and prep.cond.shape[0] != B:
        raise RuntimeError(f"ertdiff: condition batch {prep.cond.shape[0]} != noise batch {B}")
    ws = model.workspace(dev, B, prep.L)
    with torch.cuda.device(dev):
        _lib.check(_lib.lib().ertd_unet_sample(*prep.args(B, x, inj, seed, member_offset, n - 1, n,
                                                          ws), _lib.stream_of(dev)), "unet_sample")
    return x


class UNetSamplerPlan:
    """hipGraph plan of one U-Net sampler call (head graph + one step graph
    replayed n_run times); ``x`` holds the state, set it to x_T before launch."""

    def __init__(self, model: ConditionalUNet, condition, T, betas, alphas, alpha_bar, *,
                 num_steps=None, t_first=None, n_run=None, temperature=1.0, seed=0,
                 member_offset=0, B=None, shared_condition=False,
                 noise: Optional[torch.Tensor] = None):
        self.prep = _UPrepared(model, condition, T, betas, alphas, alpha_bar, num_steps,
                               temperature, shared_condition)
        n = self.prep.num_steps
        dev = self.prep.dev
        self.dev = dev
        self.t_first = n - 1 if t_first is None else int(t_first)
        self.n_run = self.t_first + 1 if n_run is None else int(n_run)
        self.B = B if B is not None else self.prep.cond.shape[0]
        self.noise = None if noise is None else _lib.f32c(noise, "noise")
        self.x = torch.zeros(self.B, model.param_dim, dtype=torch.float32, device=dev)
        # a workspace of its own (step counter, eps, embedding biases, every
        # activation): a plan launched on another stream never races the
        # model's eager calls or another plan
        nbytes = _lib.lib().ertd_unet_workspace_bytes(ctypes.byref(model.cfg), self.B, self.prep.L)
        if nbytes == 0:
            raise RuntimeError("ertdiff: unsupported U-Net configuration")
        self.ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        self._plan = ctypes.c_void_p()
        with torch.cuda.device(dev):
            _lib.check(_lib.lib().ertd_unet_sample_plan_create(
                *self.prep.args(self.B, self.x, self.noise, seed, member_offset, self.t_first,
                                self.n_run, self.ws), ctypes.byref(self._plan)),
                "unet_sample_plan_create")

    def launch(self, stream: Optional[torch.cuda.Stream] = None, n_steps: Optional[int] = None):
        """Replays the head graph and n_run steps (or only the first n_steps)."""
        s = (stream or torch.cuda.current_stream(self.dev)).cuda_stream
        with torch.cuda.device(self.dev):
            if n_steps is None:
                _lib.check(_lib.lib().ertd_unet_plan_launch(self._plan, s), "unet_plan_launch")
            else:
                _lib.check(_lib.lib().ertd_unet_plan_launch_steps(self._plan, int(n_steps), s),
                           "unet_plan_launch_steps")

    def close(self):
        if self._plan:
            _lib.lib().ertd_unet_plan_destroy(self._plan)
            self._plan = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---- single operators (ertd_conv2d / ertd_group_norm_stats / ertd_group_norm_act_bf16 /
#      ertd_attention) ----------
_MODES2D = {"same": 0, "down": 1, "up": 2}
_ACTS = {"none": 0, "gn_silu": 1, "gn": 2}


def conv2d(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, *, mode: str = "same",
           act: str = "none", gn: Optional[torch.Tensor] = None, x2: Optional[torch.Tensor] = None,
           ebias: Optional[torch.Tensor] = None, res: Optional[torch.Tensor] = None,
           precision: str = "fp32") -> torch.Tensor:
    """One U-Net convolution on the HIP kernel: conv(act(cat(x, x2))) + bias
    (+ ebias[:, :, None, None]) (+ res); padding 1 for 3x3 (stride 2 for
    mode="down", nearest x2 upsample first for mode="up").  gn: (B, Cin, 2)
    {scale, shift} as returned by group_norm_stats."""
    dev = _lib.require_device(x, weight, bias)
    x = _lib.f32c(x, "x")
    B, Ca, H, _ = x.shape
    Cb = 0 if x2 is None else x2.shape[1]
    Cout, Cin, ks, _ = weight.shape
    if Cin != Ca + Cb:
        raise RuntimeError("ertdiff: weight in-channels != input channels")
    Ho = H // 2 if mode == "down" else (2 * H if mode == "up" else H)
    out = torch.empty(B, Cout, Ho, Ho, dtype=torch.float32, device=dev)
    prec = _PRECISIONS[precision]
    n = _lib.lib().ertd_conv2d_workspace_bytes(Cin, Cout, ks, prec, B, H, _MODES2D[mode])
    if n == 0:
        raise RuntimeError("ertdiff: unsupported conv2d geometry")
    ws = torch.empty(n, dtype=torch.uint8, device=dev)
    w = _lib.f32c(weight, "weight")
    bb = _lib.f32c(bias, "bias")
    eb = None if ebias is None else _lib.f32c(ebias, "ebias")
    with torch.cuda.device(dev):
        _lib.check(_lib.lib().ertd_conv2d(
            x.data_ptr(), Ca, _lib.ptr(None if x2 is None else _lib.f32c(x2, "x2")), Cb, B, H,
            w.data_ptr(), bb.data_ptr(), Cout, ks, _MODES2D[mode],
            _lib.ptr(None if gn is None else _lib.f32c(gn, "gn")), _ACTS[act], _lib.ptr(eb),
            0 if eb is None else eb.shape[1], _lib.ptr(None if res is None else _lib.f32c(res, "res")),
            out.data_ptr(), prec, ws.data_ptr(), ws.numel(), _lib.stream_of(dev)), "conv2d")
    return out


def group_norm_stats(x: torch.Tensor, groups: int, gamma: torch.Tensor, beta: torch.Tensor,
                     x2: Optional[torch.Tensor] = None) -> torch.Tensor:
    """(B, C, 2) {scale, shift}: GroupNorm(cat(x, x2)) == x*scale + shift per channel."""
    dev = _lib.require_device(x, gamma, beta)
    x = _lib.f32c(x, "x")
    B, Ca, H, W = x.shape
    Cb = 0 if x2 is None else x2.shape[1]
    out = torch.empty(B, Ca + Cb, 2, dtype=torch.float32, device=dev)
    with torch.cuda.device(dev):
        _lib.check(_lib.lib().ertd_group_norm_stats(
            x.data_ptr(), Ca, _lib.ptr(None if x2 is None else _lib.f32c(x2, "x2")), Cb, B, H * W,
            groups, _lib.f32c(gamma, "gamma").data_ptr(), _lib.f32c(beta, "beta").data_ptr(),
            out.data_ptr(), _lib.stream_of(dev)), "group_norm_stats")
    return out


def group_norm_act_bf16(x: torch.Tensor, groups: int, gamma: torch.Tensor, beta: torch.Tensor,
                        x2: Optional[torch.Tensor] = None, silu: bool = True):
    """The bf16 path's fused 3x3-conv prologue: ((B, C, 2) {scale, shift} as
    group_norm_stats, (B, C/16, H, W, 16) int16 bf16 bits of
    act(GroupNorm(cat(x, x2)))) in one pass over x."""
    dev = _lib.require_device(x, gamma, beta)
    x = _lib.f32c(x, "x")
    B, Ca, H, W = x.shape
    Cb = 0 if x2 is None else x2.shape[1]
    C = Ca + Cb
    out = torch.empty(B, C, 2, dtype=torch.float32, device=dev)
    img = torch.empty(B, (C + 15) // 16, H, W, 16, dtype=torch.int16, device=dev)
    with torch.cuda.device(dev):
        _lib.check(_lib.lib().ertd_group_norm_act_bf16(
            x.data_ptr(), Ca, _lib.ptr(None if x2 is None else _lib.f32c(x2, "x2")), Cb, B, H,
            groups, _lib.f32c(gamma, "gamma").data_ptr(), _lib.f32c(beta, "beta").data_ptr(),
            out.data_ptr(), img.data_ptr(), 1 if silu else 0, _lib.stream_of(dev)),
            "group_norm_act_bf16")
    return out, img


def attention(qkv: torch.Tensor) -> torch.Tensor:
    """qkv (B, 3C, N) -> (B, C, N): v softmax(q^T k / sqrt(C))^T (single head)."""
    dev = _lib.require_device(qkv)
    qkv = _lib.f32c(qkv, "qkv")
    B, C3, N = qkv.shape
    out = torch.empty(B, C3 // 3, N, dtype=torch.float32, device=dev)
    with torch.cuda.device(dev):
        _lib.check(_lib.lib().ertd_attention(qkv.data_ptr(), B, C3 // 3, N, out.data_ptr(),
                                             _lib.stream_of(dev)), "attention")
    return out
