"""ORACLE (test infrastructure only) -- PyTorch-CPU definition of the
build-defined conditional U-Net denoiser (SURVEY.md 8a', BASELINE.json
north_star).  PARITY UNPINNED vs the reference: the reference has no U-Net
(SURVEY.md 0.3); this module IS the specification the HIP path is checked
against, and bench.py's CPU baseline leg for the U-configs.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
it.  Functional: weights are a dict keyed like ertdiff.ConditionalUNet's
state_dict.

Architecture (U1/U2/U3/U5 differ only in the config):
  x (B, H*W) -> (B, 1, H, W)                       [sample_model keeps (B, P)]
  emb = time_embed(sinusoid(t, ch)) + cond_proj(condition_encoder(cond))
        time_embed = Linear(ch, 4ch) -> SiLU -> Linear(4ch, 4ch)
        condition_encoder = the reference's 1-D CNN (ERT_Conditional_Diffusion.py:133-142)
        cond_proj = Linear(128, 4ch)
  h = conv_in(x)                                   3x3, 1 -> ch
  down level i (channels ch*mult[i]): num_res ResBlocks, then (not last) a
        stride-2 3x3 Downsample; every output is kept for the skips
  mid: ResBlock, [Attention], ResBlock
  up level i (reversed): num_res+1 ResBlocks on cat([h, skip]), then (i>0)
        Upsample = nearest x2 -> 3x3 conv
  out = conv_out(SiLU(GroupNorm(h)))               3x3, ch -> 1, back to (B, H*W)
ResBlock(cin, cout):
  h = conv1(SiLU(GN1(x))) + emb_proj(SiLU(emb))[:, :, None, None]
  h = conv2(SiLU(GN2(h)))
  out = skip(x) + h          skip = 1x1 conv when cin != cout, else identity
Attention(C) (single head, N = H*W tokens):
  q, k, v = qkv(GN(x)) (1x1, C -> 3C);  a = softmax(q^T k / sqrt(C)) over keys
  out = x + proj(v a^T)
GroupNorm: 32 groups, eps 1e-5, affine.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Tuple

import torch
import torch.nn.functional as F

Weights = Dict[str, torch.Tensor]


@dataclass(frozen=True)
class UNetConfig:
    image: int = 64
    ch: int = 64
    ch_mult: Tuple[int, ...] = (1, 2, 4)
    num_res: int = 2
    attn: bool = False
    groups: int = 32
    cond_channels: int = 14
    hidden: int = 128

    @property
    def param_dim(self) -> int:
        return self.image * self.image

    @property
    def temb(self) -> int:
        return 4 * self.ch


CONFIGS = {
    "U1": UNetConfig(image=32, ch=32, ch_mult=(1, 2)),
    "U2": UNetConfig(image=64, ch=64, ch_mult=(1, 2, 4)),
    "U3": UNetConfig(image=64, ch=64, ch_mult=(1, 2, 4), attn=True),
    "U5": UNetConfig(image=128, ch=128, ch_mult=(1, 1, 2, 2), attn=True),
}


def layer_shapes(cfg: UNetConfig) -> List[Tuple[str, Tuple[int, ...]]]:
    """Every parameter (name, shape) in registration order."""
    out: List[Tuple[str, Tuple[int, ...]]] = []
    H = cfg.hidden

    def lin(n, i, o):
        out.extend([(f"{n}.weight", (o, i)), (f"{n}.bias", (o,))])

    def conv(n, i, o, k):
        out.extend([(f"{n}.weight", (o, i, k, k)), (f"{n}.bias", (o,))])

    def gn(n, c):
        out.extend([(f"{n}.weight", (c,)), (f"{n}.bias", (c,))])

    def res(n, i, o):
        gn(f"{n}.norm1", i)
        conv(f"{n}.conv1", i, o, 3)
        lin(f"{n}.emb", cfg.temb, o)
        gn(f"{n}.norm2", o)
        conv(f"{n}.conv2", o, o, 3)
        if i != o:
            conv(f"{n}.skip", i, o, 1)

    out.extend([("condition_encoder.0.weight", (32, cfg.cond_channels, 3)),
                ("condition_encoder.0.bias", (32,)),
                ("condition_encoder.2.weight", (64, 32, 3)), ("condition_encoder.2.bias", (64,)),
                ("condition_encoder.6.weight", (H, 64)), ("condition_encoder.6.bias", (H,))])
    lin("time_embed.0", cfg.ch, cfg.temb)
    lin("time_embed.2", cfg.temb, cfg.temb)
    lin("cond_proj", H, cfg.temb)
    conv("conv_in", 1, cfg.ch, 3)
    chans = [cfg.ch]
    c = cfg.ch
    nl = len(cfg.ch_mult)
    for i, m in enumerate(cfg.ch_mult):
        for r in range(cfg.num_res):
            res(f"down.{i}.res.{r}", c, cfg.ch * m)
            c = cfg.ch * m
            chans.append(c)
        if i != nl - 1:
            conv(f"down.{i}.downsample", c, c, 3)
            chans.append(c)
    res("mid.res1", c, c)
    if cfg.attn:
        gn("mid.attn.norm", c)
        conv("mid.attn.qkv", c, 3 * c, 1)
        conv("mid.attn.proj", c, c, 1)
    res("mid.res2", c, c)
    for i in reversed(range(nl)):
        for r in range(cfg.num_res + 1):
            res(f"up.{i}.res.{r}", c + chans.pop(), cfg.ch * cfg.ch_mult[i])
            c = cfg.ch * cfg.ch_mult[i]
        if i != 0:
            conv(f"up.{i}.upsample", c, c, 3)
    gn("norm_out", c)
    conv("conv_out", c, 1, 3)
    return out


def sinusoid(t: torch.Tensor, dim: int) -> torch.Tensor:
    """The reference's get_timestep_embedding (ERT_Conditional_Diffusion.py:80-88)."""
    half = dim // 2
    scale = math.log(10000.0) / (half - 1)
    freqs = torch.exp(torch.arange(half, dtype=torch.float32) * -scale)
    arg = t.float().unsqueeze(1) * freqs.unsqueeze(0)
    return torch.cat([torch.sin(arg), torch.cos(arg)], dim=1)


def _conv_bf16(x, w, b, **kw):
    """The bf16-operand conv of the HIP path (cfg precision bf16): the conv
    input (after GroupNorm/SiLU) and the weights are rounded to bf16 (RNE),
    products and sums in fp32."""
    return F.conv2d(x.bfloat16().float(), w.bfloat16().float(), b, **kw)


def _gn_silu(x, W, n, groups):
    return F.silu(F.group_norm(x, groups, W[f"{n}.weight"], W[f"{n}.bias"], eps=1e-5))


def _res(x, emb_act, W, n, groups, cv=F.conv2d):
    h = cv(_gn_silu(x, W, f"{n}.norm1", groups), W[f"{n}.conv1.weight"],
           W[f"{n}.conv1.bias"], padding=1)
    h = h + F.linear(emb_act, W[f"{n}.emb.weight"], W[f"{n}.emb.bias"])[:, :, None, None]
    h = cv(_gn_silu(h, W, f"{n}.norm2", groups), W[f"{n}.conv2.weight"],
           W[f"{n}.conv2.bias"], padding=1)
    if f"{n}.skip.weight" in W:
        x = cv(x, W[f"{n}.skip.weight"], W[f"{n}.skip.bias"])
    return x + h


def _attn(x, W, n, groups, cv=F.conv2d):
    B, C, Hh, Ww = x.shape
    qkv = cv(F.group_norm(x, groups, W[f"{n}.norm.weight"], W[f"{n}.norm.bias"], eps=1e-5),
             W[f"{n}.qkv.weight"], W[f"{n}.qkv.bias"]).reshape(B, 3, C, Hh * Ww)
    q, k, v = qkv[:, 0], qkv[:, 1], qkv[:, 2]
    a = torch.softmax(torch.einsum("bci,bcj->bij", q, k) / math.sqrt(C), dim=-1)
    o = torch.einsum("bij,bcj->bci", a, v).reshape(B, C, Hh, Ww)
    return x + cv(o, W[f"{n}.proj.weight"], W[f"{n}.proj.bias"])


def condition_embedding(cond, W):
    h = F.relu(F.conv1d(cond, W["condition_encoder.0.weight"], W["condition_encoder.0.bias"],
                        stride=2, padding=1))
    h = F.relu(F.conv1d(h, W["condition_encoder.2.weight"], W["condition_encoder.2.bias"],
                        stride=2, padding=1))
    h = h.mean(dim=2)
    return F.relu(F.linear(h, W["condition_encoder.6.weight"], W["condition_encoder.6.bias"]))


def embedding(t, cond, W, cfg: UNetConfig):
    # the sinusoid is fp32 (the reference's); a float64 weight dict runs the rest in float64
    s = sinusoid(t, cfg.ch).to(W["time_embed.0.weight"].dtype)
    e = F.linear(s, W["time_embed.0.weight"], W["time_embed.0.bias"])
    e = F.linear(F.silu(e), W["time_embed.2.weight"], W["time_embed.2.bias"])
    return e + F.linear(condition_embedding(cond, W), W["cond_proj.weight"], W["cond_proj.bias"])


def forward(x, t, cond, W: Weights, cfg: UNetConfig, return_emb: bool = False, bf16: bool = False):
    """eps; ``bf16`` = the HIP path's bf16-operand convs (``_conv_bf16``)."""
    B = x.shape[0]
    g = cfg.groups
    cv = _conv_bf16 if bf16 else F.conv2d
    emb = embedding(t, cond, W, cfg)
    ea = F.silu(emb)
    h = cv(x.reshape(B, 1, cfg.image, cfg.image), W["conv_in.weight"], W["conv_in.bias"],
           padding=1)
    hs = [h]
    nl = len(cfg.ch_mult)
    for i in range(nl):
        for r in range(cfg.num_res):
            h = _res(h, ea, W, f"down.{i}.res.{r}", g, cv)
            hs.append(h)
        if i != nl - 1:
            h = cv(h, W[f"down.{i}.downsample.weight"], W[f"down.{i}.downsample.bias"],
                   stride=2, padding=1)
            hs.append(h)
    h = _res(h, ea, W, "mid.res1", g, cv)
    if cfg.attn:
        h = _attn(h, W, "mid.attn", g, cv)
    h = _res(h, ea, W, "mid.res2", g, cv)
    for i in reversed(range(nl)):
        for r in range(cfg.num_res + 1):
            h = _res(torch.cat([h, hs.pop()], dim=1), ea, W, f"up.{i}.res.{r}", g, cv)
        if i != 0:
            h = F.interpolate(h, scale_factor=2, mode="nearest")
            h = cv(h, W[f"up.{i}.upsample.weight"], W[f"up.{i}.upsample.bias"], padding=1)
    h = _gn_silu(h, W, "norm_out", g)
    out = cv(h, W["conv_out.weight"], W["conv_out.bias"], padding=1).reshape(B, -1)
    return (out, emb) if return_emb else out


@torch.no_grad()
def sample(cond, W: Weights, cfg: UNetConfig, T: int, noise, num_steps=None, temperature=1.0,
           max_steps=None, bf16: bool = False, record=()):
    """sample_model (ERT_Conditional_Diffusion.py:102-119) around this U-Net, with
    injected noise (noise[0] = x_T, noise[k] = z for t = n-k) and the same
    float64-scalar update expressions.  ``max_steps`` stops early (bounded
    CPU-baseline samples); ``bf16`` = the bf16-operand convs of the HIP
    path's bf16 precision; ``record`` = step counts after which x is kept
    (returns (x, {count: x})).  noise[k] may also be a callable's product:
    anything indexable by k."""
    betas = torch.linspace(1e-4, 0.02, T)
    alphas = 1.0 - betas
    alpha_bar = torch.cumprod(alphas, dim=0)
    n = T if num_steps is None else num_steps
    B = cond.shape[0] if noise is None else noise.shape[1]
    x = noise[0].clone()
    done = 0
    kept = {}
    for t_ in reversed(range(n)):
        if max_steps is not None and done >= max_steps:
            break
        done += 1
        tt = torch.full((B,), t_, dtype=torch.long)
        pred = forward(x, tt, cond, W, cfg, bf16=bf16)
        coef = (1 - alphas[t_]) / (math.sqrt(1 - alpha_bar[t_]) + 1e-8)
        x = (1.0 / math.sqrt(alphas[t_])) * (x - coef * pred)
        if t_ > 0:
            x = x + math.sqrt(betas[t_]) * temperature * noise[n - t_]
        if done in record:
            kept[done] = x.clone()
    return (x, kept) if record else x


def init_weights(cfg: UNetConfig, seed: int = 0, affine: str = "ones") -> Weights:
    """Deterministic init: PyTorch's default uniform(+-1/sqrt(fan_in)) for
    conv/linear, GN weight 1 / bias 0; zero-init (as is usual) is NOT used so
    every path carries signal in the parity tests.

    ``affine="random"``: every GroupNorm gamma = 1 + U(-0.5, 0.5) and beta =
    U(-0.5, 0.5), distinct per channel (a trained model's state), from a
    second generator -- every other tensor is the same as with "ones".  With
    gamma = 1 / beta = 0 a test cannot see which gamma/beta tensor feeds which
    GroupNorm, nor the channel order of a concatenated input's gamma."""
    if affine not in ("ones", "random"):
        raise ValueError("affine must be 'ones' or 'random'")
    g = torch.Generator().manual_seed(seed)
    ga = torch.Generator().manual_seed(seed + 7919)
    W: Weights = {}
    for name, shape in layer_shapes(cfg):
        if ".norm" in name or name.startswith("norm_out"):
            if affine == "random":
                u = torch.rand(shape, generator=ga) - 0.5
                W[name] = 1.0 + u if name.endswith("weight") else u
            else:
                W[name] = torch.ones(shape) if name.endswith("weight") else torch.zeros(shape)
            continue
        wshape = shape if name.endswith("weight") else None
        if name.endswith("weight"):
            fan_in = int(torch.tensor(shape[1:]).prod())
        else:
            fan_in = int(torch.tensor(dict(layer_shapes(cfg))[name[:-4] + "weight"][1:]).prod())
        bound = 1.0 / math.sqrt(fan_in)
        W[name] = (torch.rand(shape, generator=g) * 2 - 1) * bound
        del wshape
    return W
