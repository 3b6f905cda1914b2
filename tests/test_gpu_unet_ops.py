"""The U-Net's operators one by one (SURVEY.md 8a' operator rows) against
torch on the CPU with identical inputs: 3x3 conv (stride 1 / stride-2
Downsample / nearest-x2 Upsample), 1x1 conv, the GroupNorm(+SiLU) prologue,
skip concatenation, bias/embedding/residual epilogue, GroupNorm statistics,
single-head attention.  fp32: <= 1e-5 rel-L2.  bf16 operands: against torch
with the same bf16 rounding of the activated input and the weights, fp32
accumulation: <= 1e-4 rel-L2 (products are exact; only the summation order and
the ulp of the fused SiLU differ).  Split-bf16 operands ("bf16x3": x = hi + lo,
three bf16 MFMAs per product): against the fp32 torch conv, <= 3e-5 (the
dropped lo*lo term and the lo rounding are <= ~2^-17 relative per product)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from ertdiff.unet import attention, conv2d, group_norm_act_bf16, group_norm_stats
from oracle import ref_numpy as RN
from conftest import record_error

pytestmark = pytest.mark.gpu


def _rand(shape, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(shape, generator=g) * scale).float()


def _ref_conv(x, w, b, mode, act, gn, bf16):
    if act != "none":
        x = x * gn[..., 0][:, :, None, None] + gn[..., 1][:, :, None, None]
        if act == "gn_silu":
            x = F.silu(x)
    if bf16:
        x, w = x.bfloat16().float(), w.bfloat16().float()
    ks = w.shape[-1]
    if mode == "up":
        x = F.interpolate(x, scale_factor=2, mode="nearest")
    return F.conv2d(x, w, b, stride=2 if mode == "down" else 1, padding=ks // 2)


CASES = [  # (Ca, Cb, Cout, H, ks, mode, act)
    (64, 0, 64, 64, 3, "same", "gn_silu"),
    (128, 64, 128, 32, 3, "same", "gn_silu"),    # skip concatenation read in place
    (256, 256, 256, 16, 3, "same", "gn_silu"),
    (64, 0, 64, 64, 3, "down", "none"),
    (128, 0, 128, 32, 3, "down", "none"),
    (128, 0, 128, 32, 3, "up", "none"),
    (256, 0, 256, 16, 3, "up", "none"),
    (64, 0, 64, 64, 3, "up", "none"),            # 64 -> 128 (U5's last Upsample), 64-cout tiles
    (20, 0, 40, 16, 3, "up", "none"),            # partial 8-channel chunk and cout tile
    (20, 12, 40, 32, 3, "up", "none"),           # concatenated input through the sub-pixel path
    (192, 0, 64, 64, 1, "same", "none"),
    (384, 128, 256, 16, 1, "same", "none"),
    (256, 0, 768, 16, 1, "same", "gn"),          # attention qkv
    (1, 0, 64, 64, 3, "same", "none"),           # conv_in (Cin 1)
    (64, 0, 1, 64, 3, "same", "gn_silu"),        # conv_out (Cout 1)
    (32, 24, 1, 32, 3, "same", "gn_silu"),       # Cout 1, concat, partial 16-ch chunk
    (20, 0, 1, 16, 3, "same", "none"),           # Cout 1, whole image in one workgroup
    (128, 0, 1, 128, 3, "same", "gn_silu"),      # Cout 1 at U5's resolution
    # fp32 Winograd F(2x2,3x3) path (Cin, Ca % 8 == 0, Cout % 64 == 0) at every width
    (128, 0, 128, 128, 3, "same", "gn_silu"),    # U5's 128x128 level
    (32, 32, 64, 32, 3, "same", "none"),         # no activation, concatenated input
    (256, 0, 128, 16, 3, "same", "gn"),          # GroupNorm without SiLU
    (384, 128, 256, 16, 3, "same", "gn_silu"),   # U2's widest concat (K = 512)
    # ... and shapes it does not take (direct implicit GEMM)
    (20, 0, 64, 32, 3, "same", "gn_silu"),       # Cin % 8 != 0
    (64, 0, 96, 32, 3, "same", "gn_silu"),       # Cout % 64 != 0
    (60, 4, 64, 16, 3, "same", "gn_silu"),       # concat split inside an 8-channel chunk
]


CONV_TOL = {"fp32": 1e-5, "bf16": 1e-4, "bf16x3": 3e-5}


@pytest.mark.parametrize("precision", ["fp32", "bf16", "bf16x3"])
@pytest.mark.parametrize("Ca,Cb,Cout,H,ks,mode,act", CASES)
def test_conv2d(Ca, Cb, Cout, H, ks, mode, act, precision, cuda_dev):
    B = 2
    x = _rand((B, Ca, H, H), 1)
    x2 = _rand((B, Cb, H, H), 2) if Cb else None
    w = _rand((Cout, Ca + Cb, ks, ks), 3, 1.0 / np.sqrt((Ca + Cb) * ks * ks))
    b = _rand((Cout,), 4, 0.1)
    gn = None
    if act != "none":
        gn = torch.stack([_rand((B, Ca + Cb), 5, 0.3) + 1.0, _rand((B, Ca + Cb), 6, 0.2)], -1)
    out = conv2d(x.to(cuda_dev), w.to(cuda_dev), b.to(cuda_dev), mode=mode, act=act,
                 gn=None if gn is None else gn.to(cuda_dev),
                 x2=None if x2 is None else x2.to(cuda_dev), precision=precision).cpu()
    xin = x if x2 is None else torch.cat([x, x2], 1)
    ref = _ref_conv(xin, w, b, mode, act, gn, precision == "bf16")
    err = RN.rel_l2(out.double().numpy(), ref.double().numpy())
    record_error(f"conv2d_{Ca}_{Cb}_{Cout}_{H}_k{ks}_{mode}_{act}_{precision}", err)
    assert err < CONV_TOL[precision], err


# The exact variants the headline (U2, B = 64) and the train step (B = 32) run:
# (Cin, Cout, H) per Winograd level at B = 32 and 64, with bias, per-sample
# embedding add and residual.  On 256 CUs: at B = 64 every level runs the
# register-weight F(4x4) kernel unsplit (64 co x 16 tile items: 1024 / 256 /
# 256 at 64x64 / 32x32 / 16x16); at B = 32 the 64x64 and 32x32 levels too (512 /
# 256 items), the 16x16 level (128 items) with its K split in two halves.
HEADLINE_CASES = [(64, 64, 64), (128, 128, 32), (384, 128, 32), (256, 256, 16), (512, 256, 16)]


@pytest.mark.parametrize("B", [32, 64])
@pytest.mark.parametrize("Cin,Cout,H", HEADLINE_CASES)
def test_conv2d_headline_variants(Cin, Cout, H, B, cuda_dev):
    seed = Cin + Cout + H + B
    x = _rand((B, Cin, H, H), seed)
    w = _rand((Cout, Cin, 3, 3), seed + 1, 1.0 / np.sqrt(9 * Cin))
    b = _rand((Cout,), seed + 2, 0.1)
    gn = torch.stack([_rand((B, Cin), seed + 3, 0.3) + 1.0, _rand((B, Cin), seed + 4, 0.2)], -1)
    eb, res = _rand((B, Cout), seed + 5), _rand((B, Cout, H, H), seed + 6)
    out = conv2d(x.to(cuda_dev), w.to(cuda_dev), b.to(cuda_dev), act="gn_silu", gn=gn.to(cuda_dev),
                 ebias=eb.to(cuda_dev), res=res.to(cuda_dev)).cpu()
    ref = _ref_conv(x, w, b, "same", "gn_silu", gn, False) + eb[:, :, None, None] + res
    err = RN.rel_l2(out.double().numpy(), ref.double().numpy())
    record_error(f"conv2d_headline_{Cin}_{Cout}_{H}_B{B}", err)
    assert err < 1e-5, err


def _cus(dev):
    return torch.cuda.get_device_properties(dev).multi_processor_count


KSPLIT_CASES = [  # (Ca, Cb, Cout, act, emb, residual): 16x16, B = CUs / 8, always a bias
    (256, 256, 256, "gn_silu", True, True),       # concatenated input, both halves of K on different tensors
    (384, 128, 256, "none", True, True),          # ACT_NONE with a residual
    (256, 0, 256, "gn", False, False),            # GroupNorm without SiLU, bias only
]


@pytest.mark.parametrize("Ca,Cb,Cout,act,eb,resid", KSPLIT_CASES)
def test_conv2d_wino4s_ksplit(Ca, Cb, Cout, act, eb, resid, cuda_dev):
    """The register-weight F(4x4) kernel's K split (unet_conv_wino4s.hip,
    ksp = 2): at 16x16 with B = CUs / 8 its 64 co x 16 tile items fill half
    the CUs, so each item is split into two K halves (half 1's raw sums to the
    K-split buffer, added in place afterwards); B chosen from the device's CU
    count so the split geometry is hit on any part.  Against torch <= 1e-5, and
    against the unsplit dispatch of the same samples (B = CUs / 4: items fill
    the CUs) to rounding (<= 3e-6)."""
    cus = _cus(cuda_dev)
    B, H = cus // 8, 16
    seed = Ca + 3 * Cb + Cout
    x = _rand((B, Ca, H, H), seed)
    x2 = _rand((B, Cb, H, H), seed + 1) if Cb else None
    w = _rand((Cout, Ca + Cb, 3, 3), seed + 2, 1.0 / np.sqrt(9 * (Ca + Cb)))
    b = _rand((Cout,), seed + 3, 0.1)
    gn = None
    if act != "none":
        gn = torch.stack([_rand((B, Ca + Cb), seed + 4, 0.3) + 1.0, _rand((B, Ca + Cb), seed + 5, 0.2)], -1)
    e = _rand((B, Cout), seed + 6) if eb else None
    res = _rand((B, Cout, H, H), seed + 7) if resid else None
    d = lambda v: None if v is None else v.to(cuda_dev)
    out = conv2d(d(x), d(w), d(b), act=act, gn=d(gn), x2=d(x2), ebias=d(e), res=d(res)).cpu()
    xin = x if x2 is None else torch.cat([x, x2], 1)
    ref = _ref_conv(xin, w, b, "same", act, gn, False)
    if eb:
        ref = ref + e[:, :, None, None]
    if resid:
        ref = ref + res
    err = RN.rel_l2(out.double().numpy(), ref.double().numpy())
    record_error(f"conv2d_wino4s_ksplit_{Ca}_{Cb}_{Cout}_{act}_B{B}", err)
    assert err < 1e-5, err
    # the same samples twice over (B = CUs / 4): unsplit items, another summation order
    cat = lambda v: None if v is None else torch.cat([v, v])
    full = conv2d(d(cat(x)), d(w), d(b), act=act, gn=d(cat(gn)), x2=d(cat(x2)),
                  ebias=d(cat(e)), res=d(cat(res))).cpu()
    assert not torch.equal(full[:B], out)
    # (each side carries F(4x4)'s ~1e-6 rounding: measured 1.0e-6 apart)
    assert RN.rel_l2(full[:B].double().numpy(), out.double().numpy()) < 3e-6


def test_conv_input_grad_wino4s_ksplit_accumulate(cuda_dev):
    """The train step's 16x16 input-gradient conv at B = CUs / 8 through the
    register-weight F(4x4) kernel with its K split, accumulating into the
    existing gradient (accumulate = 1: the residual operand aliases the
    output) -- against float64 autograd <= 1e-5."""
    from ertdiff import _lib
    cus = _cus(cuda_dev)
    B, Cin, Cout, H = cus // 8, 256, 256, 16
    g = torch.Generator().manual_seed(91)
    w = torch.randn(Cout, Cin, 3, 3, generator=g) / (9 * Cin) ** 0.5
    dy = torch.randn(B, Cout, H, H, generator=g)
    prev = torch.randn(B, Cin, H, H, generator=g)
    ref = torch.nn.grad.conv2d_input((B, Cin, H, H), w.double(), dy.double(), padding=1) + prev.double()
    lib = _lib.lib()
    n = lib.ertd_conv_input_grad_ws_bytes(Cin, Cout, B, H, 3, 0)
    ws = torch.empty(n, dtype=torch.uint8, device=cuda_dev)
    dx = prev.to(cuda_dev)
    assert lib.ertd_conv_input_grad(dy.to(cuda_dev).data_ptr(), B, H, w.to(cuda_dev).data_ptr(), Cout, Cin, 3, 0,
                                    dx.data_ptr(), 1, ws.data_ptr(), n, _lib.stream_of(cuda_dev)) == 0
    err = RN.rel_l2(dx.cpu().double().numpy(), ref.numpy())
    record_error(f"conv_input_grad_wino4s_ksplit_B{B}", err)
    assert err < 1e-5, err


# every 1x1 skip shape of U2 (Ca, Cb, Cout, H): the batched-GEMM kernel
# (unet_skip_gemm.hip) -- 128 x 128, 128 x 64 and 64 x 256 tiles, concatenated
# inputs split inside a 32-channel chunk or on its boundary
SKIP_SHAPES = [(64, 0, 128, 32, 4), (128, 0, 256, 16, 4), (256, 256, 256, 16, 64), (256, 128, 256, 16, 4),
               (256, 128, 128, 32, 64), (128, 128, 128, 32, 4), (128, 64, 128, 32, 4), (128, 64, 64, 64, 4),
               (64, 64, 64, 64, 8), (96, 32, 128, 32, 3)]


@pytest.mark.parametrize("Ca,Cb,Cout,H,B", SKIP_SHAPES)
def test_conv2d_skip_gemm_shapes(Ca, Cb, Cout, H, B, cuda_dev):
    x = _rand((B, Ca, H, H), 70 + Ca)
    x2 = _rand((B, Cb, H, H), 71 + Cb) if Cb else None
    w, b = _rand((Cout, Ca + Cb, 1, 1), 72, 1.0 / np.sqrt(Ca + Cb)), _rand((Cout,), 73, 0.1)
    out = conv2d(x.to(cuda_dev), w.to(cuda_dev), b.to(cuda_dev),
                 x2=None if x2 is None else x2.to(cuda_dev)).cpu()
    xin = x if x2 is None else torch.cat([x, x2], 1)
    ref = F.conv2d(xin.double(), w.double(), b.double())
    err = RN.rel_l2(out.double().numpy(), ref.numpy())
    record_error(f"conv2d_skip_gemm_{Ca}+{Cb}_{Cout}_{H}_B{B}", err)
    assert err < 1e-5, err


@pytest.mark.parametrize("B", [2, 64])
def test_conv2d_1x1_skip_kernel(B, cuda_dev):
    """The 1x1 skip conv kernel (unet_conv1x1.hip: LDS-DMA'd input and gathered
    weight slices, 256-px items at B=2, 512-px items at the headline's B=64) on
    U2's u0r0.skip shape: 128 + 64 (concatenated) -> 64 at 64x64, with bias."""
    Ca, Cb, Cout, H = 128, 64, 64, 64
    x, x2 = _rand((B, Ca, H, H), 60), _rand((B, Cb, H, H), 61)
    w, b = _rand((Cout, Ca + Cb, 1, 1), 62, 1.0 / np.sqrt(Ca + Cb)), _rand((Cout,), 63, 0.1)
    out = conv2d(x.to(cuda_dev), w.to(cuda_dev), b.to(cuda_dev), x2=x2.to(cuda_dev)).cpu()
    ref = F.conv2d(torch.cat([x, x2], 1), w, b)
    err = RN.rel_l2(out.double().numpy(), ref.double().numpy())
    record_error(f"conv2d_1x1_skip_B{B}", err)
    assert err < 1e-5, err


def test_conv2d_wino4_16x16_two_sample_blocks(cuda_dev):
    """Winograd F(4x4,3x3) at 16x16 (taken only when its tile items fill the
    CUs without a K split: B=128, Cout=256 -> 256 items): a 32-tile block holds
    two samples (per-lane sample offset, GroupNorm row and epilogue base), with
    the embedding and residual epilogue."""
    B, C, H = 128, 256, 16
    x, w, b = _rand((B, C, H, H), 40), _rand((C, C, 3, 3), 41, 1.0 / np.sqrt(9 * C)), _rand((C,), 42, 0.1)
    gn = torch.stack([_rand((B, C), 43, 0.3) + 1.0, _rand((B, C), 44, 0.2)], -1)
    eb, res = _rand((B, C), 45), _rand((B, C, H, H), 46)
    out = conv2d(x.to(cuda_dev), w.to(cuda_dev), b.to(cuda_dev), act="gn_silu", gn=gn.to(cuda_dev),
                 ebias=eb.to(cuda_dev), res=res.to(cuda_dev)).cpu()
    ref = _ref_conv(x, w, b, "same", "gn_silu", gn, False) + eb[:, :, None, None] + res
    err = RN.rel_l2(out.double().numpy(), ref.double().numpy())
    record_error("conv2d_wino4_16x16_B128", err)
    assert err < 1e-5, err


def test_conv2d_up_epilogue(cuda_dev):
    """Sub-pixel Upsample conv (fp32: 4 parity classes of 2x2 taps) with the
    per-sample channel add and residual scattered to the right parity."""
    B, C, H = 2, 64, 16
    x, w, b = _rand((B, C, H, H), 30), _rand((C, C, 3, 3), 31, 0.04), _rand((C,), 32)
    eb, res = _rand((B, C), 33), _rand((B, C, 2 * H, 2 * H), 34)
    out = conv2d(x.to(cuda_dev), w.to(cuda_dev), b.to(cuda_dev), mode="up",
                 ebias=eb.to(cuda_dev), res=res.to(cuda_dev)).cpu()
    ref = F.conv2d(F.interpolate(x, scale_factor=2, mode="nearest"), w, b, padding=1)
    ref = ref + eb[:, :, None, None] + res
    assert RN.rel_l2(out.double().numpy(), ref.double().numpy()) < 1e-5


def test_conv2d_epilogue(cuda_dev):
    B, C, H = 2, 128, 32
    x, w, b = _rand((B, C, H, H), 7), _rand((C, C, 3, 3), 8, 0.03), _rand((C,), 9)
    eb, res = _rand((B, C), 10), _rand((B, C, H, H), 11)
    out = conv2d(x.to(cuda_dev), w.to(cuda_dev), b.to(cuda_dev), ebias=eb.to(cuda_dev),
                 res=res.to(cuda_dev)).cpu()
    ref = F.conv2d(x, w, b, padding=1) + eb[:, :, None, None] + res
    assert RN.rel_l2(out.double().numpy(), ref.double().numpy()) < 1e-5


def test_conv2d_out_epilogue(cuda_dev):
    """Cout = 1 path (csrc/unet_conv_out.hip) with the embedding and residual adds."""
    B, C, H = 3, 48, 32
    x, w, b = _rand((B, C, H, H), 17), _rand((1, C, 3, 3), 18, 0.05), _rand((1,), 19)
    eb, res = _rand((B, 1), 20), _rand((B, 1, H, H), 21)
    out = conv2d(x.to(cuda_dev), w.to(cuda_dev), b.to(cuda_dev), ebias=eb.to(cuda_dev),
                 res=res.to(cuda_dev)).cpu()
    ref = F.conv2d(x, w, b, padding=1) + eb[:, :, None, None] + res
    assert RN.rel_l2(out.double().numpy(), ref.double().numpy()) < 1e-5


@pytest.mark.parametrize("Ca,Cb,H,G", [(64, 0, 64, 32), (256, 128, 16, 32), (128, 64, 32, 32),
                                        (512, 0, 16, 1), (256, 256, 16, 1), (384, 0, 16, 2)])
def test_group_norm_stats(Ca, Cb, H, G, cuda_dev):
    """G = 1 / 2: groups wider than the 256-thread workgroup (every channel of
    the group still gets its {scale, shift})."""
    B = 3
    x = _rand((B, Ca, H, H), 12, 2.0) + 0.5
    x2 = _rand((B, Cb, H, H), 13) if Cb else None
    gamma, beta = _rand((Ca + Cb,), 14) + 1, _rand((Ca + Cb,), 15)
    ss = group_norm_stats(x.to(cuda_dev), G, gamma.to(cuda_dev), beta.to(cuda_dev),
                          x2=None if x2 is None else x2.to(cuda_dev)).cpu()
    xin = x if x2 is None else torch.cat([x, x2], 1)
    y = xin * ss[..., 0][:, :, None, None] + ss[..., 1][:, :, None, None]
    ref = F.group_norm(xin, G, gamma, beta, eps=1e-5)
    assert RN.rel_l2(y.double().numpy(), ref.double().numpy()) < 1e-5


@pytest.mark.parametrize("Ca,Cb,H,G,npa,npb", [(64, 0, 64, 32, 16, 0), (128, 64, 32, 32, 4, 4),
                                               (192, 64, 64, 32, 16, 16), (256, 256, 16, 32, 1, 1),
                                               (512, 0, 16, 1, 1, 0), (100, 92, 32, 32, 4, 4)])
def test_group_norm_from_partials(Ca, Cb, H, G, npa, npb, cuda_dev):
    """GroupNorm statistics from per-part {sum, M2} partials (what the fp32
    Winograd convs emit from their epilogue): finalize == ertd_group_norm_stats
    within 1e-6, and the normalized tensor == torch's group_norm within 1e-5,
    for groups straddling the skip concatenation and parts of different sizes."""
    from ertdiff import _lib
    lib = _lib.lib()
    B = 3
    x = (_rand((B, Ca, H, H), 51, 2.0) + 0.5).to(cuda_dev)
    x2 = (_rand((B, Cb, H, H), 52) - 0.3).to(cuda_dev) if Cb else None
    gamma, beta = (_rand((Ca + Cb,), 53) + 1).to(cuda_dev), _rand((Ca + Cb,), 54).to(cuda_dev)
    s = _lib.stream_of(cuda_dev)
    pa = torch.empty(B, Ca, npa, 2, device=cuda_dev)
    assert lib.ertd_group_norm_partials(x.data_ptr(), Ca, B, H * H, npa, pa.data_ptr(), s) == 0
    pb = None
    if Cb:
        pb = torch.empty(B, Cb, npb, 2, device=cuda_dev)
        assert lib.ertd_group_norm_partials(x2.data_ptr(), Cb, B, H * H, npb, pb.data_ptr(), s) == 0
    ss = torch.empty(B, Ca + Cb, 2, device=cuda_dev)
    mr = torch.empty(B, G, 2, device=cuda_dev)
    assert lib.ertd_group_norm_finalize(pa.data_ptr(), npa, Ca, None if pb is None else pb.data_ptr(), npb,
                                        Cb, B, H * H, G, gamma.data_ptr(), beta.data_ptr(), ss.data_ptr(),
                                        mr.data_ptr(), s) == 0
    ref_ss = group_norm_stats(x, G, gamma, beta, x2=x2)
    assert torch.allclose(ss, ref_ss, rtol=1e-6, atol=1e-6)
    xin = (x if x2 is None else torch.cat([x, x2], 1)).cpu()
    y = xin * ss.cpu()[..., 0][:, :, None, None] + ss.cpu()[..., 1][:, :, None, None]
    ref = F.group_norm(xin, G, gamma.cpu(), beta.cpu(), eps=1e-5)
    err = RN.rel_l2(y.double().numpy(), ref.double().numpy())
    record_error(f"gn_from_partials_{Ca}_{Cb}_{H}_{G}", err)
    assert err < 1e-5, err


@pytest.mark.parametrize("Ca,Cb,H,silu", [(64, 0, 64, True), (128, 64, 32, True),
                                          (256, 128, 16, True), (192, 0, 32, False),
                                          (512, 0, 16, True), (64, 0, 16, True)])
def test_group_norm_act_bf16(Ca, Cb, H, silu, cuda_dev):
    """Fused statistics + GN(+SiLU) + bf16 image (the bf16 3x3 convs' prologue):
    {scale, shift} within 1e-6 of group_norm_stats (same float64 sum/sumsq
    form, another summation order); image = RNE bf16 of the fp32 activation:
    >= 99 % of elements bit-equal to torch's, every element within 1 bf16 ulp
    (the kernel's fast exp/rcp SiLU), pixel records in [B][C/16][H][W][16]."""
    B, G = 3, 32
    x = _rand((B, Ca, H, H), 22, 2.0) + 0.5
    x2 = _rand((B, Cb, H, H), 23) if Cb else None
    gamma, beta = _rand((Ca + Cb,), 24) + 1, _rand((Ca + Cb,), 25)
    dx2 = None if x2 is None else x2.to(cuda_dev)
    ss, img = group_norm_act_bf16(x.to(cuda_dev), G, gamma.to(cuda_dev), beta.to(cuda_dev),
                                  x2=dx2, silu=silu)
    ref_ss = group_norm_stats(x.to(cuda_dev), G, gamma.to(cuda_dev), beta.to(cuda_dev), x2=dx2)
    ss, ref_ss, img = ss.cpu(), ref_ss.cpu(), img.cpu()
    assert torch.allclose(ss, ref_ss, rtol=1e-6, atol=1e-6)
    xin = x if x2 is None else torch.cat([x, x2], 1)
    # the kernel applies x*scale+shift as ONE fma: the reference rounds once too
    # (float64 product of two floats is exact), else cancellation near zero
    # differs in relative terms
    y = (xin.double() * ss[..., 0][:, :, None, None].double()
         + ss[..., 1][:, :, None, None].double()).float()
    if silu:
        y = F.silu(y)
    C = Ca + Cb
    ref = y.to(torch.bfloat16).view(torch.int16).reshape(B, C // 16, 16, H, H).permute(0, 1, 3, 4, 2)
    got_f = img.view(torch.bfloat16).float()
    ref_f = ref.contiguous().view(torch.bfloat16).float()
    eq = (img == ref.contiguous()).float().mean().item()
    assert eq >= 0.99, f"only {eq:.4f} of the image bit-equal"
    ulp = (ref_f.abs() * 2.0 ** -7).clamp_min(1e-6)
    assert bool(((got_f - ref_f).abs() <= ulp).all())


def test_group_norm_act_bf16_rejects_shapes(cuda_dev):
    x = torch.zeros(1, 24, 16, 16, device=cuda_dev)   # C % 16 != 0
    g = torch.ones(24, device=cuda_dev)
    with pytest.raises(RuntimeError):
        group_norm_act_bf16(x, 8, g, g)


def test_attention(cuda_dev):
    B, C, N = 2, 256, 256
    qkv = _rand((B, 3 * C, N), 16, 0.5)
    out = attention(qkv.to(cuda_dev)).cpu()
    q, k, v = qkv[:, :C], qkv[:, C:2 * C], qkv[:, 2 * C:]
    a = torch.softmax(torch.einsum("bci,bcj->bij", q, k) / 16.0, dim=-1)
    ref = torch.einsum("bij,bcj->bci", a, v)
    assert RN.rel_l2(out.double().numpy(), ref.double().numpy()) < 1e-5


@pytest.mark.parametrize("Ca,Cb,H,act,up", [(128, 64, 16, 1, 0), (64, 0, 32, 2, 0), (48, 16, 16, 0, 1)])
def test_act_bf16_image(Ca, Cb, H, act, up, cuda_dev):
    """ertd_act_bf16 (the bf16 path's standalone image transform): RNE bf16 of
    act(x*scale+shift) (or of the nearest-x2 upsample) in [B][C/16][Ho][Ho][16]
    records; every element within 1 bf16 ulp of torch's, >= 99 % bit-equal."""
    from ertdiff import _lib
    B, C = 2, Ca + Cb
    x = _rand((B, Ca, H, H), 31, 2.0)
    x2 = _rand((B, Cb, H, H), 32) if Cb else None
    ss = torch.stack([_rand((B, C), 33) + 1, _rand((B, C), 34)], -1)
    Ho = 2 * H if up else H
    img = torch.empty(B, C // 16, Ho, Ho, 16, dtype=torch.int16, device=cuda_dev)
    dx, dss = x.to(cuda_dev), ss.to(cuda_dev)
    dx2 = None if x2 is None else x2.to(cuda_dev)
    rc = _lib.lib().ertd_act_bf16(dx.data_ptr(), Ca, None if dx2 is None else dx2.data_ptr(), Cb, B, H,
                                  dss.data_ptr() if act else None, act, up, img.data_ptr(),
                                  _lib.stream_of(cuda_dev))
    assert rc == 0
    xin = x if x2 is None else torch.cat([x, x2], 1)
    if up:
        y = F.interpolate(xin, scale_factor=2, mode="nearest")
    else:
        y = (xin.double() * ss[..., 0][:, :, None, None].double()
             + ss[..., 1][:, :, None, None].double()).float()
        if act == 1:
            y = F.silu(y)
    ref = y.to(torch.bfloat16).view(torch.int16).reshape(B, C // 16, 16, Ho, Ho).permute(0, 1, 3, 4, 2)
    got = img.cpu()
    ref = ref.contiguous()
    assert (got == ref).float().mean().item() >= 0.99
    got_f, ref_f = got.view(torch.bfloat16).float(), ref.view(torch.bfloat16).float()
    ulp = (ref_f.abs() * 2.0 ** -7).clamp_min(1e-6)
    assert bool(((got_f - ref_f).abs() <= ulp).all())


def test_conv2d_run_reuses_packing(cuda_dev):
    """ertd_conv2d_run (the conv kernel alone on a packing an earlier
    ertd_conv2d left in the workspace) == ertd_conv2d bit for bit."""
    from ertdiff import _lib
    lib = _lib.lib()
    B, C, H = 4, 64, 32
    x = _rand((B, C, H, H), 61).to(cuda_dev)
    w = _rand((C, C, 3, 3), 62, 1.0 / np.sqrt(9 * C)).to(cuda_dev)
    b = _rand((C,), 63, 0.1).to(cuda_dev)
    gn = torch.stack([_rand((B, C), 64, 0.3) + 1.0, _rand((B, C), 65, 0.2)], -1).to(cuda_dev)
    y1, y2 = torch.empty(B, C, H, H, device=cuda_dev), torch.empty(B, C, H, H, device=cuda_dev)
    n = lib.ertd_conv2d_workspace_bytes(C, C, 3, 0, B, H, 0)
    ws = torch.empty(n, dtype=torch.uint8, device=cuda_dev)
    s = _lib.stream_of(cuda_dev)
    assert lib.ertd_conv2d(x.data_ptr(), C, None, 0, B, H, w.data_ptr(), b.data_ptr(), C, 3, 0,
                           gn.data_ptr(), 1, None, 0, None, y1.data_ptr(), 0, ws.data_ptr(), n, s) == 0
    assert lib.ertd_conv2d_run(x.data_ptr(), C, None, 0, B, H, b.data_ptr(), C, 3, 0, gn.data_ptr(), 1,
                               None, 0, None, y2.data_ptr(), 0, ws.data_ptr(), n, s) == 0
    torch.cuda.synchronize()
    assert torch.equal(y1, y2)
