"""Diagnostic: elements where the fused GN+SiLU bf16 image differs from torch by more than 1 ulp."""
import sys

sys.path.insert(0, "ert-conditional-diffusion-model_amd")
sys.path.insert(0, ".")
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from ertdiff.unet import group_norm_act_bf16  # noqa: E402

dev = torch.device("cuda", 0)
for (Ca, Cb, H) in [(128, 64, 32), (64, 0, 64), (256, 128, 16)]:
    g = torch.Generator().manual_seed(22)
    B, G = 3, 32
    x = torch.randn((B, Ca, H, H), generator=g) * 2 + 0.5
    x2 = torch.randn((B, Cb, H, H), generator=g) if Cb else None
    gamma, beta = torch.randn(Ca + Cb, generator=g) + 1, torch.randn(Ca + Cb, generator=g)
    ss, img = group_norm_act_bf16(x.to(dev), G, gamma.to(dev), beta.to(dev),
                                  x2=None if x2 is None else x2.to(dev))
    ss, img = ss.cpu(), img.cpu()
    xin = x if x2 is None else torch.cat([x, x2], 1)
    y = (xin.double() * ss[..., 0][:, :, None, None].double()
         + ss[..., 1][:, :, None, None].double()).float()
    y = F.silu(y)
    C = Ca + Cb
    ref = y.to(torch.bfloat16).view(torch.int16).reshape(B, C // 16, 16, H, H)
    ref = ref.permute(0, 1, 3, 4, 2).contiguous()
    gf = img.view(torch.bfloat16).float()
    rf = ref.view(torch.bfloat16).float()
    d = (gf - rf).abs()
    bad = d > (rf.abs() * 2 ** -7).clamp_min(1e-6)
    print(Ca, Cb, H, "eq", (img == ref).float().mean().item(), "nbad", int(bad.sum()))
    for i in bad.nonzero()[:10].tolist():
        b, blk, yy, xx, cc = i
        print(i, "ch", blk * 16 + cc, "got", gf[tuple(i)].item(), "ref", rf[tuple(i)].item(),
              "y", y[b, blk * 16 + cc, yy, xx].item())
