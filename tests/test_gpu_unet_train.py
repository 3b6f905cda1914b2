"""U-Net train step on the GPU (ertdiff.unet_train_step: HIP forward with saved
activations, hand-written backward, multi-tensor Adam) against torch autograd
on the specification oracle/unet_torch.forward (CPU float64).  PARITY UNPINNED vs
the reference (it has no U-Net); the call surface is the reference train step
(ERT_Conditional_Diffusion.py:309-320).

Tolerances (rel-L2 per tensor): loss 1e-5, every parameter gradient 1e-4, and
one Adam step 1e-6 against torch.optim.Adam on our own gradients (the update
kernel).  Against torch.optim.Adam on the float64 oracle gradients the
parameter delta is held to ADAM_TOL = 3e-3: Adam's first step is
-lr g / (|g| + 1e-8), so an element whose gradient is within rounding of zero
moves by up to +-lr whichever side of zero its fp32 value lands -- a 1e-5
gradient error shows up as a 1e-3 delta error on those few elements (the
1-D model's train test carries the same 1e-3 budget, test_gpu_train.py)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import ertdiff
from ertdiff.unet_train import unet_train_step
from oracle import ref_numpy as RN
from oracle import unet_torch as U
from synth import synth_normal, synth_timesteps, synth_uniform
from conftest import record_error

pytestmark = pytest.mark.gpu
GRAD_TOL = 1e-4
ADAM_TOL = 3e-3


def _rel(a, b):
    return RN.rel_l2(a.detach().double().cpu().numpy(), b.detach().double().cpu().numpy())


@pytest.mark.parametrize("name,L,seed", [("U1", 257, 0), ("U2", 1001, 1), ("U3", 129, 2)])
def test_unet_train_step_vs_autograd(name, L, seed, cuda_dev):
    B, T, lr = 2, 1000, 1e-3
    cfg = U.CONFIGS[name]
    m = ertdiff.ConditionalUNet.from_config(name, seed=seed).to(cuda_dev)
    W0 = {k: p.detach().cpu().clone() for k, p in m.named_parameters()}
    x0 = torch.from_numpy(synth_normal((B, cfg.param_dim), 500 + seed)).to(cuda_dev)
    cond = torch.from_numpy(synth_uniform((B, 14, L), 501 + seed)).to(cuda_dev)
    t = torch.from_numpy(synth_timesteps(B, T, 502 + seed)).to(cuda_dev)
    noise = torch.from_numpy(synth_normal((B, cfg.param_dim), 503 + seed)).to(cuda_dev)
    _, _, ab = ertdiff.get_diffusion_schedule(T, device=cuda_dev)
    opt = torch.optim.Adam(m.parameters(), lr=lr)
    loss = unet_train_step(m, opt, x0, cond, T, ab, t=t, noise=noise)

    # oracle: autograd through the spec forward on the same noised input
    xn = ertdiff.q_sample(x0, t, noise, ab).cpu().double()
    W = {k: v.double().requires_grad_(True) for k, v in W0.items()}
    eps = U.forward(xn, t.cpu(), cond.cpu().double(), W, cfg)
    ref = F.mse_loss(eps, noise.cpu().double())
    ref.backward()
    assert abs(loss - ref.item()) <= 1e-5 * abs(ref.item()), (loss, ref.item())
    # rel-L2 per tensor, the denominator floored at 1e-3 x the RMS gradient
    # norm: with one channel per GroupNorm group (U1: 32 channels, 32 groups)
    # conv1.bias / emb.* of a ResBlock have exactly zero true gradient (GN2
    # removes a per-channel constant), and both sides hold only rounding noise
    norms = [float(W[k].grad.double().norm()) for k in W]
    floor = 1e-3 * float(np.sqrt(np.mean(np.square(norms))))
    worst = 0.0
    for (k, p), nr in zip(m.named_parameters(), norms):
        e = float((p.grad.detach().double().cpu() - W[k].grad.double()).norm()) / max(nr, floor)
        worst = max(worst, e)
        assert e < GRAD_TOL, (k, e, nr)
    record_error(f"unet_train_grads_{name}", worst)
    # one Adam step: vs torch Adam on the oracle grads, and on our grads
    oref = torch.optim.Adam(list(W.values()), lr=lr)
    oref.step()
    mine = {k: (p.detach().cpu().double() - W0[k].double()) for k, p in m.named_parameters()}
    # (tensors with no true gradient -- norm below the floor -- are excluded:
    # Adam's first step maps their rounding noise to +-lr; the check on our own
    # gradients below covers them)
    errs = {k: _rel(mine[k], w.detach() - W0[k].double()) for (k, w), nr in zip(W.items(), norms)
            if nr >= floor}
    worst_k = max(errs, key=errs.get)
    record_error(f"unet_train_adam_{name}", errs[worst_k])
    assert errs[worst_k] < ADAM_TOL, (worst_k, errs[worst_k], sorted(errs.values())[-5:])
    P2 = [torch.nn.Parameter(W0[k].to(cuda_dev)) for k in W0]
    for p2, (k, p) in zip(P2, m.named_parameters()):
        p2.grad = p.grad.clone()
    o2 = torch.optim.Adam(P2, lr=lr)
    o2.step()
    for p2, (k, p) in zip(P2, m.named_parameters()):
        assert _rel(p, p2) < 1e-6, k
    assert float(opt.state_dict()["state"][0]["step"]) == 1.0


def test_unet_train_step_deterministic_and_learns(cuda_dev):
    B, L, T = 4, 257, 1000
    cfg = U.CONFIGS["U1"]
    x0 = torch.from_numpy(synth_normal((B, cfg.param_dim), 510)).to(cuda_dev)
    cond = torch.from_numpy(synth_uniform((B, 14, L), 511)).to(cuda_dev)
    _, _, ab = ertdiff.get_diffusion_schedule(T, device=cuda_dev)
    runs = []
    for _ in range(2):
        m = ertdiff.ConditionalUNet.from_config("U1", seed=7).to(cuda_dev)
        opt = torch.optim.Adam(m.parameters(), lr=1e-3)
        g = torch.Generator(device=cuda_dev).manual_seed(3)
        t = torch.randint(0, T, (B,), device=cuda_dev, generator=g)
        n = torch.randn(B, cfg.param_dim, device=cuda_dev, generator=g)
        losses = [unet_train_step(m, opt, x0, cond, T, ab, t=t, noise=n) for _ in range(6)]
        runs.append((losses, [p.detach().clone() for p in m.parameters()]))
    assert runs[0][0] == runs[1][0]
    assert all(torch.equal(a, b) for a, b in zip(runs[0][1], runs[1][1]))
    # same batch repeated: the loss goes down
    assert runs[0][0][-1] < runs[0][0][0], runs[0][0]
    # the sampler sees the updated weights (packed cache invalidated)
    m = ertdiff.ConditionalUNet.from_config("U1", seed=7).to(cuda_dev)
    for p, q in zip(m.parameters(), runs[0][1]):
        p.data.copy_(q)
    tt = torch.full((B,), 10, device=cuda_dev, dtype=torch.long)
    a = m(x0, tt, cond)
    with torch.no_grad():
        ref = U.forward(x0.cpu(), tt.cpu(), cond.cpu(),
                        {k: v.detach().cpu() for k, v in m.named_parameters()}, cfg)
    assert _rel(a, ref) < 1e-5


def test_unet_train_rejects_bf16(cuda_dev):
    m = ertdiff.ConditionalUNet.from_config("U1", seed=0, precision="bf16").to(cuda_dev)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    _, _, ab = ertdiff.get_diffusion_schedule(1000, device=cuda_dev)
    x0 = torch.zeros(2, m.param_dim, device=cuda_dev)
    cond = torch.zeros(2, 14, 33, device=cuda_dev)
    with pytest.raises(RuntimeError, match="fp32"):
        unet_train_step(m, opt, x0, cond, 1000, ab)


@pytest.mark.parametrize("Ca,Cb,Cout,H,ks,mode,B", [
    (64, 0, 64, 64, 3, 0, 3),      # ResBlock conv, 64x64
    (128, 64, 64, 32, 3, 0, 2),    # concat input, Cout < Cin
    (256, 0, 256, 16, 3, 0, 2),
    (1, 0, 32, 32, 3, 0, 2),       # conv_in: Cin = 1 (masked ci tile)
    (32, 0, 1, 32, 3, 0, 2),       # conv_out: Cout = 1 (masked co tile)
    (48, 0, 40, 128, 3, 0, 1),     # ragged channel tiles, 128x128 rows
    (64, 0, 64, 64, 3, 1, 2),      # Downsample (stride 2): 64 -> 32
    (128, 0, 128, 32, 3, 1, 2),    # 32 -> 16
    (128, 0, 128, 16, 3, 2, 2),    # Upsample 16 -> 32
    (64, 0, 64, 64, 3, 2, 1),      # Upsample 64 -> 128
    (96, 32, 64, 32, 1, 0, 2),     # 1x1 skip on a concat
    (256, 0, 768, 16, 1, 0, 2),    # attention qkv
])
def test_conv_wgrad_vs_autograd(Ca, Cb, Cout, H, ks, mode, B, cuda_dev):
    from ertdiff import _lib
    g = torch.Generator().manual_seed(Ca * 7 + Cout + H + mode)
    Cin = Ca + Cb
    x = torch.randn(B, Cin, H, H, generator=g)
    Ho = H // 2 if mode == 1 else (2 * H if mode == 2 else H)
    dy = torch.randn(B, Cout, Ho, Ho, generator=g)
    xin = F.interpolate(x.double(), scale_factor=2, mode="nearest") if mode == 2 else x.double()
    ref = torch.nn.grad.conv2d_weight(xin, (Cout, Cin, ks, ks), dy.double(),
                                      stride=2 if mode == 1 else 1, padding=ks // 2)
    lib = _lib.lib()
    n = lib.ertd_conv_wgrad_ws_bytes(Cin, Cout, B, H, ks, mode)
    assert n > 0
    ws = torch.empty(n, dtype=torch.uint8, device=cuda_dev)
    xa = x[:, :Ca].contiguous().to(cuda_dev)
    xb = x[:, Ca:].contiguous().to(cuda_dev) if Cb else None
    dyd = dy.to(cuda_dev)
    out = torch.full((Cout, Cin, ks, ks), 0.5, device=cuda_dev)
    for acc in (0, 1):
        rc = lib.ertd_conv_wgrad(dyd.data_ptr(), xa.data_ptr(), Ca,
                                 None if xb is None else xb.data_ptr(), Cb, B, H, Cout, ks, mode,
                                 out.data_ptr(), acc, ws.data_ptr(), n, _lib.stream_of(cuda_dev))
        assert rc == 0
    err = _rel(out, 2 * ref)                    # written, then accumulated once more
    record_error(f"conv_wgrad_{Cin}_{Cout}_{H}_k{ks}_m{mode}", err)
    assert err < 1e-5, err


def test_conv_wgrad_rejects_bad_geometry(cuda_dev):
    from ertdiff import _lib
    lib = _lib.lib()
    assert lib.ertd_conv_wgrad_ws_bytes(64, 64, 2, 8, 3, 0) == 0       # 8x8 rows: outside
    assert lib.ertd_conv_wgrad_ws_bytes(64, 64, 2, 48, 3, 0) == 0      # not a power of two
    assert lib.ertd_conv_wgrad_ws_bytes(64, 64, 2, 32, 1, 1) == 0      # 1x1 stride 2
    assert lib.ertd_conv_wgrad(None, None, 1, None, 0, 1, 16, 1, 3, 0, None, 0, None, 0, None) != 0
