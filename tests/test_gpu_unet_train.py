"""U-Net train step on the GPU (ertdiff.unet_train_step: HIP forward with saved
activations, hand-written backward, multi-tensor Adam) against torch autograd
on the specification oracle/unet_torch.forward (CPU float64).  PARITY UNPINNED vs
the reference (it has no U-Net); the call surface is the reference train step
(ERT_Conditional_Diffusion.py:309-320).

Tolerances (rel-L2 per tensor): loss 1e-5, every parameter gradient 1e-4, and
one Adam step 1e-6 against torch.optim.Adam on our own gradients (the update
kernel).  Against torch.optim.Adam on the float64 oracle gradients the
parameter delta is held to ADAM_TOL = 1e-2: Adam's first step is
-lr g / (|g| + 1e-8), so an element whose gradient is within rounding of zero
moves by up to +-lr whichever side of zero its fp32 value lands -- a 1e-5
gradient error shows up as a 1e-3 delta error on those few elements.  Measured
on U1 (the worst): 2.9e-3 with the F(2x2) Winograd convs, 4.7e-3 with F(4x4)
at the same gradient error (2.3e-5 vs 2.2e-5): which near-zero elements flip
is rounding noise, so this gate is a sanity bound; the gradient gate above and
the Adam-on-our-gradients gate are the parity checks."""
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
ADAM_TOL = 1e-2


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
    with torch.no_grad():
        a = m(x0, tt, cond)
    with torch.no_grad():
        ref = U.forward(x0.cpu(), tt.cpu(), cond.cpu(),
                        {k: v.detach().cpu() for k, v in m.named_parameters()}, cfg)
    assert _rel(a, ref) < 1e-5


@pytest.mark.parametrize("name,B,L", [("U1", 4, 257), ("U3", 2, 129)])
def test_unet_train_plan_matches_eager_steps(name, B, L, cuda_dev):
    """UNetTrainPlan (the train step captured once as a graph, Adam eager) ==
    unet_train_step bit for bit over 4 optimizer steps with fresh batches:
    losses, parameters, Adam moments."""
    from ertdiff.unet_train import UNetTrainPlan
    T = 1000
    cfg = U.CONFIGS[name]
    _, _, ab = ertdiff.get_diffusion_schedule(T, device=cuda_dev)
    g = torch.Generator(device=cuda_dev).manual_seed(21)
    data = [(torch.randn(B, cfg.param_dim, device=cuda_dev, generator=g),
             torch.rand(B, 14, L, device=cuda_dev, generator=g),
             torch.randint(0, T, (B,), device=cuda_dev, generator=g),
             torch.randn(B, cfg.param_dim, device=cuda_dev, generator=g)) for _ in range(4)]
    runs = []
    for graph in (False, True):
        m = ertdiff.ConditionalUNet.from_config(name, seed=8).to(cuda_dev)
        opt = torch.optim.Adam(m.parameters(), lr=1e-3)
        plan = UNetTrainPlan(m, opt, B, L, T, ab) if graph else None
        losses = []
        for x0, cond, t, n in data:
            if graph:
                losses.append(plan.step(x0, cond, t=t, noise=n))
            else:
                losses.append(unet_train_step(m, opt, x0, cond, T, ab, t=t, noise=n))
        st = opt.state_dict()["state"]
        runs.append((losses, [p.detach().clone() for p in m.parameters()],
                     [st[i]["exp_avg_sq"].clone() for i in range(len(st))]))
    assert runs[0][0] == runs[1][0], (runs[0][0], runs[1][0])
    assert all(torch.equal(a, b) for a, b in zip(runs[0][1], runs[1][1]))
    assert all(torch.equal(a, b) for a, b in zip(runs[0][2], runs[1][2]))
    with pytest.raises(RuntimeError):
        plan.step(data[0][0][:1], data[0][1][:1])


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
    (64, 0, 64, 64, 3, 0, 32),     # ... at the train step's B = 32 (Winograd F(4x4) wgrad)
    (384, 128, 256, 16, 3, 0, 32), # the widest decoder conv1 at B = 32
    (128, 64, 64, 32, 3, 0, 2),    # concat input, Cout < Cin
    (128, 64, 128, 32, 3, 0, 2),   # Winograd wgrad tile 128 co x 64 ci (Cin % 128 != 0)
    (64, 64, 64, 32, 3, 0, 2),     # ... 64 co x 128 ci
    (256, 0, 256, 16, 3, 0, 2),
    (1, 0, 32, 32, 3, 0, 2),       # conv_in: Cin = 1 (single-channel-side kernel)
    (32, 0, 1, 32, 3, 0, 2),       # conv_out: Cout = 1
    (1, 0, 64, 64, 3, 0, 32),      # conv_in at the train batch
    (1, 0, 64, 16, 3, 0, 3),       # 16x16: 8-row bands
    (1, 0, 80, 32, 3, 0, 2),       # Cout > 64: the implicit GEMM's masked tile
    (48, 0, 40, 128, 3, 0, 1),     # ragged channel tiles, 128x128 rows
    (64, 0, 64, 64, 3, 1, 2),      # Downsample (stride 2): 64 -> 32
    (128, 0, 128, 32, 3, 1, 2),    # 32 -> 16
    (128, 0, 128, 16, 3, 2, 2),    # Upsample 16 -> 32
    (64, 0, 64, 64, 3, 2, 1),      # Upsample 64 -> 128
    (128, 0, 128, 32, 3, 2, 8),    # u1.up 32 -> 64 (Winograd wgrad over the upsampled input)
    (256, 0, 256, 16, 3, 2, 8),    # u2.up 16 -> 32
    (96, 32, 64, 32, 1, 0, 2),     # 1x1 skip on a concat (LDS GEMM; concat split inside a ci tile)
    (256, 0, 768, 16, 1, 0, 2),    # attention qkv
    (128, 64, 64, 64, 1, 0, 32),   # u0 skip 192 -> 64 at the train batch (64 co x 64 ci tiles)
    (384, 128, 256, 16, 1, 0, 32), # u2 skip 512 -> 256 (128 x 128 tiles)
    (64, 0, 128, 32, 1, 0, 3),     # d1 skip 64 -> 128 (128 co x 64 ci tiles)
    (48, 0, 40, 32, 1, 0, 2),      # ragged channels: the implicit-GEMM 1x1 path
    (64, 0, 64, 16, 1, 0, 1),      # K = 256: a single K range
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
                                 None, 0, out.data_ptr(), acc, ws.data_ptr(), n,
                                 _lib.stream_of(cuda_dev))
        assert rc == 0
    err = _rel(out, 2 * ref)                    # written, then accumulated once more
    record_error(f"conv_wgrad_{Cin}_{Cout}_{H}_k{ks}_m{mode}", err)
    assert err < 1e-5, err


@pytest.mark.parametrize("Ca,Cb,Cout,H,mode,B", [
    (64, 0, 64, 64, 0, 32),        # 64x64 ResBlock conv2 at the train batch
    (128, 64, 128, 32, 0, 8),      # concat input
    (128, 0, 128, 32, 2, 8),       # Upsample conv
])
def test_conv_wgrad_fused_bias(Ca, Cb, Cout, H, mode, B, cuda_dev):
    """ertd_conv_wgrad_bias: the same dW bits as ertd_conv_wgrad, plus the bias
    gradient sum(dy) (into two outputs) from the Winograd path's dy transform."""
    from ertdiff import _lib
    g = torch.Generator().manual_seed(Ca + 3 * Cout + H)
    Cin = Ca + Cb
    Ho = 2 * H if mode == 2 else H
    x = torch.randn(B, Cin, H, H, generator=g)
    dy = torch.randn(B, Cout, Ho, Ho, generator=g)
    lib = _lib.lib()
    assert lib.ertd_conv_wgrad_bias_ok(Cin, Cout, B, H, 3, mode) == 1
    n = lib.ertd_conv_wgrad_ws_bytes(Cin, Cout, B, H, 3, mode)
    ws = torch.empty(n, dtype=torch.uint8, device=cuda_dev)
    xa = x[:, :Ca].contiguous().to(cuda_dev)
    xb = x[:, Ca:].contiguous().to(cuda_dev) if Cb else None
    dyd = dy.to(cuda_dev)
    s = _lib.stream_of(cuda_dev)
    dw0, dw1 = (torch.empty(Cout, Cin, 3, 3, device=cuda_dev) for _ in range(2))
    db, db2 = torch.full((Cout,), 7.0, device=cuda_dev), torch.full((Cout,), 7.0, device=cuda_dev)
    assert lib.ertd_conv_wgrad(dyd.data_ptr(), xa.data_ptr(), Ca, None if xb is None else xb.data_ptr(),
                               Cb, B, H, Cout, 3, mode, None, 0, dw0.data_ptr(), 0, ws.data_ptr(), n, s) == 0
    assert lib.ertd_conv_wgrad_bias(dyd.data_ptr(), xa.data_ptr(), Ca,
                                    None if xb is None else xb.data_ptr(), Cb, B, H, Cout, 3, mode, None,
                                    0, dw1.data_ptr(), 0, db.data_ptr(), db2.data_ptr(), ws.data_ptr(), n,
                                    s) == 0
    assert torch.equal(dw0, dw1)
    assert torch.equal(db, db2)
    err = _rel(db, dy.double().sum((0, 2, 3)))
    record_error(f"conv_wgrad_fused_bias_{Cin}_{Cout}_{H}_m{mode}", err)
    assert err < 1e-5, err
    # outside the fused geometry (B * tiles not a multiple of 256) the query says so
    assert lib.ertd_conv_wgrad_bias_ok(64, 64, 1, 16, 3, 0) == 0


@pytest.mark.parametrize("Ca,Cb,Cout,H,ks,act,B", [
    (64, 0, 64, 64, 3, 1, 2),      # conv1 / conv2 / conv_out: GroupNorm + SiLU staged
    (96, 32, 64, 32, 3, 1, 2),     # decoder conv1 on a concat
    (256, 0, 768, 16, 1, 2, 2),    # attention qkv: GroupNorm only
    (64, 0, 1, 64, 3, 1, 32),      # conv_out at the train batch (single-output-channel kernel)
    (32, 0, 1, 128, 3, 1, 2),      # ... 128x128 rows (2-row bands)
])
def test_conv_wgrad_fused_activation(Ca, Cb, Cout, H, ks, act, B, cuda_dev):
    """dL/dW of conv(act(x)) with act(v) = v * scale + shift (+ SiLU) applied by the
    kernel while staging x (the forward never materializes act(x))."""
    from ertdiff import _lib
    g = torch.Generator().manual_seed(Ca + 3 * Cout + H + act)
    Cin = Ca + Cb
    x = torch.randn(B, Cin, H, H, generator=g)
    ss = torch.stack([torch.rand(B, Cin, generator=g) + 0.5, torch.randn(B, Cin, generator=g)], -1)
    dy = torch.randn(B, Cout, H, H, generator=g)
    a = x.double() * ss[..., 0, None, None].double() + ss[..., 1, None, None].double()
    if act == 1:
        a = F.silu(a)
    ref = torch.nn.grad.conv2d_weight(a, (Cout, Cin, ks, ks), dy.double(), padding=ks // 2)
    lib = _lib.lib()
    n = lib.ertd_conv_wgrad_ws_bytes(Cin, Cout, B, H, ks, 0)
    ws = torch.empty(n, dtype=torch.uint8, device=cuda_dev)
    xa = x[:, :Ca].contiguous().to(cuda_dev)
    xb = x[:, Ca:].contiguous().to(cuda_dev) if Cb else None
    ssd, dyd = ss.contiguous().to(cuda_dev), dy.to(cuda_dev)
    out = torch.empty((Cout, Cin, ks, ks), device=cuda_dev)
    rc = lib.ertd_conv_wgrad(dyd.data_ptr(), xa.data_ptr(), Ca, None if xb is None else xb.data_ptr(),
                             Cb, B, H, Cout, ks, 0, ssd.data_ptr(), act, out.data_ptr(), 0,
                             ws.data_ptr(), n, _lib.stream_of(cuda_dev))
    assert rc == 0
    err = _rel(out, ref)
    record_error(f"conv_wgrad_act{act}_{Cin}_{Cout}_{H}_k{ks}", err)
    assert err < 1e-5, err
    # an activation needs its scale/shift and is only fused for stride-1 convs
    assert lib.ertd_conv_wgrad(dyd.data_ptr(), xa.data_ptr(), Ca, None if xb is None else xb.data_ptr(),
                               Cb, B, H, Cout, ks, 0, None, act, out.data_ptr(), 0,
                               ws.data_ptr(), n, _lib.stream_of(cuda_dev)) != 0


def test_conv_wgrad_rejects_bad_geometry(cuda_dev):
    from ertdiff import _lib
    lib = _lib.lib()
    assert lib.ertd_conv_wgrad_ws_bytes(64, 64, 2, 8, 3, 0) == 0       # 8x8 rows: outside
    assert lib.ertd_conv_wgrad_ws_bytes(64, 64, 2, 48, 3, 0) == 0      # not a power of two
    assert lib.ertd_conv_wgrad_ws_bytes(64, 64, 2, 32, 1, 1) == 0      # 1x1 stride 2
    assert lib.ertd_conv_wgrad(None, None, 1, None, 0, 1, 16, 1, 3, 0, None, 0, None, 0, None, 0,
                               None) != 0


def test_unet_autograd_matches_fused_step(cuda_dev):
    """The reference loop shape -- pred = model(x_noisy, t, cond); MSELoss;
    loss.backward() -- runs the same HIP kernels as unet_train_step (same
    parameter gradients); dL/dx against float64 autograd."""
    B, L, T = 2, 129, 1000
    cfg = U.CONFIGS["U1"]
    x0 = torch.from_numpy(synth_normal((B, cfg.param_dim), 520)).to(cuda_dev)
    cond = torch.from_numpy(synth_uniform((B, 14, L), 521)).to(cuda_dev)
    t = torch.from_numpy(synth_timesteps(B, T, 522)).to(cuda_dev)
    noise = torch.from_numpy(synth_normal((B, cfg.param_dim), 523)).to(cuda_dev)
    _, _, ab = ertdiff.get_diffusion_schedule(T, device=cuda_dev)
    m1 = ertdiff.ConditionalUNet.from_config("U1", seed=5).to(cuda_dev)
    opt = torch.optim.SGD(m1.parameters(), lr=0.0)     # lr 0: grads only
    m2 = ertdiff.ConditionalUNet.from_config("U1", seed=5).to(cuda_dev)
    opt2 = torch.optim.Adam(m2.parameters(), lr=1e-3)
    ertdiff.train_step(m2, opt2, x0, cond, T, ab, t=t, noise=noise)   # U-Net dispatch
    xn = ertdiff.q_sample(x0, t, noise, ab).requires_grad_(True)
    pred = m1(xn, t, cond)
    assert pred.grad_fn is not None
    loss = F.mse_loss(pred, noise)
    opt.zero_grad()
    loss.backward()
    # (dL/dpred comes from torch's mse_loss backward on one side and ertd_mse_loss
    # on the other: equal up to the rounding of 2 (e - z) / n)
    for (k, p1), (_, p2) in zip(m1.named_parameters(), m2.named_parameters()):
        assert _rel(p1.grad, p2.grad) < 1e-6, k
    W = {k: v.detach().cpu().double() for k, v in m1.named_parameters()}
    xr = xn.detach().cpu().double().requires_grad_(True)
    F.mse_loss(U.forward(xr, t.cpu(), cond.cpu().double(), W, cfg), noise.cpu().double()).backward()
    err = _rel(xn.grad, xr.grad)
    record_error("unet_autograd_dx_U1", err)
    assert err < GRAD_TOL, err


@pytest.mark.parametrize("Ca,Cb,HW,groups,act,acc", [
    (64, 0, 4096, 32, 1, 0),
    (128, 64, 4096, 32, 1, 1),     # concat input at 64x64, accumulate into dx
    (256, 0, 256, 32, 1, 0),       # 16x16: one wave per channel, 4 channels at once
    (128, 64, 1024, 32, 1, 1),     # concat input, accumulate into dx
    (128, 0, 256, 1, 1, 0),        # one group of 128 channels (> 64 per LDS batch)
    (96, 32, 64, 2, 2, 1),         # GN without SiLU (attention norm)
])
def test_gn_act_backward_vs_autograd(Ca, Cb, HW, groups, act, acc, cuda_dev):
    from ertdiff import _lib
    g = torch.Generator().manual_seed(HW + Ca + groups)
    B, C = 3, Ca + Cb
    x = (torch.randn(B, C, HW, generator=g) * 1.7 + 0.3).double()
    gamma = (1 + 0.2 * torch.randn(C, generator=g)).double()
    beta = (0.1 * torch.randn(C, generator=g)).double()
    dy = torch.randn(B, C, HW, generator=g).double()
    prev = torch.randn(B, C, HW, generator=g)
    xr, gr, br = (t.clone().requires_grad_(True) for t in (x, gamma, beta))
    y = F.group_norm(xr.view(B, C, HW, 1), groups, gr, br, eps=1e-5).view(B, C, HW)
    if act == 1:
        y = F.silu(y)
    (y * dy).sum().backward()
    lib = _lib.lib()
    dev = cuda_dev
    xa = x[:, :Ca].float().contiguous().to(dev)
    xb = x[:, Ca:].float().contiguous().to(dev) if Cb else None
    gam, bet = gamma.float().to(dev), beta.float().to(dev)
    ss = torch.empty(B, C, 2, device=dev)
    mr = torch.empty(B, groups, 2, device=dev)
    s = _lib.stream_of(dev)
    assert lib.ertd_gn_stats_mr(xa.data_ptr(), Ca, None if xb is None else xb.data_ptr(), Cb, B, HW,
                                groups, gam.data_ptr(), bet.data_ptr(), ss.data_ptr(), mr.data_ptr(),
                                s) == 0
    dxa = prev[:, :Ca].contiguous().to(dev)
    dxb = prev[:, Ca:].contiguous().to(dev) if Cb else None
    part = torch.empty(B, 2, C, device=dev)
    dyd = dy.float().to(dev)
    assert lib.ertd_gn_act_backward(xa.data_ptr(), Ca, None if xb is None else xb.data_ptr(), Cb, B, HW,
                                    groups, gam.data_ptr(), bet.data_ptr(), mr.data_ptr(), act,
                                    dyd.data_ptr(), dxa.data_ptr(),
                                    None if dxb is None else dxb.data_ptr(), acc, part.data_ptr(),
                                    s) == 0
    dgb = torch.empty(2, C, device=dev)
    assert lib.ertd_reduce_rows(part.data_ptr(), B, 2 * C, dgb.data_ptr(), 0, s) == 0
    dx = dxa if dxb is None else torch.cat([dxa, dxb], 1)
    want = xr.grad + (prev.double() if acc else 0)
    e = [_rel(dx, want), _rel(dgb[0], gr.grad), _rel(dgb[1], br.grad)]
    record_error(f"gn_act_backward_{C}_{HW}_g{groups}_a{act}", max(e))
    assert max(e) < 1e-5, e
    if C // groups <= 64:
        # the fused per-sample pixel sums of the added gradient (into a column
        # block of a wider matrix), and the same dx bits as the plain entry
        dxa2 = prev[:, :Ca].contiguous().to(dev)
        dxb2 = prev[:, Ca:].contiguous().to(dev) if Cb else None
        wide = torch.full((B, C + 7), 5.0, device=dev)
        part2 = torch.empty(B, 2, C, device=dev)
        assert lib.ertd_gn_act_backward_csum(
            xa.data_ptr(), Ca, None if xb is None else xb.data_ptr(), Cb, B, HW, groups, gam.data_ptr(),
            bet.data_ptr(), mr.data_ptr(), act, dyd.data_ptr(), dxa2.data_ptr(),
            None if dxb2 is None else dxb2.data_ptr(), acc, part2.data_ptr(), wide[:, 3:].data_ptr(),
            C + 7, s) == 0
        assert torch.equal(dxa2, dxa) and torch.equal(part2, part)
        if dxb2 is not None:
            assert torch.equal(dxb2, dxb)
        assert torch.all(wide[:, :3] == 5.0) and torch.all(wide[:, 3 + C:] == 5.0)
        ec = _rel(wide[:, 3:3 + C], xr.grad.sum(2))
        record_error(f"gn_act_backward_csum_{C}_{HW}_g{groups}", ec)
        assert ec < 1e-4, ec    # fp32 sums of HW terms (the gradient tests' tolerance)
    # the fused addend (a ResBlock's skip / identity gradient, concatenated
    # channel order): bitwise the separate add (prev + addc, or addc) followed
    # by the plain entry; csum (when given) sums the GroupNorm term only
    addc = torch.randn(B, C, HW, generator=g).to(dev)
    sep = (prev.to(dev) + addc) if acc else addc.clone()
    sa, sb = sep[:, :Ca].contiguous(), (sep[:, Ca:].contiguous() if Cb else None)
    part_s = torch.empty(B, 2, C, device=dev)
    assert lib.ertd_gn_act_backward(xa.data_ptr(), Ca, None if xb is None else xb.data_ptr(), Cb, B, HW,
                                    groups, gam.data_ptr(), bet.data_ptr(), mr.data_ptr(), act,
                                    dyd.data_ptr(), sa.data_ptr(), None if sb is None else sb.data_ptr(),
                                    1, part_s.data_ptr(), s) == 0
    fa = prev[:, :Ca].contiguous().to(dev) if acc else torch.full((B, Ca, HW), float("nan"), device=dev)
    fb = None
    if Cb:
        fb = prev[:, Ca:].contiguous().to(dev) if acc else torch.full((B, Cb, HW), float("nan"), device=dev)
    part_f = torch.empty(B, 2, C, device=dev)
    cs = torch.empty(B, C, device=dev) if C // groups <= 64 else None
    assert lib.ertd_gn_act_backward_add(
        xa.data_ptr(), Ca, None if xb is None else xb.data_ptr(), Cb, B, HW, groups, gam.data_ptr(),
        bet.data_ptr(), mr.data_ptr(), act, dyd.data_ptr(), addc.data_ptr(), fa.data_ptr(),
        None if fb is None else fb.data_ptr(), acc, part_f.data_ptr(),
        None if cs is None else cs.data_ptr(), C, s) == 0
    assert torch.equal(fa, sa) and torch.equal(part_f, part)
    if Cb:
        assert torch.equal(fb, sb)
    if cs is not None:
        assert _rel(cs, xr.grad.sum(2)) < 1e-4
    assert lib.ertd_gn_act_backward_add(
        xa.data_ptr(), Ca, None if xb is None else xb.data_ptr(), Cb, B, HW, groups, gam.data_ptr(),
        bet.data_ptr(), mr.data_ptr(), act, dyd.data_ptr(), None, fa.data_ptr(),
        None if fb is None else fb.data_ptr(), acc, part_f.data_ptr(), None, 0, s) != 0


@pytest.mark.gpu
def test_reduce_rows_multi_bitwise(cuda_dev):
    """ertd_reduce_rows_multi (the train walk's deferred dgamma/dbeta sums): 53
    problems of ragged shapes (two launches of <= 48), accumulate on and off,
    every output bitwise equal to its own ertd_reduce_rows call."""
    import ctypes
    from ertdiff import _lib
    lib = _lib.lib()
    s = _lib.stream_of(cuda_dev)
    g = torch.Generator().manual_seed(11)
    probs = []
    for i in range(53):
        rows = [1, 3, 4, 5, 8, 9, 32, 33][i % 8]
        cols = [1, 63, 64, 65, 128, 1000, 2 * 384][i % 7]
        part = torch.randn(rows, cols, generator=g).to(cuda_dev)
        init = torch.randn(cols, generator=g).to(cuda_dev)
        probs.append((part, rows, cols, init, i % 3 == 0))
    want, outs = [], []
    for part, rows, cols, init, acc in probs:
        o = init.clone()
        assert lib.ertd_reduce_rows(part.data_ptr(), rows, cols, o.data_ptr(), int(acc), s) == 0
        want.append(o)
        outs.append(init.clone())
    arr = lambda v, t=ctypes.c_void_p: (t * len(v))(*v)
    assert lib.ertd_reduce_rows_multi(arr([p[0].data_ptr() for p in probs]), arr([p[1] for p in probs], ctypes.c_int),
                                      arr([p[2] for p in probs], ctypes.c_longlong), arr([o.data_ptr() for o in outs]),
                                      arr([int(p[4]) for p in probs], ctypes.c_int), len(probs), s) == 0
    torch.cuda.synchronize(cuda_dev)
    for w, o in zip(want, outs):
        assert torch.equal(w, o)
    assert lib.ertd_reduce_rows_multi(None, None, None, None, None, 1, s) != 0


@pytest.mark.parametrize("Cin,Cout,H,ks,mode,B,acc", [
    (64, 64, 64, 3, 0, 2, 0),      # Winograd-eligible gradient conv
    (192, 64, 32, 3, 0, 2, 1),     # Cin_grad = 64 -> Cout_grad = 192, accumulate
    (64, 1, 32, 3, 0, 2, 0),       # conv_out's gradient (Cin_grad = 1)
    (1, 32, 32, 3, 0, 2, 0),       # conv_in's gradient (Cout_grad = 1: the Cout = 1 kernel)
    (64, 64, 64, 3, 1, 2, 1),      # stride 2
    (128, 128, 16, 3, 2, 2, 0),    # upsample
    (96, 64, 32, 1, 0, 2, 1),      # 1x1
])
def test_conv_input_grad_vs_autograd(Cin, Cout, H, ks, mode, B, acc, cuda_dev):
    from ertdiff import _lib
    g = torch.Generator().manual_seed(Cin + 3 * Cout + H + mode)
    w = torch.randn(Cout, Cin, ks, ks, generator=g) / (Cin * ks * ks) ** 0.5
    Ho = H // 2 if mode == 1 else (2 * H if mode == 2 else H)
    dy = torch.randn(B, Cout, Ho, Ho, generator=g)
    prev = torch.randn(B, Cin, H, H, generator=g)
    if mode == 2:
        ref = torch.nn.grad.conv2d_input((B, Cin, 2 * H, 2 * H), w.double(), dy.double(), padding=1)
        ref = ref.view(B, Cin, H, 2, H, 2).sum((3, 5))
    else:
        ref = torch.nn.grad.conv2d_input((B, Cin, H, H), w.double(), dy.double(),
                                         stride=2 if mode == 1 else 1, padding=ks // 2)
    if acc:
        ref = ref + prev.double()
    lib = _lib.lib()
    n = lib.ertd_conv_input_grad_ws_bytes(Cin, Cout, B, H, ks, mode)
    ws = torch.empty(n, dtype=torch.uint8, device=cuda_dev)
    dx = prev.to(cuda_dev)
    wd, dyd = w.to(cuda_dev), dy.to(cuda_dev)
    assert lib.ertd_conv_input_grad(dyd.data_ptr(), B, H, wd.data_ptr(), Cout, Cin, ks, mode,
                                    dx.data_ptr(), acc, ws.data_ptr(), n, _lib.stream_of(cuda_dev)) == 0
    err = _rel(dx, ref)
    record_error(f"conv_input_grad_{Cin}_{Cout}_{H}_k{ks}_m{mode}", err)
    assert err < 1e-5, err


def _dp_train_worker(rank, world, port, q):
    import os
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    # both ranks on the one GPU of the box: gloo carries the (device) gradient bucket
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        cfg = U.CONFIGS["U1"]
        Bg, L, T = 4, 65, 1000
        x0 = torch.from_numpy(synth_normal((Bg, cfg.param_dim), 530)).to(dev)
        cond = torch.from_numpy(synth_uniform((Bg, 14, L), 531)).to(dev)
        t = torch.from_numpy(synth_timesteps(Bg, T, 532)).to(dev)
        noise = torch.from_numpy(synth_normal((Bg, cfg.param_dim), 533)).to(dev)
        _, _, ab = ertdiff.get_diffusion_schedule(T, device=dev)
        m = ertdiff.ConditionalUNet.from_config("U1", seed=9).to(dev)
        opt = torch.optim.Adam(m.parameters(), lr=1e-3)
        sh = slice(rank * Bg // world, (rank + 1) * Bg // world)
        unet_train_step(m, opt, x0[sh], cond[sh], T, ab, t=t[sh], noise=noise[sh])
        # numpy (pickled by value): torch CPU tensors would travel as shared-memory
        # handles that die with this process
        q.put((rank, {k: p.grad.cpu().numpy() for k, p in m.named_parameters()},
               {k: p.detach().cpu().numpy() for k, p in m.named_parameters()}))
    finally:
        dist.destroy_process_group()


def test_unet_train_data_parallel(cuda_dev):
    """Two data-parallel ranks with half the batch each end with the full-batch
    gradient (the mean of their shard means) and identical parameters."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dp_train_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (g, w)) for r, g, w in (q.get(timeout=300) for _ in range(2)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single process, whole batch
    cfg = U.CONFIGS["U1"]
    Bg, L, T = 4, 65, 1000
    x0 = torch.from_numpy(synth_normal((Bg, cfg.param_dim), 530)).to(cuda_dev)
    cond = torch.from_numpy(synth_uniform((Bg, 14, L), 531)).to(cuda_dev)
    t = torch.from_numpy(synth_timesteps(Bg, T, 532)).to(cuda_dev)
    noise = torch.from_numpy(synth_normal((Bg, cfg.param_dim), 533)).to(cuda_dev)
    _, _, ab = ertdiff.get_diffusion_schedule(T, device=cuda_dev)
    m = ertdiff.ConditionalUNet.from_config("U1", seed=9).to(cuda_dev)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    unet_train_step(m, opt, x0, cond, T, ab, t=t, noise=noise)
    norms = [float(p.grad.double().norm()) for p in m.parameters()]
    floor = 1e-3 * float(np.sqrt(np.mean(np.square(norms))))
    worst = 0.0
    for (k, p), nr in zip(m.named_parameters(), norms):
        for r in range(2):
            e = float(np.linalg.norm(res[r][0][k].astype(np.float64) -
                                     p.grad.detach().cpu().double().numpy())) / max(nr, floor)
            worst = max(worst, e)
        assert np.array_equal(res[0][1][k], res[1][1][k]), k     # replicas identical
    record_error("unet_train_dp2_vs_single", worst)
    assert worst < 1e-5, worst


def test_unet_train_step_u5_runs(cuda_dev):
    """configs[4]'s network (128x128, 4 levels, ch 128, mid attention) through
    the fp32 train step: finite loss, every gradient finite, and a second step
    on the same batch lowers the loss (no spec comparison at this size: the
    float64 CPU autograd of U5 is minutes; U1/U2/U3 are pinned above)."""
    cfg = U.CONFIGS["U5"]
    B, L, T = 1, 65, 1000
    m = ertdiff.ConditionalUNet.from_config("U5", seed=1).to(cuda_dev)
    opt = torch.optim.Adam(m.parameters(), lr=1e-4)
    x0 = torch.from_numpy(synth_normal((B, cfg.param_dim), 540)).to(cuda_dev)
    cond = torch.from_numpy(synth_uniform((B, 14, L), 541)).to(cuda_dev)
    t = torch.tensor([321], device=cuda_dev)
    noise = torch.from_numpy(synth_normal((B, cfg.param_dim), 542)).to(cuda_dev)
    _, _, ab = ertdiff.get_diffusion_schedule(T, device=cuda_dev)
    l0 = unet_train_step(m, opt, x0, cond, T, ab, t=t, noise=noise)
    assert np.isfinite(l0)
    assert all(bool(torch.isfinite(p.grad).all()) for p in m.parameters())
    l1 = unet_train_step(m, opt, x0, cond, T, ab, t=t, noise=noise)
    assert l1 < l0, (l0, l1)


@pytest.mark.parametrize("Ca,Cb,Cout,H,mode,act,B", [
    (64, 0, 64, 64, 0, 1, 4),      # ResBlock conv at 64x64 (register-weight F(4x4))
    (128, 64, 128, 32, 0, 1, 4),   # concat input
    (128, 0, 128, 16, 2, 0, 4),    # Upsample conv 16 -> 32
    (64, 0, 64, 64, 0, 1, 32),     # the train batch
    (1, 0, 64, 64, 0, 0, 4),       # conv_in (one input channel)
    (1, 0, 96, 32, 0, 0, 2),       # conv_in, a partial 64-channel group
])
def test_conv2d_gn_parts_finalize(Ca, Cb, Cout, H, mode, act, B, cuda_dev):
    """ertd_conv2d_gn / _run_gn (the train walk's forward convs): the same output
    bits as ertd_conv2d, and the epilogue's GroupNorm partials finalized give
    the statistics of a separate pass (ertd_gn_stats_mr) to fp32 rounding."""
    from ertdiff import _lib
    lib = _lib.lib()
    dev, s = cuda_dev, _lib.stream_of(cuda_dev)
    g = torch.Generator(device=dev).manual_seed(Ca + Cout + H + mode)
    Cin = Ca + Cb
    Ho = 2 * H if mode == 2 else H
    xa = torch.randn(B, Ca, H, H, device=dev, generator=g)
    xb = torch.randn(B, Cb, H, H, device=dev, generator=g) if Cb else None
    w = torch.randn(Cout, Cin, 3, 3, device=dev, generator=g) * 0.05
    bias = torch.randn(Cout, device=dev, generator=g)
    gn = torch.randn(B, Cin, 2, device=dev, generator=g) * 0.5 if act else None
    np_ = lib.ertd_conv2d_gn_parts(Ca, Cb, Cout, 3, mode, act, 0, B, H)
    assert np_ > 0
    assert lib.ertd_conv2d_gn_parts(Ca, Cb, 1, 3, 0, act, 0, B, H) == 0     # conv_out: none
    n = lib.ertd_conv2d_workspace_bytes(Cin, Cout, 3, 0, B, H, mode)
    ws = torch.empty(n, dtype=torch.uint8, device=dev)
    ref = torch.empty(B, Cout, Ho, Ho, device=dev)
    args = (xa.data_ptr(), Ca, None if xb is None else xb.data_ptr(), Cb, B, H)
    tail = (Cout, 3, mode, None if gn is None else gn.data_ptr(), act, None, 0, None)
    assert lib.ertd_conv2d(*args, w.data_ptr(), bias.data_ptr(), *tail, ref.data_ptr(), 0, ws.data_ptr(), n,
                           s) == 0
    out = torch.empty_like(ref)
    parts = torch.empty(B, Cout, np_, 2, device=dev)
    assert lib.ertd_conv2d_gn(*args, w.data_ptr(), bias.data_ptr(), *tail, out.data_ptr(), 0, ws.data_ptr(),
                              n, parts.data_ptr(), np_, s) == 0
    assert torch.equal(out, ref)
    out2, parts2 = torch.empty_like(ref), torch.empty_like(parts)
    assert lib.ertd_conv2d_run_gn(*args, bias.data_ptr(), *tail, out2.data_ptr(), 0, ws.data_ptr(), n,
                                  parts2.data_ptr(), np_, s) == 0
    assert torch.equal(out2, ref) and torch.equal(parts2, parts)
    assert lib.ertd_conv2d_run_gn(*args, bias.data_ptr(), *tail, out2.data_ptr(), 0, ws.data_ptr(), n,
                                  parts2.data_ptr(), np_ + 1, s) != 0           # wrong part count
    groups = 32
    gam = 1 + 0.1 * torch.randn(Cout, device=dev, generator=g)
    bet = 0.1 * torch.randn(Cout, device=dev, generator=g)
    ss, mr = torch.empty(B, Cout, 2, device=dev), torch.empty(B, groups, 2, device=dev)
    assert lib.ertd_group_norm_finalize(parts.data_ptr(), np_, Cout, None, 0, 0, B, Ho * Ho, groups,
                                        gam.data_ptr(), bet.data_ptr(), ss.data_ptr(), mr.data_ptr(), s) == 0
    ss_r, mr_r = torch.empty_like(ss), torch.empty_like(mr)
    assert lib.ertd_gn_stats_mr(ref.data_ptr(), Cout, None, 0, B, Ho * Ho, groups, gam.data_ptr(),
                                bet.data_ptr(), ss_r.data_ptr(), mr_r.data_ptr(), s) == 0
    e = max(_rel(ss, ss_r), _rel(mr, mr_r))
    record_error(f"conv2d_gn_parts_{Cin}_{Cout}_{Ho}_m{mode}", e)
    assert e < 1e-6, e
