"""GPU train step (ERT_Conditional_Diffusion.py:309-319) vs the golden vectors
of the reference's own train step (fixed t / noise, seed-42 weights, 3 Adam
steps) and vs the float64 hand-derived backward.  fp32 tolerances: loss 1e-5
rel, gradients 1e-4 rel-L2 per tensor (the reference's own fp32 gradients sit
up to 3.3e-5 from float64), Adam parameter deltas 1e-3 rel-L2 (tiny gradients
make m/sqrt(v) sign-sensitive)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

import ertdiff
from oracle import ref_numpy as RN
from synth import synth_normal, synth_timesteps, synth_uniform

pytestmark = pytest.mark.gpu
GRAD_TOL = 1e-4


def _fresh_model(golden_weights, dev):
    m = ertdiff.ConditionalDiffusionModel(29, 128)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in golden_weights.items()})
    return m.to(dev).train()


def _rel(a, b):
    return RN.rel_l2(a.detach().double().cpu().numpy(), np.asarray(b, np.float64))


def test_train_step_vs_golden(golden_weights, train_kat, cuda_dev):
    m = _fresh_model(golden_weights, cuda_dev)
    opt = torch.optim.Adam(m.parameters(), lr=1e-4)
    T = int(train_kat["T"])
    _, _, ab = ertdiff.get_diffusion_schedule(T, device=cuda_dev)
    x0 = torch.from_numpy(train_kat["x0"]).to(cuda_dev)
    cond = torch.from_numpy(synth_uniform((8, 14, 4693), int(train_kat["cs"]))).to(cuda_dev)
    for step in range(3):
        t = torch.from_numpy(train_kat[f"t{step}"]).to(cuda_dev)
        noise = torch.from_numpy(train_kat[f"noise{step}"]).to(cuda_dev)
        loss = ertdiff.train_step(m, opt, x0, cond, T, ab, t=t, noise=noise)
        ref = float(train_kat[f"loss{step}"])
        assert abs(loss - ref) <= 1e-5 * abs(ref), (step, loss, ref)
        if step == 0:
            for k, p in m.named_parameters():
                assert _rel(p.grad, train_kat[f"grad0/{k}"]) < GRAD_TOL, k
        if step in (0, 2):
            for k, p in m.named_parameters():
                d = p.detach().double().cpu().numpy() - golden_weights[k]
                dref = train_kat[f"param{step}/{k}"].astype(np.float64) - golden_weights[k]
                assert RN.rel_l2(d, dref) < 1e-3, (step, k)
    # Adam state is torch's: step counters and buffers round-trip through state_dict
    sd = opt.state_dict()
    assert float(sd["state"][0]["step"]) == 3.0
    opt2 = torch.optim.Adam(ertdiff.ConditionalDiffusionModel(29).parameters(), lr=1e-4)
    opt2.load_state_dict(sd)


def test_autograd_backward_vs_golden(golden_weights, train_kat, cuda_dev):
    m = _fresh_model(golden_weights, cuda_dev)
    x = torch.from_numpy(train_kat["x_noisy0"]).to(cuda_dev).requires_grad_(True)
    t = torch.from_numpy(train_kat["t0"]).to(cuda_dev)
    noise = torch.from_numpy(train_kat["noise0"]).to(cuda_dev)
    cond = torch.from_numpy(synth_uniform((8, 14, 4693), int(train_kat["cs"]))).to(cuda_dev)
    pred = m(x, t, cond)
    assert _rel(pred, train_kat["pred0"]) < 1e-5
    loss = F.mse_loss(pred, noise)
    assert abs(loss.item() - float(train_kat["loss0"])) <= 1e-5 * float(train_kat["loss0"])
    loss.backward()
    for k, p in m.named_parameters():
        assert _rel(p.grad, train_kat[f"grad0/{k}"]) < GRAD_TOL, k
    # dL/dx against the float64 backward
    W = golden_weights
    f = RN.forward_full(train_kat["x_noisy0"], train_kat["t0"],
                        synth_uniform((8, 14, 4693), int(train_kat["cs"])), W)
    dout = 2.0 * (f["out"] - train_kat["noise0"]) / f["out"].size
    dz5 = (dout @ W["mlp.2.weight"].astype(np.float64)) * (f["z5"] > 0)
    dx_ref = dz5 @ W["mlp.0.weight"].astype(np.float64)[:, :29]
    assert _rel(x.grad, dx_ref) < GRAD_TOL


def test_fused_step_equals_autograd_grads(golden_weights, cuda_dev):
    """train_step's fused path and the autograd path run the same kernels."""
    B, L, T = 6, 700, 500
    x0 = torch.from_numpy(synth_normal((B, 29), 201)).to(cuda_dev)
    cond = torch.from_numpy(synth_uniform((B, 14, L), 202)).to(cuda_dev)
    t = torch.from_numpy(synth_timesteps(B, T, 203)).to(cuda_dev)
    noise = torch.from_numpy(synth_normal((B, 29), 204)).to(cuda_dev)
    _, _, ab = ertdiff.get_diffusion_schedule(T, device=cuda_dev)
    m1 = _fresh_model(golden_weights, cuda_dev)
    opt = torch.optim.Adam(m1.parameters(), lr=1e-4)
    ertdiff.train_step(m1, opt, x0, cond, T, ab, t=t, noise=noise)
    g1 = {k: p.grad.clone() for k, p in m1.named_parameters()}
    m2 = _fresh_model(golden_weights, cuda_dev)
    x = ertdiff.q_sample(x0, t, noise, ab)
    F.mse_loss(m2(x, t, cond), noise).backward()
    for k, p in m2.named_parameters():
        assert torch.equal(p.grad, g1[k]), k


@pytest.mark.parametrize("B,L", [(3, 37), (5, 250), (2, 1), (4, 4693), (32, 4693)])
def test_grads_vs_fp64_backward(B, L, golden_weights, cuda_dev):
    x = synth_normal((B, 29), 300 + L)
    t = synth_timesteps(B, 500, 301 + L)
    noise = synth_normal((B, 29), 302 + L)
    cond = synth_uniform((B, 14, L), 303 + L)
    m = _fresh_model(golden_weights, cuda_dev)
    xd = torch.from_numpy(x).to(cuda_dev)
    loss = F.mse_loss(m(xd, torch.from_numpy(t).to(cuda_dev), torch.from_numpy(cond).to(cuda_dev)),
                      torch.from_numpy(noise).to(cuda_dev))
    loss.backward()
    f = RN.forward_full(x, t, cond, golden_weights)
    ref_loss, g = RN.backward(f, noise, golden_weights)
    assert abs(loss.item() - ref_loss) < 1e-5 * ref_loss
    for k, p in m.named_parameters():
        if np.linalg.norm(g[k]) == 0:
            assert float(p.grad.abs().max()) == 0.0, k
            continue
        assert _rel(p.grad, g[k]) < GRAD_TOL, (k, _rel(p.grad, g[k]))


def test_train_step_deterministic(golden_weights, cuda_dev):
    B, L, T = 32, 4693, 500
    x0 = torch.from_numpy(synth_normal((B, 29), 401)).to(cuda_dev)
    cond = torch.from_numpy(synth_uniform((B, 14, L), 402)).to(cuda_dev)
    _, _, ab = ertdiff.get_diffusion_schedule(T, device=cuda_dev)
    outs = []
    for _ in range(2):
        m = _fresh_model(golden_weights, cuda_dev)
        opt = torch.optim.Adam(m.parameters(), lr=1e-4)
        g = torch.Generator(device=cuda_dev).manual_seed(5)
        losses = []
        for s in range(5):
            t = torch.randint(0, T, (B,), device=cuda_dev, generator=g)
            n = torch.randn(B, 29, device=cuda_dev, generator=g)
            losses.append(ertdiff.train_step(m, opt, x0, cond, T, ab, t=t, noise=n))
        outs.append((losses, [p.detach().clone() for p in m.parameters()]))
    assert outs[0][0] == outs[1][0]
    assert all(torch.equal(a, b) for a, b in zip(outs[0][1], outs[1][1]))
    assert all(np.isfinite(outs[0][0]))


def _train_inputs(B, L, T, seed, dev):
    x0 = torch.from_numpy(synth_normal((B, 29), seed)).to(dev)
    cond = torch.from_numpy(synth_uniform((B, 14, L), seed + 1)).to(dev)
    g = torch.Generator(device=dev).manual_seed(seed + 2)
    ts = [torch.randint(0, T, (B,), device=dev, generator=g) for _ in range(4)]
    ns = [torch.randn(B, 29, device=dev, generator=g) for _ in range(4)]
    return x0, cond, ts, ns


@pytest.mark.parametrize("B,L", [(32, 4693), (3, 37)])
def test_train_plan_equals_eager(B, L, golden_weights, cuda_dev):
    """TrainPlan (one captured graph per step, device-side Adam step count)
    replays the eager train_step bit for bit: losses, gradients, parameters,
    and the torch.optim.Adam state (step counters, exp_avg, exp_avg_sq)."""
    T = 500
    x0, cond, ts, ns = _train_inputs(B, L, T, 610, cuda_dev)
    _, _, ab = ertdiff.get_diffusion_schedule(T, device=cuda_dev)
    m1 = _fresh_model(golden_weights, cuda_dev)
    o1 = torch.optim.Adam(m1.parameters(), lr=1e-4)
    l1 = [ertdiff.train_step(m1, o1, x0, cond, T, ab, t=ts[i], noise=ns[i]) for i in range(4)]
    m2 = _fresh_model(golden_weights, cuda_dev)
    o2 = torch.optim.Adam(m2.parameters(), lr=1e-4)
    plan = ertdiff.TrainPlan(m2, o2, B, L, T, ab)
    l2 = [plan.step(x0, cond, t=ts[i], noise=ns[i]) for i in range(4)]
    assert l1 == l2
    for (k, p1), p2 in zip(m1.named_parameters(), m2.parameters()):
        assert torch.equal(p1, p2), k
        assert torch.equal(p1.grad, p2.grad), k
        s1, s2 = o1.state[p1], o2.state[p2]
        assert float(s1["step"]) == float(s2["step"]) == 4.0
        assert torch.equal(s1["exp_avg"], s2["exp_avg"]) and torch.equal(s1["exp_avg_sq"], s2["exp_avg_sq"])
    # the eager path continues from the plan's state
    la = ertdiff.train_step(m1, o1, x0, cond, T, ab, t=ts[0], noise=ns[0])
    lb = ertdiff.train_step(m2, o2, x0, cond, T, ab, t=ts[0], noise=ns[0])
    assert la == lb
    # ... and the plan from weights and Adam steps changed outside it (eager
    # steps, a user's in-place edit): it follows the step count
    with torch.no_grad():
        for m in (m1, m2):
            m.condition_encoder[0].weight.mul_(0.75)
            m.condition_encoder[2].weight.add_(0.01)
    la = [ertdiff.train_step(m1, o1, x0, cond, T, ab, t=ts[i], noise=ns[i]) for i in (1, 2)]
    lb = [plan.step(x0, cond, t=ts[i], noise=ns[i]) for i in (1, 2)]
    assert la == lb
    for (k, p1), p2 in zip(m1.named_parameters(), m2.parameters()):
        assert torch.equal(p1, p2), k


def test_train_plan_draws_match_torch(golden_weights, cuda_dev):
    """The graph's draws are torch's own: after manual_seed, a replay draws the
    t and noise that torch.randint / torch.randn_like draw eagerly (:312-313),
    and the step equals the eager step on them."""
    B, L, T = 8, 4693, 1000
    x0, cond, _, _ = _train_inputs(B, L, T, 620, cuda_dev)
    _, _, ab = ertdiff.get_diffusion_schedule(T, device=cuda_dev)
    m2 = _fresh_model(golden_weights, cuda_dev)
    o2 = torch.optim.Adam(m2.parameters(), lr=1e-4)
    plan = ertdiff.TrainPlan(m2, o2, B, L, T, ab, rng="torch")
    m1 = _fresh_model(golden_weights, cuda_dev)
    o1 = torch.optim.Adam(m1.parameters(), lr=1e-4)
    for s in range(3):
        torch.manual_seed(77 + s)
        lp = plan.step(x0, cond)
        torch.manual_seed(77 + s)
        t = torch.randint(0, T, (B,), device=cuda_dev).long()
        n = torch.randn_like(x0)
        assert torch.equal(plan.t, t) and torch.equal(plan.noise, n), s
        assert ertdiff.train_step(m1, o1, x0, cond, T, ab, t=t, noise=n) == lp, s
    plan.run(5)
    torch.cuda.synchronize()
    assert float(o2.state_dict()["state"][0]["step"]) == 8.0
    assert np.isfinite(float(plan.loss))


def test_train_plan_philox_draws(golden_weights, cuda_dev):
    """rng="philox": the step draws t ~ U{0..T-1} and noise ~ N(0,1) in its head
    kernel (keyed by seed, member, Adam step); the step equals the eager step
    on the drawn values, and a second plan with the same seed repeats it."""
    B, L, T = 32, 4693, 1000
    x0, cond, _, _ = _train_inputs(B, L, T, 630, cuda_dev)
    _, _, ab = ertdiff.get_diffusion_schedule(T, device=cuda_dev)
    runs = []
    for rep in range(2):
        m2 = _fresh_model(golden_weights, cuda_dev)
        o2 = torch.optim.Adam(m2.parameters(), lr=1e-4)
        plan = ertdiff.TrainPlan(m2, o2, B, L, T, ab, seed=1234)
        m1 = _fresh_model(golden_weights, cuda_dev)
        o1 = torch.optim.Adam(m1.parameters(), lr=1e-4)
        ts, ns, ls = [], [], []
        for s in range(3):
            lp = plan.step(x0, cond)
            t, n = plan.t.clone(), plan.noise.clone()
            assert int(t.min()) >= 0 and int(t.max()) < T
            assert ertdiff.train_step(m1, o1, x0, cond, T, ab, t=t, noise=n) == lp, s
            ts.append(t); ns.append(n); ls.append(lp)
        assert not torch.equal(ts[0], ts[1]) and not torch.equal(ns[0], ns[1])
        runs.append((ts, ns, ls))
    assert runs[0][2] == runs[1][2]
    assert all(torch.equal(a, b) for a, b in zip(runs[0][0], runs[1][0]))
    # the draws are standard normal / uniform over many steps
    m = _fresh_model(golden_weights, cuda_dev)
    plan = ertdiff.TrainPlan(m, torch.optim.Adam(m.parameters(), lr=1e-4), B, L, T, ab, seed=99)
    zs, tt = [], []
    for _ in range(40):
        plan.step(x0, cond, return_tensor=True)
        zs.append(plan.noise.clone()); tt.append(plan.t.clone())
    z = torch.cat(zs).double()
    assert abs(float(z.mean())) < 0.05 and abs(float(z.std()) - 1.0) < 0.05
    tv = torch.cat(tt).double()
    assert abs(float(tv.mean()) - (T - 1) / 2) < 0.06 * T


def test_train_plan_input_checks_and_state(golden_weights, cuda_dev):
    """TrainPlan guards: a schedule shorter than T and an out-of-range
    or misshapen t raise before anything reaches the device; building a plan
    leaves p.grad untouched; an lr edited between steps (a scheduler) is
    followed exactly as the eager step follows it; a replay bumps the
    parameters' autograd version counters."""
    B, L, T = 4, 256, 100
    x0, cond, ts, ns = _train_inputs(B, L, T, 640, cuda_dev)
    _, _, ab = ertdiff.get_diffusion_schedule(T, device=cuda_dev)
    m2 = _fresh_model(golden_weights, cuda_dev)
    o2 = torch.optim.Adam(m2.parameters(), lr=1e-4)
    with pytest.raises(IndexError):
        ertdiff.TrainPlan(m2, o2, B, L, T + 1, ab)
    for p in m2.parameters():
        p.grad = torch.full_like(p, 3.0)
    plan = ertdiff.TrainPlan(m2, o2, B, L, T, ab)
    assert all(bool((p.grad == 3.0).all()) for p in m2.parameters())
    bad_t = ts[0].clone()
    bad_t[1] = T
    with pytest.raises(IndexError):
        plan.step(x0, cond, t=bad_t, noise=ns[0])
    with pytest.raises(RuntimeError):
        plan.step(x0, cond, t=ts[0][:2], noise=ns[0])
    m1 = _fresh_model(golden_weights, cuda_dev)
    o1 = torch.optim.Adam(m1.parameters(), lr=1e-4)
    v0 = [p._version for p in m2.parameters()]
    for i in range(4):
        if i == 2:
            for o in (o1, o2):
                o.param_groups[0]["lr"] = 3e-4
        la = ertdiff.train_step(m1, o1, x0, cond, T, ab, t=ts[i], noise=ns[i])
        lb = plan.step(x0, cond, t=ts[i], noise=ns[i])
        assert la == lb, i
    assert all(p._version > v for p, v in zip(m2.parameters(), v0))
    for (k, p1), p2 in zip(m1.named_parameters(), m2.parameters()):
        assert torch.equal(p1, p2), k
        assert float(o1.state[p1]["step"]) == float(o2.state[p2]["step"]) == 4.0


def test_train_plan_run_multistep_graph_equals_steps(golden_weights, cuda_dev):
    """run(n) replays a 32-step graph, then 8-step graphs (RUN_STEPS), then the
    1-step graph for the rest; with Philox draws keyed by (seed, member, Adam
    step) that is bitwise the same as n single replays."""
    B, L, T = 8, 4693, 1000
    x0, cond, _, _ = _train_inputs(B, L, T, 650, cuda_dev)
    _, _, ab = ertdiff.get_diffusion_schedule(T, device=cuda_dev)
    ms, os_, plans = [], [], []
    for _ in range(2):
        m = _fresh_model(golden_weights, cuda_dev)
        o = torch.optim.Adam(m.parameters(), lr=1e-4)
        p = ertdiff.TrainPlan(m, o, B, L, T, ab, seed=4242)
        p.x0.copy_(x0)
        p.cond.copy_(cond)
        ms.append(m); os_.append(o); plans.append(p)
    plans[0].run(43)                       # one 32-step, one 8-step replay + three single steps
    for _ in range(43):
        plans[1].step()
    torch.cuda.synchronize()
    assert torch.equal(plans[0].loss, plans[1].loss)
    for (k, p1), p2 in zip(ms[0].named_parameters(), ms[1].parameters()):
        assert torch.equal(p1, p2), k
        s1, s2 = os_[0].state[p1], os_[1].state[p2]
        assert float(s1["step"]) == float(s2["step"]) == 43.0, k
        assert torch.equal(s1["exp_avg"], s2["exp_avg"]) and torch.equal(s1["exp_avg_sq"], s2["exp_avg_sq"]), k
