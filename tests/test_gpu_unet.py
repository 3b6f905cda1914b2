"""Build-defined U-Net (SURVEY.md 8a') on the GPU against its specification,
oracle/unet_torch.py on the CPU.  PARITY UNPINNED vs the reference (which has
no U-Net): these tests pin the HIP path to the build's own fp32 module.

Tolerances: forward <= 1e-5 rel-L2 (fp32 MFMA k-ordered chains vs oneDNN's
blocked sums), T-step sampler <= 1e-4 (north star), at every recorded step of
a full T = 1000 chain of the headline network (tests/golden/unet_sampler_kat.npz).
bf16-operand precision (configs[2] / configs[4]): budgets stated below, measured
values in DESIGN.md 4.3."""
import numpy as np
import pytest
import torch

import ertdiff
from oracle import unet_torch as U
from oracle import ref_numpy as RN
from synth import synth_normal, synth_uniform
from conftest import record_error

pytestmark = pytest.mark.gpu


def _pair(name, dev, seed=0):
    m = ertdiff.ConditionalUNet.from_config(name, seed=seed).to(dev).eval()
    W = U.init_weights(U.CONFIGS[name], seed)
    return m, W


def _model_from_spec(name, W, dev, precision="fp32"):
    """The GPU model holding exactly the spec's weight dict (e.g. random GN affine)."""
    m = ertdiff.ConditionalUNet.from_config(name, seed=0, precision=precision)
    m.load_state_dict(W)
    return m.to(dev).eval()


@pytest.mark.parametrize("name,B,L,ts", [
    ("U1", 3, 257, [0, 17, 999]),
    ("U2", 2, 4693, [5, 640]),
    ("U3", 2, 1001, [999, 1]),
    ("U5", 1, 257, [777]),
])
def test_unet_forward_vs_oracle(name, B, L, ts, cuda_dev):
    m, W = _pair(name, cuda_dev)
    cfg = U.CONFIGS[name]
    x = torch.from_numpy(synth_normal((B, cfg.param_dim), 101))
    cond = torch.from_numpy(synth_uniform((B, 14, L), 102))
    t = torch.tensor(ts)
    out, cemb = m(x.to(cuda_dev), t.to(cuda_dev), cond.to(cuda_dev), return_cond_emb=True)
    with torch.no_grad():
        ref = U.forward(x, t, cond, W, cfg)
        rc = U.condition_embedding(cond, W)
    assert RN.rel_l2(cemb.cpu().double().numpy(), rc.double().numpy()) < 1e-5
    err = RN.rel_l2(out.cpu().double().numpy(), ref.double().numpy())
    record_error(f"unet_forward_{name}_fp32", err)
    assert err < 1e-5, err


def _cus(dev):
    return torch.cuda.get_device_properties(dev).multi_processor_count


def test_unet_u2_b64_forward_headline_path_random_affine(cuda_dev):
    """The exact headline kernel path (configs[1]: U2, B = 64, L = 4693): at
    B = 64 every ResBlock 3x3 conv runs the register-weight F(4x4) kernel
    unsplit (at 16x16 its 64 co x 16 tile items are 64 x 4 = 256 >= the CUs) --
    the variants the bench times -- against the spec, with trained-model-like
    GroupNorm gamma/beta (random per channel), so a gamma/beta tensor wired to
    the wrong GroupNorm, or a concatenated input's gamma in the wrong channel
    order, fails here."""
    name, B, L = "U2", 64, 4693
    cfg = U.CONFIGS[name]
    W = U.init_weights(cfg, 11, affine="random")
    m = _model_from_spec(name, W, cuda_dev)
    x = torch.from_numpy(synth_normal((B, cfg.param_dim), 141))
    cond = torch.from_numpy(synth_uniform((B, 14, L), 142))
    t = torch.arange(B) * 997 % 1000
    with torch.no_grad():
        out = m(x.to(cuda_dev), t.to(cuda_dev), cond.to(cuda_dev)).cpu()
        ref = U.forward(x, t, cond, W, cfg)
    err = RN.rel_l2(out.double().numpy(), ref.double().numpy())
    record_error("unet_forward_U2_B64_L4693_affine_random", err)
    assert err < 1e-5, err


def test_unet_forward_batch_split_consistency(cuda_dev):
    """Two different dispatches of the 16x16 ResBlock convs on the same members:
    at B = CUs / 4 (64 on 256 CUs, the headline) the register-weight F(4x4)
    kernel's 64 co x 16 tile items fill the CUs and run unsplit; each half
    (B = CUs / 8) has half as many items and splits its K in two (half 1's sums
    to the K-split buffer, added afterwards) -- another summation order, same
    math.  The two must agree to rounding, and one member of each against the
    spec (test above for the whole B = 64 batch)."""
    cus = _cus(cuda_dev)
    m = ertdiff.ConditionalUNet.from_config("U2", seed=3).to(cuda_dev).eval()
    cfg = U.CONFIGS["U2"]
    W = U.init_weights(cfg, 3)
    B = cus // 4
    x = torch.from_numpy(synth_normal((B, cfg.param_dim), 131))
    cond = torch.from_numpy(synth_uniform((B, 14, 257), 132))
    t = torch.arange(B) * 7 % 1000
    xd, cd, td = x.to(cuda_dev), cond.to(cuda_dev), t.to(cuda_dev)
    h = B // 2
    with torch.no_grad():
        full = m(xd, td, cd).cpu()
        split = torch.cat([m(xd[:h], td[:h], cd[:h]), m(xd[h:], td[h:], cd[h:])]).cpu()
        ref = U.forward(x[h - 1:h + 1], t[h - 1:h + 1], cond[h - 1:h + 1], W, cfg)
    err = RN.rel_l2(full.double().numpy(), split.double().numpy())
    record_error(f"unet_forward_U2_B{B}_vs_two_halves", err)
    assert not torch.equal(full, split)      # different schedules: not the same sums
    assert err < 1e-5, err
    for got, name in ((full, "unsplit"), (split, "ksplit")):
        e = RN.rel_l2(got[h - 1:h + 1].double().numpy(), ref.double().numpy())
        record_error(f"unet_forward_U2_{name}_members_vs_spec", e)
        assert e < 1e-5, (name, e)


SAMPLER_TOL = 1e-4
# PLAIN bf16 operands (precision="bf16": one bf16 MFMA per product) are NOT the
# mode the bench reports for configs[2] / configs[4] -- that is split-bf16
# (bf16x3, gated at the north star's 1e-4 below, BF16X3_SAMPLER_TOL).  Plain
# bf16 is kept as a faster, lower-accuracy mode (bench extra *_bf16_plain,
# "meets_tolerance": false); these budgets bound its drift, they are not a
# parity claim.  Budget at T = 1000: against the bf16 spec (same
# operand rounding, another fp32 summation order: flips of single bf16
# roundings cascade through ~40 convs per step and 1000 steps) and against the
# fp32 spec (the price of bf16 operands itself).
# measured: 1.5e-4 vs the bf16 spec and 1.5e-3 vs the fp32 spec
# at step 1000 -- the latter is the spec-vs-spec gap itself (1.5e-3,
# test_host.test_unet_sampler_golden_fixture_shape)
BF16_SAMPLER_TOL = {"bf16_spec": 1e-3, "fp32_spec": 3e-3}


def _noise(T, B, P, seed, dev):
    """synth_normal((T, B, P), seed) on the device, made one step at a time."""
    out = torch.empty(T, B, P, dtype=torch.float32, device=dev)
    for k in range(T):
        out[k] = torch.from_numpy(synth_normal((B, P), seed, k * B * P))
    return out


def _run_golden_chain(kat, key, dev, precision=None):
    """Replays the golden case on the GPU as consecutive plan segments ending at
    each recorded step count; returns {count: x}.  precision: the model's (default:
    the case's spec precision)."""
    name = {"u2": "U2", "u3": "U3", "u5": "U5"}[key[:2]]
    meta = [int(v) for v in kat[f"{key}_meta"]]
    wseed, B, L, cseed, nseed, bf16 = meta[:6]
    aff = meta[6] if len(meta) > 6 else 0
    T = int(kat["T"])
    W = U.init_weights(U.CONFIGS[name], wseed, affine="random" if aff else "ones")
    m = _model_from_spec(name, W, dev, precision=precision or ("bf16" if bf16 else "fp32"))
    P = m.param_dim
    cond = torch.from_numpy(synth_uniform((B, 14, L), cseed)).to(dev)
    noise = _noise(T, B, P, nseed, dev)
    sched = ertdiff.get_diffusion_schedule(T, device=dev)
    x = noise[0].clone()
    done, out = 0, {}
    for k in (int(r) for r in kat["record"]):
        plan = ertdiff.UNetSamplerPlan(m, cond, T, *sched, t_first=T - 1 - done, n_run=k - done,
                                       noise=noise)
        plan.x.copy_(x)
        plan.launch()
        torch.cuda.synchronize()
        x = plan.x.clone()
        plan.close()
        done = k
        out[k] = x.cpu().double().numpy()
    return out


def test_unet_u2_sampler_full_chain_vs_golden(unet_sampler_kat, cuda_dev):
    """The headline network (U2, fp32) over a full T = 1000 chain with injected
    noise: <= 1e-4 rel-L2 against the spec at steps 1, 10, 100, 500, 1000."""
    xs = _run_golden_chain(unet_sampler_kat, "u2_fp32", cuda_dev)
    for k, x in xs.items():
        err = RN.rel_l2(x, unet_sampler_kat[f"u2_fp32_x{k}"].astype(np.float64))
        record_error(f"unet_sampler_U2_fp32_step{k}", err)
        assert err < SAMPLER_TOL, (k, err)


def test_unet_u2_b64_sampler_full_chain_vs_golden(cuda_dev):
    """configs[1] exactly -- U2, fp32, B = 64, L = 4693, random GroupNorm affine
    -- over a full T = 1000 chain with injected noise: the kernel dispatch the
    bench times (unsplit register-weight F(4x4) at every level), <= 1e-4 rel-L2
    against the spec at steps 1, 10, 100 and 1000
    (tests/golden/unet_sampler_b64_kat.npz)."""
    from conftest import load_golden
    kat = load_golden("unet_sampler_b64_kat.npz")
    xs = _run_golden_chain(kat, "u2_b64_aff", cuda_dev)
    for k, x in xs.items():
        err = RN.rel_l2(x, kat[f"u2_b64_aff_x{k}"].astype(np.float64))
        record_error(f"unet_sampler_U2_B64_aff_step{k}", err)
        assert err < SAMPLER_TOL, (k, err)


# The bf16 configs at their per-GPU bench batch (configs[2]: U3 B = 256;
# configs[4]: U5 B = 64) -- the tile counts, K splits and workgroup grids of the
# bench, which the B <= 2 golden chains do not reach -- over a 10-step chain
# (T = 10 schedule, injected noise) against the spec on members spread over the
# batch (the spec's members are independent: GroupNorm and attention are per
# sample, so the spec run on those members alone is the batch's reference).
BATCH_CASES = [("U3", "bf16", 256, 1001), ("U3", "bf16x3", 256, 1001),
               ("U5", "bf16", 64, 513), ("U5", "bf16x3", 64, 513), ("U5", "fp32", 64, 513)]
# 10 steps; per-forward budgets of test_unet_bf16_forward / test_unet_bf16x3_forward
BATCH_TOL = {"bf16": (1.2e-2, 1.6e-2), "bf16x3": (None, 1e-4), "fp32": (None, 1e-4)}


@pytest.mark.parametrize("name,precision,B,L", BATCH_CASES)
def test_unet_bench_batch_chain_vs_spec(name, precision, B, L, cuda_dev):
    cfg = U.CONFIGS[name]
    T = 10
    W = U.init_weights(cfg, 15, affine="random")
    m = _model_from_spec(name, W, cuda_dev, precision=precision)
    P = m.param_dim
    cond = torch.from_numpy(synth_uniform((B, 14, L), 161))
    noise = torch.from_numpy(synth_normal((T, B, P), 162))
    sched = ertdiff.get_diffusion_schedule(T, device=cuda_dev)
    xs = ertdiff.sample_model(m, cond.to(cuda_dev), T, *sched, P, cuda_dev, noise=noise.to(cuda_dev)).cpu()
    assert bool(torch.isfinite(xs).all())
    idx = [0, B // 2 + 1, B - 1]
    got = xs[idx].double().numpy()
    tol16, tol32 = BATCH_TOL[precision]
    with torch.no_grad():
        ref32 = U.sample(cond[idx], W, cfg, T, noise[:, idx])
        e32 = RN.rel_l2(got, ref32.double().numpy())
        record_error(f"unet_chain10_{name}_B{B}_{precision}_vs_fp32spec", e32)
        assert e32 < tol32, e32
        if tol16 is not None:
            ref16 = U.sample(cond[idx], W, cfg, T, noise[:, idx], bf16=True)
            e16 = RN.rel_l2(got, ref16.double().numpy())
            record_error(f"unet_chain10_{name}_B{B}_{precision}_vs_bf16spec", e16)
            assert e16 < tol16, e16


def test_unet_u3_bf16_sampler_full_chain_vs_golden(unet_sampler_kat, cuda_dev):
    """configs[2]'s network at bf16 operands over a full T = 1000 chain, against
    the bf16-operand spec and the fp32 spec (budgets BF16_SAMPLER_TOL)."""
    xs = _run_golden_chain(unet_sampler_kat, "u3_bf16", cuda_dev)
    for k, x in xs.items():
        e16 = RN.rel_l2(x, unet_sampler_kat[f"u3_bf16_x{k}"].astype(np.float64))
        e32 = RN.rel_l2(x, unet_sampler_kat[f"u3_fp32_x{k}"].astype(np.float64))
        record_error(f"unet_sampler_U3_bf16_vs_bf16spec_step{k}", e16)
        record_error(f"unet_sampler_U3_bf16_vs_fp32spec_step{k}", e32)
        assert e16 < BF16_SAMPLER_TOL["bf16_spec"], (k, e16)
        assert e32 < BF16_SAMPLER_TOL["fp32_spec"], (k, e32)


# split-bf16 operands (precision "bf16x3": hi + lo bf16 planes, three bf16
# MFMAs per product, fp32 accumulate) at the north star's output tolerance:
# the bf16 configs' networks over full T = 1000 chains against the FP32 spec.
BF16X3_SAMPLER_TOL = 1e-4


@pytest.mark.parametrize("key", ["u3_fp32", "u3_fp32_aff", "u5_fp32_aff"])
def test_unet_bf16x3_sampler_full_chain_vs_fp32_golden(key, unet_sampler_kat, cuda_dev):
    """configs[2] (U3) / configs[4] (U5) networks at split-bf16 operands over a
    full T = 1000 chain: <= 1e-4 rel-L2 vs the fp32 spec at every recorded step."""
    xs = _run_golden_chain(unet_sampler_kat, key, cuda_dev, precision="bf16x3")
    for k, x in xs.items():
        err = RN.rel_l2(x, unet_sampler_kat[f"{key}_x{k}"].astype(np.float64))
        record_error(f"unet_sampler_{key}_bf16x3_vs_fp32spec_step{k}", err)
        assert err < BF16X3_SAMPLER_TOL, (k, err)


def test_unet_u5_sampler_full_chain_vs_golden(unet_sampler_kat, cuda_dev):
    """configs[4]'s network (U5: 128x128, 4 levels, ch 128, mid attention; random
    GN affine) over a full T = 1000 chain: fp32 <= 1e-4 vs the fp32 spec; plain
    bf16 operands within the bf16 budget of the same spec."""
    key = "u5_fp32_aff"
    xs = _run_golden_chain(unet_sampler_kat, key, cuda_dev)
    for k, x in xs.items():
        err = RN.rel_l2(x, unet_sampler_kat[f"{key}_x{k}"].astype(np.float64))
        record_error(f"unet_sampler_U5_fp32_step{k}", err)
        assert err < SAMPLER_TOL, (k, err)
    xs = _run_golden_chain(unet_sampler_kat, key, cuda_dev, precision="bf16")
    for k, x in xs.items():
        err = RN.rel_l2(x, unet_sampler_kat[f"{key}_x{k}"].astype(np.float64))
        record_error(f"unet_sampler_U5_bf16_vs_fp32spec_step{k}", err)
        assert err < BF16_SAMPLER_TOL["fp32_spec"], (k, err)


def test_unet_u3_fp32_sampler_full_chain_vs_golden(unet_sampler_kat, cuda_dev):
    """U3 (mid attention) at fp32 over the same chain: <= 1e-4."""
    kat = unet_sampler_kat
    key = "u3_fp32"
    xs = _run_golden_chain(kat, key, cuda_dev)
    for k, x in xs.items():
        err = RN.rel_l2(x, kat[f"{key}_x{k}"].astype(np.float64))
        record_error(f"unet_sampler_U3_fp32_step{k}", err)
        assert err < SAMPLER_TOL, (k, err)


@pytest.mark.parametrize("key", ["u2_fp32_aff", "u3_fp32_aff"])
def test_unet_sampler_full_chain_random_affine_vs_golden(key, unet_sampler_kat, cuda_dev):
    """Full T = 1000 chains (U2; U3 with mid attention) whose GroupNorms carry
    random per-channel gamma/beta: <= 1e-4 at every recorded step."""
    xs = _run_golden_chain(unet_sampler_kat, key, cuda_dev)
    for k, x in xs.items():
        err = RN.rel_l2(x, unet_sampler_kat[f"{key}_x{k}"].astype(np.float64))
        record_error(f"unet_sampler_{key}_step{k}", err)
        assert err < SAMPLER_TOL, (k, err)


def test_unet_sampler_vs_oracle(cuda_dev):
    name, B, L, T = "U1", 2, 129, 10
    m, W = _pair(name, cuda_dev, seed=3)
    cfg = U.CONFIGS[name]
    cond = torch.from_numpy(synth_uniform((B, 14, L), 103))
    noise = torch.from_numpy(synth_normal((T, B, cfg.param_dim), 104))
    sched = ertdiff.get_diffusion_schedule(T, device=cuda_dev)
    xs = ertdiff.sample_model(m, cond.to(cuda_dev), T, *sched, cfg.param_dim, cuda_dev,
                              noise=noise.to(cuda_dev))
    xr = U.sample(cond, W, cfg, T, noise)
    err = RN.rel_l2(xs.cpu().double().numpy(), xr.double().numpy())
    assert err < 1e-4, err


@pytest.mark.parametrize("name,precision,T", [("U1", "fp32", 6), ("U2", "fp32", 3),
                                              ("U3", "bf16", 3), ("U5", "fp32", 2),
                                              ("U5", "bf16", 2), ("U3", "bf16x3", 3),
                                              ("U5", "bf16x3", 2)])
def test_unet_plan_matches_direct_and_deterministic(name, precision, T, cuda_dev):
    """The captured step graph (skip convs on a forked branch, fused bf16 GN
    prologue) equals the eagerly launched sampler bit for bit."""
    B, L = 2, 65
    m = ertdiff.ConditionalUNet.from_config(name, seed=4, precision=precision).to(cuda_dev).eval()
    cond = torch.from_numpy(synth_uniform((B, 14, L), 105)).to(cuda_dev)
    sched = ertdiff.get_diffusion_schedule(T, device=cuda_dev)
    P = m.param_dim
    a = ertdiff.sample_model(m, cond, T, *sched, P, cuda_dev, noise="philox", seed=9)
    b = ertdiff.sample_model(m, cond, T, *sched, P, cuda_dev, noise="philox", seed=9)
    assert torch.equal(a, b)
    plan = ertdiff.UNetSamplerPlan(m, cond, T, *sched, seed=9)
    plan.x.copy_(ertdiff.philox_normal(B, P, T, 1, 9, 0, cuda_dev))
    plan.launch()
    torch.cuda.synchronize()
    assert torch.equal(plan.x, a)
    plan.close()


def test_unet_member_sharding_invariance(cuda_dev):
    """Philox keyed by global member id: a 4-member run equals two 2-member runs."""
    name, L, T = "U1", 33, 4
    m, _ = _pair(name, cuda_dev, seed=5)
    cond = torch.from_numpy(synth_uniform((1, 14, L), 106)).to(cuda_dev)
    sched = ertdiff.get_diffusion_schedule(T, device=cuda_dev)
    P = m.param_dim
    full = ertdiff.sample_model(m, cond, T, *sched, P, cuda_dev, noise="philox", seed=2,
                                shared_condition=True, n_members=4)
    lo = ertdiff.sample_model(m, cond, T, *sched, P, cuda_dev, noise="philox", seed=2,
                              shared_condition=True, n_members=2)
    hi = ertdiff.sample_model(m, cond, T, *sched, P, cuda_dev, noise="philox", seed=2,
                              shared_condition=True, n_members=2, member_offset=2)
    assert torch.equal(full, torch.cat([lo, hi]))


def test_configs3_ensemble_1024_members_sharded(cuda_dev):
    """BASELINE configs[3]: ONE condition, 1024 U2 members sharded over 8
    GPUs by member_range (the reference's realisation loops,
    ERT_Conditional_Diffusion.py:398-410, :1052-1069), Philox keyed by the
    global member id.  On one device: the 1024-member shared-condition run
    (stride 0) is bitwise equal to the concatenation of the 8 member_range
    shards and to the run with the condition materialised per member (stride
    14 * L) -- i.e. what each rank computes is exactly its slice of the
    single-GPU ensemble.  T = 4 steps of the T = 1000 schedule."""
    from ertdiff.ensemble import member_range
    name, n, L, T, steps, world, seed = "U2", 1024, 4693, 1000, 4, 8, 77
    m = ertdiff.ConditionalUNet.from_config(name, seed=12).to(cuda_dev).eval()
    P = m.param_dim
    cond = torch.from_numpy(synth_uniform((1, 14, L), 151)).to(cuda_dev)
    sched = ertdiff.get_diffusion_schedule(T, device=cuda_dev)
    kw = dict(num_steps=steps, noise="philox", seed=seed)
    full = ertdiff.sample_model(m, cond, T, *sched, P, cuda_dev, shared_condition=True, n_members=n,
                                **kw)
    shards = []
    for r in range(world):
        lo, hi = member_range(n, world, r)
        shards.append(ertdiff.sample_model(m, cond, T, *sched, P, cuda_dev, shared_condition=True,
                                           n_members=hi - lo, member_offset=lo, **kw))
    assert torch.equal(full, torch.cat(shards))
    del shards
    mat = cond.expand(n, 14, L).contiguous()
    per = ertdiff.sample_model(m, mat, T, *sched, P, cuda_dev, **kw)
    assert torch.equal(full, per)
    assert bool(torch.isfinite(full).all())
    # the members differ (each its own Philox stream)
    assert float((full[0] - full[1]).abs().max()) > 0


@pytest.mark.parametrize("name,B,L,ts", [("U1", 3, 129, [0, 17, 999]), ("U3", 2, 257, [999, 5]),
                                         ("U5", 1, 129, [321])])
def test_unet_bf16_forward(name, B, L, ts, cuda_dev):
    """bf16 conv operands, fp32 accumulation: against the spec with the same
    bf16 rounding of conv inputs/weights, and against the fp32 spec (bf16 has
    8 significant bits; measured 0.85 % rel-L2 between the two specs)."""
    cfg = U.CONFIGS[name]
    m = ertdiff.ConditionalUNet.from_config(name, seed=0, precision="bf16").to(cuda_dev).eval()
    W = U.init_weights(cfg, 0)
    x = torch.from_numpy(synth_normal((B, cfg.param_dim), 111))
    cond = torch.from_numpy(synth_uniform((B, 14, L), 112))
    t = torch.tensor(ts)
    with torch.no_grad():      # bf16 has no backward: forward under autograd raises
        out = m(x.to(cuda_dev), t.to(cuda_dev), cond.to(cuda_dev)).cpu().double().numpy()
        ref16 = U.forward(x, t, cond, W, cfg, bf16=True).double().numpy()
        ref32 = U.forward(x, t, cond, W, cfg).double().numpy()
    e16, e32 = RN.rel_l2(out, ref16), RN.rel_l2(out, ref32)
    record_error(f"unet_forward_{name}_bf16_vs_bf16spec", e16)
    record_error(f"unet_forward_{name}_bf16_vs_fp32spec", e32)
    # ~20 chained bf16 roundings: two correct bf16 paths whose fp32 sums differ
    # only in order still drift apart by a fraction of the bf16-vs-fp32 gap
    # (rounding flips cascade); per-operator tightness is tested in
    # test_gpu_unet_ops.py.
    # measured 4.6e-3..6.0e-3 vs the bf16 spec, 6.4e-3..8.5e-3 vs fp32 (U1/U3/U5)
    assert e16 < 1.2e-2, e16
    assert e32 < 1.6e-2, e32


@pytest.mark.parametrize("name,B,L,ts", [("U1", 3, 129, [0, 17, 999]), ("U3", 2, 257, [999, 5]),
                                         ("U5", 1, 129, [321])])
def test_unet_bf16x3_forward(name, B, L, ts, cuda_dev):
    """Split-bf16 conv operands (hi + lo planes, three bf16 MFMAs per product,
    fp32 accumulate), random GN affine: against the FP32 spec <= 1e-4 rel-L2
    (the north star's output tolerance; plain bf16 sits at ~7e-3)."""
    cfg = U.CONFIGS[name]
    W = U.init_weights(cfg, 13, affine="random")
    m = _model_from_spec(name, W, cuda_dev, precision="bf16x3")
    x = torch.from_numpy(synth_normal((B, cfg.param_dim), 113))
    cond = torch.from_numpy(synth_uniform((B, 14, L), 114))
    t = torch.tensor(ts)
    with torch.no_grad():
        out = m(x.to(cuda_dev), t.to(cuda_dev), cond.to(cuda_dev)).cpu().double().numpy()
        ref32 = U.forward(x, t, cond, W, cfg).double().numpy()
    e32 = RN.rel_l2(out, ref32)
    record_error(f"unet_forward_{name}_bf16x3_vs_fp32spec", e32)
    assert e32 < 1e-4, e32
