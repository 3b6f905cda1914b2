"""HIP path vs the oracle / golden vectors (needs an MI355X).

Tolerances: fp32 forward <= 1e-5 rel-L2, fp32 T-step sampler
<= 1e-4 rel-L2 (north star).  bf16 operands (R3/R5; not pinned by the
reference, which cannot run bf16): the encoder against a float64 oracle with
the kernel's own bf16 roundings <= 1e-5 (FWD_TOL), and the T = 1000 sampler
output against the fp32 sampler <= 1e-4 (BF16_TOL, SURVEY.md 8c's bf16 gate)."""
import numpy as np
import pytest
import torch

import ertdiff
from ertdiff import _lib
from oracle import ref_numpy as RN
from synth import synth_normal, synth_uniform
from conftest import record_error

pytestmark = pytest.mark.gpu

FWD_TOL = 1e-5
SAMPLER_TOL = 1e-4
BF16_TOL = 1e-4


def rel(a, b):
    a = a.detach().double().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a, np.float64)
    return RN.rel_l2(a, b)


@pytest.mark.parametrize("case", ["full", "short", "tiny", "odd"])
def test_forward_vs_golden(case, gpu_model, fwd_kat, cuda_dev):
    x = torch.from_numpy(fwd_kat[f"{case}_x"]).to(cuda_dev)
    t = torch.from_numpy(fwd_kat[f"{case}_t"]).to(cuda_dev)
    L = int(fwd_kat[f"{case}_L"])
    cond = torch.from_numpy(synth_uniform((x.shape[0], 14, L), int(fwd_kat[f"{case}_cs"]))).to(cuda_dev)
    with torch.no_grad():
        out, cemb, temb = gpu_model(x, t, cond, return_intermediates=True)
    torch.cuda.synchronize()
    assert rel(cemb, fwd_kat[f"{case}_cond_emb"]) < FWD_TOL
    assert rel(temb, fwd_kat[f"{case}_t_emb"]) < FWD_TOL
    assert rel(out, fwd_kat[f"{case}_out"]) < FWD_TOL


def test_encoder_vs_fp64_oracle(gpu_model, golden_weights, cuda_dev):
    """Full-size encoder at B=16, L=4693 against the float64 oracle."""
    cond_np = synth_uniform((16, 14, 4693), 77)
    cemb = gpu_model.encode_condition(torch.from_numpy(cond_np).to(cuda_dev))
    ref = RN.encoder(cond_np, golden_weights)
    assert rel(cemb, ref) < 2e-6


@pytest.mark.parametrize("L", [1, 2, 3, 4, 5, 7, 9, 13, 251, 252, 253, 254, 255, 500, 4693, 5000])
def test_encoder_ragged_lengths(L, gpu_model, golden_weights, cuda_dev):
    """Strip boundaries / zero padding at every residue of L mod 4 and across strips."""
    cond_np = synth_uniform((3, 14, L), 1000 + L)
    cemb = gpu_model.encode_condition(torch.from_numpy(cond_np).to(cuda_dev))
    assert rel(cemb, RN.encoder(cond_np, golden_weights)) < 2e-6


@pytest.mark.parametrize("dim", [7, 33, 128])
def test_timestep_embedding_vs_golden(dim, fwd_kat, cuda_dev):
    t = torch.from_numpy(fwd_kat["temb_t"]).to(cuda_dev)
    e = ertdiff.get_timestep_embedding(t, dim).cpu().numpy()
    ref = fwd_kat[f"temb_dim{dim}"]
    assert e.shape == ref.shape
    assert np.max(np.abs(e - ref)) < 2e-6  # sin/cos of the same fp32 argument, ulp-level


def test_q_sample_one_ulp(cuda_dev):
    """torch's CPU sqrt (the reference's) is not correctly rounded -- it is 1 ulp
    off np.sqrt on some inputs -- while the device sqrt is; so the bound is 1 ulp."""
    b, a, ab = ertdiff.get_diffusion_schedule(500)
    x0 = torch.from_numpy(synth_normal((64, 29), 5))
    n = torch.from_numpy(synth_normal((64, 29), 6))
    t = torch.arange(64, dtype=torch.long) * 7 % 500
    ref = torch.sqrt(ab[t]).unsqueeze(1) * x0 + torch.sqrt(1 - ab[t]).unsqueeze(1) * n
    got = ertdiff.q_sample(x0.to(cuda_dev), t.to(cuda_dev), n.to(cuda_dev), ab.to(cuda_dev))
    # one ulp of either product (the sqrt factors may differ by 1 ulp), plus the final rounding
    mag = (torch.sqrt(ab[t]).unsqueeze(1) * x0).abs() + (torch.sqrt(1 - ab[t]).unsqueeze(1) * n).abs()
    assert ((got.cpu() - ref).abs() <= 2 * torch.finfo(torch.float32).eps * mag).all()


def _sched(T, dev):
    return ertdiff.get_diffusion_schedule(T, device=dev)


@pytest.mark.parametrize("mode", ["hoisted", "faithful", "faithful_steps"])
def test_sampler_vs_golden(mode, gpu_model, sampler_kat, cuda_dev):
    cond = torch.from_numpy(synth_uniform((8, 14, 4693), int(sampler_kat["r1_cs"]))).to(cuda_dev)
    noise = torch.from_numpy(sampler_kat["r1_noise"]).to(cuda_dev)
    x = ertdiff.sample_model(gpu_model, cond, 50, *_sched(50, cuda_dev), 29, cuda_dev,
                             mode=mode, noise=noise)
    assert rel(x, sampler_kat["r1_out"]) < SAMPLER_TOL


def test_sampler_truncated_temperature(gpu_model, sampler_kat, cuda_dev):
    cond = torch.from_numpy(synth_uniform((3, 14, 4693), int(sampler_kat["trunc_cs"]))).to(cuda_dev)
    noise = torch.from_numpy(sampler_kat["trunc_noise"]).to(cuda_dev)
    x = ertdiff.sample_model(gpu_model, cond, 50, *_sched(50, cuda_dev), 29, cuda_dev,
                             num_steps=int(sampler_kat["trunc_num_steps"]),
                             temperature=float(sampler_kat["trunc_temperature"]), noise=noise)
    assert rel(x, sampler_kat["trunc_out"]) < SAMPLER_TOL


def test_faithful_equals_hoisted_bitwise(gpu_model, cuda_dev):
    cond = torch.from_numpy(synth_uniform((16, 14, 4693), 91)).to(cuda_dev)
    sched = _sched(200, cuda_dev)
    xs = [ertdiff.sample_model(gpu_model, cond, 200, *sched, 29, cuda_dev, mode=m,
                               noise="philox", seed=1234)
          for m in ("hoisted", "faithful", "faithful_steps")]
    assert torch.equal(xs[0], xs[1]) and torch.equal(xs[0], xs[2])
    assert torch.isfinite(xs[0]).all()


@pytest.mark.parametrize("B,L,T", [(1, 1, 3), (3, 37, 20), (5, 250, 17), (2, 4694, 9),
                                   (7, 1003, 40), (40, 4693, 12), (4, 2600, 35)])
def test_faithful_schedules_bitwise(B, L, T, gpu_model, cuda_dev):
    """The persistent chain (ring of 16 slots: T > 16 wraps it; work items of
    two strips, the last one a single strip when S is odd), the per-step
    schedule and the hoisted sampler agree bit for bit on ragged shapes, with
    injected (reference-order) noise."""
    cond = torch.from_numpy(synth_uniform((B, 14, L), 500 + L)).to(cuda_dev)
    noise = torch.from_numpy(synth_normal((T, B, 29), 600 + B)).to(cuda_dev)
    sched = _sched(T, cuda_dev)
    xs = {m: ertdiff.sample_model(gpu_model, cond, T, *sched, 29, cuda_dev, mode=m, noise=noise)
          for m in ("faithful", "faithful_steps", "hoisted")}
    assert torch.equal(xs["faithful"], xs["faithful_steps"])
    assert torch.equal(xs["faithful"], xs["hoisted"])
    assert torch.isfinite(xs["faithful"]).all()


def test_faithful_chain_shared_condition(gpu_model, cuda_dev):
    cond1 = torch.from_numpy(synth_uniform((1, 14, 4693), 97)).to(cuda_dev)
    sched = _sched(30, cuda_dev)
    a = ertdiff.sample_model(gpu_model, cond1, 30, *sched, 29, cuda_dev, noise="philox", seed=8,
                             shared_condition=True, n_members=24, mode="faithful")
    b = ertdiff.sample_model(gpu_model, cond1, 30, *sched, 29, cuda_dev, noise="philox", seed=8,
                             shared_condition=True, n_members=24, mode="hoisted")
    assert torch.equal(a, b)


def test_faithful_chain_status_and_rerun(gpu_model, cuda_dev):
    """Plan replays re-zero the chain's counters and granules every call."""
    cond = torch.from_numpy(synth_uniform((8, 14, 4693), 98)).to(cuda_dev)
    sched = _sched(40, cuda_dev)
    x0 = ertdiff.philox_normal(8, 29, 40, 1, 4, 0, cuda_dev)
    p = ertdiff.SamplerPlan(gpu_model, cond, 40, *sched, mode="faithful", seed=4)
    outs = []
    for _ in range(3):
        p.x.copy_(x0)
        p.launch()
        assert p.status() == 0
        outs.append(p.x.clone())
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    ref = ertdiff.sample_model(gpu_model, cond, 40, *sched, 29, cuda_dev, mode="hoisted",
                               noise="philox", seed=4)
    assert torch.equal(outs[0], ref)


def test_deterministic_rerun(gpu_model, cuda_dev):
    cond = torch.from_numpy(synth_uniform((8, 14, 4693), 92)).to(cuda_dev)
    sched = _sched(100, cuda_dev)
    a = ertdiff.sample_model(gpu_model, cond, 100, *sched, 29, cuda_dev, noise="philox", seed=5,
                             mode="faithful")
    b = ertdiff.sample_model(gpu_model, cond, 100, *sched, 29, cuda_dev, noise="philox", seed=5,
                             mode="faithful")
    assert torch.equal(a, b)


def test_member_sharding_invariance(gpu_model, cuda_dev):
    """Members keyed by global id: splitting an ensemble into shards (what each
    GPU of a node runs) reproduces the unsplit result bit for bit."""
    cond1 = torch.from_numpy(synth_uniform((1, 14, 4693), 93)).to(cuda_dev)
    sched = _sched(100, cuda_dev)
    full = ertdiff.sample_model(gpu_model, cond1, 100, *sched, 29, cuda_dev, noise="philox",
                                seed=77, shared_condition=True, n_members=16)
    parts = [ertdiff.sample_model(gpu_model, cond1, 100, *sched, 29, cuda_dev, noise="philox",
                                  seed=77, shared_condition=True, n_members=n, member_offset=o)
             for o, n in ((0, 5), (5, 3), (8, 8))]
    assert torch.equal(torch.cat(parts), full)
    # shared condition read in place == the condition materialised per member
    rep = ertdiff.sample_model(gpu_model, cond1.expand(16, 14, 4693).contiguous(), 100, *sched, 29,
                               cuda_dev, noise="philox", seed=77)
    assert torch.equal(rep, full)


def test_philox_stream(cuda_dev):
    z = ertdiff.philox_normal(4096, 29, 3, 0, 11, 0, cuda_dev).double().cpu().numpy()
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1) < 0.01
    z2 = ertdiff.philox_normal(100, 29, 3, 0, 11, 4000, cuda_dev).cpu().numpy()
    assert np.array_equal(z2[:96], z[4000:4096].astype(np.float32))
    from oracle.philox import philox_normal_np
    ref = philox_normal_np(11, np.arange(64), 3, 0, 29)
    assert np.max(np.abs(z[:64] - ref)) < 1e-5


def test_graph_plan_matches_direct(gpu_model, cuda_dev):
    cond = torch.from_numpy(synth_uniform((8, 14, 4693), 94)).to(cuda_dev)
    sched = _sched(60, cuda_dev)
    x0 = ertdiff.philox_normal(8, 29, 60, 1, 3, 0, cuda_dev)
    for mode in ("faithful", "faithful_steps", "hoisted"):
        # the chain split into two graph segments == one direct call
        pa = ertdiff.SamplerPlan(gpu_model, cond, 60, *sched, t_first=59, n_run=25, mode=mode, seed=3)
        pb = ertdiff.SamplerPlan(gpu_model, cond, 60, *sched, t_first=34, n_run=35, mode=mode, seed=3)
        pa.x.copy_(x0)
        pa.launch()
        pb.x.copy_(pa.x)
        pb.launch()
        ref = ertdiff.sample_model(gpu_model, cond, 60, *sched, 29, cuda_dev, mode=mode,
                                   noise="philox", seed=3)
        torch.cuda.synchronize()
        assert torch.equal(pb.x, ref), mode


def test_full_size_r2_properties(gpu_model, cuda_dev):
    """BASELINE config 2 shape (B=64, T=1000): finite, deterministic, hoisted ==
    faithful bitwise, and the first 3 steps (injected noise) agree with the
    float64 oracle at the fp32 forward tolerance."""
    cond_np = synth_uniform((64, 14, 4693), 95)
    cond = torch.from_numpy(cond_np).to(cuda_dev)
    sched = _sched(1000, cuda_dev)
    xh = ertdiff.sample_model(gpu_model, cond, 1000, *sched, 29, cuda_dev, noise="philox", seed=9)
    xf = ertdiff.sample_model(gpu_model, cond, 1000, *sched, 29, cuda_dev, noise="philox", seed=9,
                              mode="faithful")
    assert torch.equal(xh, xf) and torch.isfinite(xh).all()
    # first steps of the same chain: num_steps = 1000, stopped after 3 reverse steps
    noise = synth_normal((1000, 64, 29), 97)
    plan = ertdiff.SamplerPlan(gpu_model, cond, 1000, *sched, t_first=999, n_run=3, mode="faithful",
                               noise=torch.from_numpy(noise).to(cuda_dev))
    plan.x.copy_(torch.from_numpy(noise[0]).to(cuda_dev))
    plan.launch()
    torch.cuda.synchronize()
    W = {k: v.detach().cpu().double().numpy() for k, v in gpu_model.state_dict().items()}
    ref = RN.sample(cond_np, W, 1000, noise, max_steps=3)
    err = rel(plan.x, ref)
    record_error("R2_first3_steps_vs_fp64", err)
    assert err < FWD_TOL, err


def _bf16(a):
    """RNE bf16 rounding of a float64/float32 array, back to float64."""
    return torch.from_numpy(np.asarray(a, np.float32)).bfloat16().double().numpy()


def encoder_bf16_oracle(cond, W):
    """The bf16-operand encoder (enc_bf16_kernel) in float64: cond, conv
    weights and the conv1 activation rounded to bf16, everything else exact."""
    w = {k: np.asarray(v, np.float64) for k, v in W.items()}
    h = np.maximum(RN.conv1d_s2(_bf16(cond), _bf16(w["condition_encoder.0.weight"]),
                                w["condition_encoder.0.bias"])[0], 0)
    h = np.maximum(RN.conv1d_s2(_bf16(h), _bf16(w["condition_encoder.2.weight"]),
                                w["condition_encoder.2.bias"])[0], 0)
    m = h.mean(axis=2)
    return np.maximum(m @ w["condition_encoder.6.weight"].T + w["condition_encoder.6.bias"], 0)


def test_bf16_encoder_tolerance(gpu_model, golden_weights, cuda_dev):
    """bf16 operands, fp32 accumulation: <= FWD_TOL against the float64 oracle
    with the same bf16 roundings; the bf16-vs-fp32 gap itself is recorded."""
    cond_np = synth_uniform((16, 14, 4693), 96)
    cond = torch.from_numpy(cond_np).to(cuda_dev)
    gpu_model.precision = "bf16"
    try:
        cemb = gpu_model.encode_condition(cond)
    finally:
        gpu_model.precision = "fp32"
    e16 = rel(cemb, encoder_bf16_oracle(cond_np, golden_weights))
    e32 = rel(cemb, RN.encoder(cond_np, golden_weights))
    record_error("R_encoder_bf16_vs_bf16oracle", e16)
    record_error("R_encoder_bf16_vs_fp64oracle", e32)
    assert e16 < FWD_TOL, e16
    assert e32 < 1e-2, e32


def test_bf16_sampler_budget(gpu_model, cuda_dev):
    """R3's precision (bf16 encoder operands, fp32 MLP and state) over a full
    T = 1000 chain: the output within BF16_TOL of the fp32 chain (same Philox
    noise) -- SURVEY.md 8c's bf16 gate, measured 1.9e-5 there."""
    cond = torch.from_numpy(synth_uniform((8, 14, 4693), 98)).to(cuda_dev)
    sched = _sched(1000, cuda_dev)
    x32 = ertdiff.sample_model(gpu_model, cond, 1000, *sched, 29, cuda_dev, noise="philox", seed=11)
    x16 = ertdiff.sample_model(gpu_model, cond, 1000, *sched, 29, cuda_dev, noise="philox", seed=11,
                               precision="bf16")
    err = rel(x16, x32.double().cpu().numpy())
    record_error("R3_bf16_sampler_vs_fp32_T1000", err)
    assert err < BF16_TOL, err
