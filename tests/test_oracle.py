"""Pin the oracle against the golden vectors generated from the reference
(tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest
import torch

from oracle import ref_numpy as RN
from oracle import ref_torch as RT
from synth import synth_uniform


def _tw(golden_weights):
    return {k: torch.from_numpy(v) for k, v in golden_weights.items()}


@pytest.mark.parametrize("case", ["full", "short", "tiny", "odd"])
def test_torch_oracle_forward_bitexact(case, fwd_kat, golden_weights):
    W = _tw(golden_weights)
    x = torch.from_numpy(fwd_kat[f"{case}_x"])
    t = torch.from_numpy(fwd_kat[f"{case}_t"])
    L = int(fwd_kat[f"{case}_L"])
    cond = torch.from_numpy(synth_uniform((x.shape[0], 14, L), int(fwd_kat[f"{case}_cs"])))
    assert torch.equal(RT.forward(x, t, cond, W), torch.from_numpy(fwd_kat[f"{case}_out"]))
    assert torch.equal(RT.encoder(cond, W), torch.from_numpy(fwd_kat[f"{case}_cond_emb"]))
    assert torch.equal(RT.time_mlp(t, W), torch.from_numpy(fwd_kat[f"{case}_t_emb"]))


@pytest.mark.parametrize("case", ["full", "short", "tiny", "odd"])
def test_numpy_oracle_forward(case, fwd_kat, golden_weights):
    x = fwd_kat[f"{case}_x"]
    t = fwd_kat[f"{case}_t"]
    L = int(fwd_kat[f"{case}_L"])
    cond = synth_uniform((x.shape[0], 14, L), int(fwd_kat[f"{case}_cs"]))
    f = RN.forward_full(x, t, cond, golden_weights)
    # fp64 truth vs the reference's fp32 arithmetic (fp32 sin/cos of t*f at t=999 dominates)
    assert RN.rel_l2(f["out"], fwd_kat[f"{case}_out"]) < 1e-5
    assert RN.rel_l2(f["cond_emb"], fwd_kat[f"{case}_cond_emb"]) < 1e-6


@pytest.mark.parametrize("dim", [7, 33, 128])
def test_timestep_embedding(dim, fwd_kat):
    t = torch.from_numpy(fwd_kat["temb_t"])
    assert torch.equal(RT.timestep_embedding(t, dim), torch.from_numpy(fwd_kat[f"temb_dim{dim}"]))
    ref = fwd_kat[f"temb_dim{dim}"].astype(np.float64)
    got = RN.timestep_embedding(fwd_kat["temb_t"], dim)
    assert np.max(np.abs(got - ref)) < 2e-3  # fp32 argument rounding at t=12345


@pytest.mark.parametrize("T", [50, 500, 1000])
def test_schedule_tables(T, sched_kat):
    b, a, ab = RT.diffusion_schedule(T)
    assert torch.equal(b, torch.from_numpy(sched_kat[f"T{T}_betas"]))
    assert torch.equal(a, torch.from_numpy(sched_kat[f"T{T}_alphas"]))
    assert torch.equal(ab, torch.from_numpy(sched_kat[f"T{T}_alpha_bar"]))
    c1, c2, sg = RT.step_tables(b, a, ab)
    assert np.array_equal(np.array(c1), sched_kat[f"T{T}_c1"])
    assert np.array_equal(np.array(c2, np.float32), sched_kat[f"T{T}_c2"])
    assert np.array_equal(np.array(sg), sched_kat[f"T{T}_sigma"])


def test_torch_oracle_sampler_bitexact(sampler_kat, golden_weights):
    W = _tw(golden_weights)
    cond = torch.from_numpy(synth_uniform((8, 14, 4693), int(sampler_kat["r1_cs"])))
    noise = torch.from_numpy(sampler_kat["r1_noise"])
    assert torch.equal(RT.sample(cond, W, 50, noise), torch.from_numpy(sampler_kat["r1_out"]))
    # hoisting the t-invariant encoder is bit-identical on CPU too
    assert torch.equal(RT.sample(cond, W, 50, noise, encoder_every_step=False),
                       torch.from_numpy(sampler_kat["r1_out"]))
    cond2 = torch.from_numpy(synth_uniform((3, 14, 4693), int(sampler_kat["trunc_cs"])))
    out2 = RT.sample(cond2, W, 50, torch.from_numpy(sampler_kat["trunc_noise"]),
                     num_steps=int(sampler_kat["trunc_num_steps"]),
                     temperature=float(sampler_kat["trunc_temperature"]))
    assert torch.equal(out2, torch.from_numpy(sampler_kat["trunc_out"]))


def test_numpy_oracle_sampler(sampler_kat, golden_weights):
    cond = synth_uniform((8, 14, 4693), int(sampler_kat["r1_cs"]))
    x = RN.sample(cond, golden_weights, 50, sampler_kat["r1_noise"])
    assert RN.rel_l2(x, sampler_kat["r1_out"]) < 1e-5


def test_torch_oracle_train_bitexact(train_kat, golden_weights):
    W = _tw(golden_weights)
    cond = torch.from_numpy(synth_uniform((8, 14, 4693), int(train_kat["cs"])))
    ts = [torch.from_numpy(train_kat[f"t{i}"]) for i in range(3)]
    ns = [torch.from_numpy(train_kat[f"noise{i}"]) for i in range(3)]
    losses, g0, p = RT.train_steps(W, torch.from_numpy(train_kat["x0"]), cond, 500, ts, ns)
    assert losses == [float(train_kat[f"loss{i}"]) for i in range(3)]
    for k in W:
        assert torch.equal(g0[k], torch.from_numpy(train_kat[f"grad0/{k}"])), k
        assert torch.equal(p[k], torch.from_numpy(train_kat[f"param2/{k}"])), k


def test_numpy_oracle_train(train_kat, golden_weights):
    cond = synth_uniform((8, 14, 4693), int(train_kat["cs"]))
    ts = [train_kat[f"t{i}"] for i in range(3)]
    ns = [train_kat[f"noise{i}"] for i in range(3)]
    losses, g0, p = RN.train_steps(golden_weights, train_kat["x0"], cond, 500, ts, ns)
    for i in range(3):
        assert abs(losses[i] - float(train_kat[f"loss{i}"])) < 1e-6 * abs(losses[i]) + 1e-7
    for k in golden_weights:
        assert RN.rel_l2(g0[k], train_kat[f"grad0/{k}"]) < 1e-4, k
        d_ref = train_kat[f"param2/{k}"].astype(np.float64) - golden_weights[k]
        assert RN.rel_l2(p[k] - golden_weights[k], d_ref) < 1e-3, k


def test_postproc(postproc_kat):
    k = postproc_kat
    assert np.array_equal(RN.transform_to_unconstrained(k["x"], 0.0, 1.0), k["unc"])
    np.testing.assert_allclose(RN.inverse_transform(k["unc"], 0.0, 1.0), k["inv"], rtol=0, atol=1e-15)
    mask = RN.bounds_mask(k["sets"], k["limits"])
    assert np.array_equal(mask, k["mask"])
    assert np.array_equal(k["sets"][mask], k["valid"])


def test_philox_known_answers():
    """Random123 Philox4x32-10 known-answer vectors pin the numpy port."""
    from oracle.philox import philox4x32_10
    out = [int(v) for v in philox4x32_10(0, 0, 0, 0, 0, 0)]
    assert out == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    f = 0xFFFFFFFF
    out = [int(v) for v in philox4x32_10(f, f, f, f, f, f)]
    assert out == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    out = [int(v) for v in philox4x32_10(0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344,
                                         0xA4093822, 0x299F31D0)]
    assert out == [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_postproc_chain_oracle(postproc_chain_kat):
    """The numpy restatement of the post-sampling chain reproduces the
    reference chain (torch sigmoid -> sklearn MinMaxScaler -> check_param_bounds)."""
    k = postproc_chain_kat
    R = k["u"].shape[0]
    for r in range(R):
        out, mask = RN.postprocess_chain(k["u"][r], k["min_"], k["scale_"], k["limits"])
        # error in units of each feature's data range (x - min_ cancels near
        # the range ends, so a 1-ulp sigmoid difference is not 1 ulp of out)
        err = np.abs(out.astype(np.float64) - k["out"][r]) * k["scale_"]
        assert err.max() <= 2.0 ** -22, err.max()
        assert np.array_equal(mask, k["mask"][r])
        assert mask.sum() == k["n_valid"][r]
