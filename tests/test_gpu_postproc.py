"""Device post-processing (ertd_postprocess) against the reference chain's
golden outputs and the numpy oracle."""
import numpy as np
import pytest
import torch

import ertdiff
from oracle import ref_numpy as RN

pytestmark = pytest.mark.gpu


def test_postprocess_vs_golden(postproc_chain_kat, cuda_dev):
    k = postproc_chain_kat
    u = torch.from_numpy(k["u"]).to(cuda_dev)
    out, valid = ertdiff.postprocess(u, (k["min_"], k["scale_"]), k["limits"])
    out = out.cpu().numpy()
    # error in units of each feature's data range; the mask is exact
    err = np.abs(out.astype(np.float64) - k["out"]) * k["scale_"]
    assert err.max() <= 2.0 ** -22, err.max()
    assert np.array_equal(valid.cpu().numpy(), k["mask"])
    kept = ertdiff.compact(out, valid)
    for r, rows in enumerate(kept):
        assert (0 if rows is None else len(rows)) == int(k["n_valid"][r])


def test_postprocess_vs_oracle_large(postproc_chain_kat, cuda_dev):
    """Ragged row count (not a multiple of the 8 rows per block), P=29 and a
    NaN row (passes the bounds check, as in the reference)."""
    k = postproc_chain_kat
    rng = np.random.default_rng(5)
    u = (rng.standard_normal((1001, 29)) * 3).astype(np.float32)
    u[17] = 0.0  # mid-range: inside every limit
    u[17, 4] = np.nan
    out, valid = ertdiff.postprocess(torch.from_numpy(u).to(cuda_dev), (k["min_"], k["scale_"]),
                                     k["limits"])
    ro, rm = RN.postprocess_chain(u, k["min_"], k["scale_"], k["limits"])
    out = out.cpu().numpy()
    fin = np.isfinite(ro)
    assert np.array_equal(np.isfinite(out), fin)
    err = np.abs(out[fin].astype(np.float64) - ro[fin]) * np.broadcast_to(k["scale_"], ro.shape)[fin]
    assert err.max() <= 2.0 ** -22
    assert np.array_equal(valid.cpu().numpy(), rm)
    assert bool(valid[17])  # NaN passes check_param_bounds (:205)


def test_postprocess_small_param_dim(cuda_dev):
    P = 5
    u = torch.linspace(-8, 8, 3 * P).reshape(3, P).to(cuda_dev)
    mn = np.zeros(P)
    sc = np.ones(P) * 2.0
    lim = np.stack([np.zeros(P), np.full(P, 0.25)], 1)
    out, valid = ertdiff.postprocess(u, (mn, sc), lim)
    ro, rm = RN.postprocess_chain(u.cpu().numpy(), mn, sc, lim)
    np.testing.assert_array_equal(out.cpu().numpy(), ro)
    assert np.array_equal(valid.cpu().numpy(), rm)


def test_sample_realisations(gpu_model, postproc_chain_kat, cuda_dev):
    k = postproc_chain_kat
    from synth import synth_uniform
    cond = torch.from_numpy(synth_uniform((4, 14, 257), 81)).to(cuda_dev)
    T = 12
    sched = ertdiff.get_diffusion_schedule(T, device=cuda_dev)
    params, valid, unc = ertdiff.sample_realisations(
        gpu_model, cond, 3, T, *sched, 29, cuda_dev, (k["min_"], k["scale_"]), k["limits"],
        noise="philox", seed=7, mode="faithful")
    assert params.shape == (3, 4, 29) and valid.shape == (3, 4)
    for r in range(3):
        x = ertdiff.sample_model(gpu_model, cond, T, *sched, 29, cuda_dev, noise="philox",
                                 seed=7, member_offset=4 * r, mode="faithful")
        assert torch.equal(x, unc[r])
        o, m = ertdiff.postprocess(x, (k["min_"], k["scale_"]), k["limits"])
        assert torch.equal(o, params[r]) and torch.equal(m, valid[r])
    # the n_samples x B members as ONE launch: the same bits
    pb, vb, ub = ertdiff.sample_realisations(
        gpu_model, cond, 3, T, *sched, 29, cuda_dev, (k["min_"], k["scale_"]), k["limits"],
        noise="philox", seed=7, mode="faithful", batched=True)
    assert torch.equal(ub, unc) and torch.equal(pb, params) and torch.equal(vb, valid)


@pytest.mark.parametrize("mode", ["hoisted", "faithful", "faithful_steps"])
def test_sample_conditions_one_launch(gpu_model, mode, cuda_dev):
    """The test-set evaluation (ERT_Conditional_Diffusion.py:1042-1069): every
    condition x n_samples realisations as ONE sampler launch
    (ertd_sample_conditions) == the per-realisation sample_model loop with
    member ids r * N + c, bit for bit, in every schedule; and the condition
    slices a sharded run gives each rank ([0, 2) and [2, 5) of N = 5, condition
    offset + id period N) concatenate to the same array."""
    from synth import synth_uniform
    N, ns, T = 5, 3, 9
    cond = torch.from_numpy(synth_uniform((N, 14, 301), 83)).to(cuda_dev)
    sched = ertdiff.get_diffusion_schedule(T, device=cuda_dev)
    full = ertdiff.sample_conditions(gpu_model, cond, ns, T, *sched, 29, cuda_dev, mode=mode, seed=11)
    assert full.shape == (ns, N, 29)
    for r in range(ns):
        x = ertdiff.sample_model(gpu_model, cond, T, *sched, 29, cuda_dev, noise="philox", seed=11,
                                 member_offset=r * N, mode=mode)
        assert torch.equal(x, full[r]), r
    parts = [ertdiff.sample_conditions(gpu_model, cond[c0:c1].contiguous(), ns, T, *sched, 29, cuda_dev,
                                       mode=mode, seed=11, cond_offset=c0, n_conditions_total=N)
             for c0, c1 in ((0, 2), (2, 5))]
    assert torch.equal(torch.cat(parts, 1), full)
    assert float((full[0] - full[1]).abs().max()) > 0     # realisations differ
