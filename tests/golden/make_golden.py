"""Generate the golden vectors that pin the oracle and the HIP path.

Runs ONLY in the build container, where the reference checkout is mounted at
/root/reference.  It parses ERT_Conditional_Diffusion.py, keeps the top-level
function/class definitions that precede the script's data-loading cell
(reference lines 26-218: transforms, DiffusionDataset, get_timestep_embedding,
get_diffusion_schedule, q_sample, sample_model, ConditionalDiffusionModel,
mode_kde_calculation, check_param_bounds) and executes just those definitions
in a fresh namespace.  The module-level script (np.load of private datasets,
500-epoch training, PFLOTRAN runs) is never executed.  Generate_ERT_utils is
imported normally for ParameterLimits.

Only numeric arrays are written (tests/golden/*.npz); nothing derived from the
reference's source text is stored.  Usage:

    python tests/golden/make_golden.py [--ref /root/reference]
"""
from __future__ import annotations

import argparse
import ast
import math
import os
import sys

import numpy as np
import torch
import torch.nn as nn
from torch.utils.data import Dataset

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from synth import synth_normal, synth_timesteps, synth_uniform  # noqa: E402

L_FULL = 4693
P = 29


def load_reference(ref_dir: str) -> dict:
    path = os.path.join(ref_dir, "ERT_Conditional_Diffusion.py")
    with open(path) as f:
        tree = ast.parse(f.read(), filename=path)
    keep = [n for n in tree.body
            if isinstance(n, (ast.FunctionDef, ast.ClassDef)) and n.lineno < 220]
    mod = ast.Module(body=keep, type_ignores=[])
    ns = {"torch": torch, "nn": nn, "math": math, "np": np, "Dataset": Dataset,
          "a": 0.0, "b": 1.0, "__name__": "ert_reference_defs"}
    exec(compile(mod, path, "exec"), ns)
    return ns


def state_np(model) -> dict:
    return {k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items()}


def make_weights(ref):
    torch.manual_seed(42)
    model = ref["ConditionalDiffusionModel"](param_dim=P, hidden_dim=128)
    return model


def gen_forward(ref, out_dir):
    model = make_weights(ref).eval()
    res = {}
    cases = {
        "full": dict(B=4, L=L_FULL, t=[0, 1, 499, 999], xs=11, cs=12),
        "short": dict(B=3, L=37, t=[5, 0, 42], xs=13, cs=14),
        "tiny": dict(B=2, L=1, t=[3, 7], xs=15, cs=16),
        "odd": dict(B=5, L=250, t=[10, 20, 30, 40, 49], xs=17, cs=18),
    }
    for name, c in cases.items():
        x = torch.from_numpy(synth_normal((c["B"], P), c["xs"]))
        cond = torch.from_numpy(synth_uniform((c["B"], 14, c["L"]), c["cs"]))
        t = torch.tensor(c["t"], dtype=torch.long)
        with torch.no_grad():
            out = model(x, t, cond)
            cemb = model.condition_encoder(cond)
            traw = ref["get_timestep_embedding"](t, 128)
            temb = model.time_embed(traw)
        res[f"{name}_x"] = x.numpy()
        res[f"{name}_t"] = t.numpy()
        res[f"{name}_L"] = np.array(c["L"])
        res[f"{name}_xs"] = np.array(c["xs"])
        res[f"{name}_cs"] = np.array(c["cs"])
        res[f"{name}_out"] = out.numpy()
        res[f"{name}_cond_emb"] = cemb.numpy()
        res[f"{name}_t_raw"] = traw.numpy()
        res[f"{name}_t_emb"] = temb.numpy()
    # timestep embedding standalone, odd dimension (zero pad branch)
    tt = torch.tensor([0, 1, 2, 17, 499, 999, 12345], dtype=torch.long)
    res["temb_t"] = tt.numpy()
    for dim in (7, 128, 33):
        res[f"temb_dim{dim}"] = ref["get_timestep_embedding"](tt, dim).numpy()
    np.savez_compressed(os.path.join(out_dir, "forward_kat.npz"), **res)
    np.savez_compressed(os.path.join(out_dir, "weights_seed42.npz"), **state_np(model))


def sched_tables(ref, T, temperature=1.0):
    betas, alphas, alpha_bar = ref["get_diffusion_schedule"](T, beta_start=1e-4, beta_end=0.02)
    c1, c2, sig = [], [], []
    for t_ in range(T):
        alpha_t = alphas[t_]
        alpha_bar_t = alpha_bar[t_]
        coef = (1 - alpha_t) / (math.sqrt(1 - alpha_bar_t) + 1e-8)
        c1.append(1.0 / math.sqrt(alpha_t))
        c2.append(float(coef))
        sig.append(math.sqrt(betas[t_]) * temperature)
    return (betas.numpy(), alphas.numpy(), alpha_bar.numpy(),
            np.array(c1, np.float64), np.array(c2, np.float32), np.array(sig, np.float64))


def gen_schedule(ref, out_dir):
    res = {}
    for T in (50, 500, 1000):
        b, a, ab, c1, c2, s = sched_tables(ref, T)
        res.update({f"T{T}_betas": b, f"T{T}_alphas": a, f"T{T}_alpha_bar": ab,
                    f"T{T}_c1": c1, f"T{T}_c2": c2, f"T{T}_sigma": s})
    np.savez_compressed(os.path.join(out_dir, "schedule.npz"), **res)


def capture_sampler(ref, model, cond, T, seed, num_steps=None, temperature=1.0, eps_steps=()):
    """Run the reference sample_model, then replay its RNG draws to record the
    noise it consumed, and re-run the loop with injected noise to capture eps."""
    betas, alphas, alpha_bar = ref["get_diffusion_schedule"](T)
    B = cond.shape[0]
    n = T if num_steps is None else num_steps
    torch.manual_seed(seed)
    out = ref["sample_model"](model, cond, T, betas, alphas, alpha_bar, P, "cpu",
                              num_steps=num_steps, temperature=temperature)
    torch.manual_seed(seed)
    draws = [torch.randn(B, P)]
    x_like = draws[0]
    for t_ in reversed(range(n)):
        if t_ > 0:
            draws.append(torch.randn_like(x_like))
    noise = torch.stack(draws)  # [n, B, P]: draw 0 = x_T, draw k = z for t = n-k
    # replay with injected noise (must be bit-identical to `out`)
    eps = {}
    with torch.no_grad():
        x = noise[0].clone()
        for t_ in reversed(range(n)):
            tt = torch.full((B,), t_, dtype=torch.long)
            pred = model(x, tt, cond)
            if t_ in eps_steps:
                eps[t_] = pred.numpy().copy()
            alpha_t = alphas[t_]
            alpha_bar_t = alpha_bar[t_]
            coef = (1 - alpha_t) / (math.sqrt(1 - alpha_bar_t) + 1e-8)
            x = (1.0 / math.sqrt(alpha_t)) * (x - coef * pred)
            if t_ > 0:
                x = x + math.sqrt(betas[t_]) * temperature * noise[n - t_]
    assert torch.equal(x, out), "noise replay is not bit-identical to sample_model"
    return out.numpy(), noise.numpy(), eps


def gen_sampler(ref, out_dir):
    model = make_weights(ref).eval()
    res = {}
    cond = torch.from_numpy(synth_uniform((8, 14, L_FULL), 21))
    out, noise, eps = capture_sampler(ref, model, cond, 50, 1234, eps_steps=(49, 25, 0))
    res.update({"r1_out": out, "r1_noise": noise, "r1_cs": np.array(21), "r1_T": np.array(50),
                "r1_eps49": eps[49], "r1_eps25": eps[25], "r1_eps0": eps[0]})
    cond2 = torch.from_numpy(synth_uniform((3, 14, L_FULL), 22))
    out2, noise2, _ = capture_sampler(ref, model, cond2, 50, 99, num_steps=20, temperature=0.5)
    res.update({"trunc_out": out2, "trunc_noise": noise2, "trunc_cs": np.array(22),
                "trunc_T": np.array(50), "trunc_num_steps": np.array(20),
                "trunc_temperature": np.array(0.5)})
    np.savez_compressed(os.path.join(out_dir, "sampler_kat.npz"), **res)


def gen_train(ref, out_dir):
    model = make_weights(ref)
    model.train()
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    crit = nn.MSELoss()
    T = 500
    _, _, alpha_bar = ref["get_diffusion_schedule"](T)
    B = 8
    x0 = torch.from_numpy(synth_normal((B, P), 31) * np.float32(2.0))
    cond = torch.from_numpy(synth_uniform((B, 14, L_FULL), 32))
    res = {"x0": x0.numpy(), "cs": np.array(32), "T": np.array(T)}
    names = [k for k, _ in model.named_parameters()]
    for step in range(3):
        t = torch.from_numpy(synth_timesteps(B, T, 40 + step))
        noise = torch.from_numpy(synth_normal((B, P), 50 + step))
        x_noisy = ref["q_sample"](x0, t, noise, alpha_bar)
        pred = model(x_noisy, t, cond)
        loss = crit(pred, noise)
        opt.zero_grad()
        loss.backward()
        if step == 0:
            res["x_noisy0"] = x_noisy.detach().numpy()
            res["pred0"] = pred.detach().numpy()
            for k, p in model.named_parameters():
                res[f"grad0/{k}"] = p.grad.numpy().copy()
        opt.step()
        res[f"t{step}"] = t.numpy()
        res[f"noise{step}"] = noise.numpy()
        res[f"loss{step}"] = np.array(loss.item(), np.float32)
        if step in (0, 2):
            for k, p in model.named_parameters():
                res[f"param{step}/{k}"] = p.detach().numpy().copy()
    res["param_names"] = np.array(names)
    np.savez_compressed(os.path.join(out_dir, "train_kat.npz"), **res)


def gen_postproc(ref, ref_dir, out_dir):
    sys.path.insert(0, ref_dir)
    import Generate_ERT_utils as ert_utils  # importable: see SURVEY.md 8c
    limits = np.asarray(ert_utils.ParameterLimits().plims, dtype=np.float64)
    x = synth_uniform((6, P), 61).astype(np.float64)
    unc = ref["transform_to_unconstrained"](x, 0.0, 1.0)
    inv = ref["inverse_transform"](unc, 0.0, 1.0)
    xt = torch.from_numpy(synth_uniform((6, P), 62))
    unc_t = ref["transform_to_unconstrained"](xt, 0.0, 1.0)
    inv_t = ref["inverse_transform"](unc_t, 0.0, 1.0)
    # a parameter set straddling the limits for check_param_bounds
    lo, hi = limits[:, 0], limits[:, 1]
    u = synth_uniform((10, P), 63).astype(np.float64)
    sets = lo + (hi - lo) * (u * 1.2 - 0.1)
    sets[0] = lo + (hi - lo) * 0.5
    sets[1] = lo + (hi - lo) * 0.25
    import contextlib, io
    with contextlib.redirect_stdout(io.StringIO()):
        valid = ref["check_param_bounds"](sets, limits)
    mask = np.array([bool(np.all((s >= lo) & (s <= hi))) for s in sets])
    np.savez_compressed(os.path.join(out_dir, "postproc_kat.npz"),
                        limits=limits, x=x, unc=unc, inv=inv, xt=xt.numpy(),
                        unc_t=unc_t.numpy(), inv_t=inv_t.numpy(), sets=sets,
                        valid=np.zeros((0, P)) if valid is None else valid, mask=mask)


def gen_postproc_chain(ref, ref_dir, out_dir):
    """The reference's whole post-sampling chain (:398-410, :1054-1064):
    inverse_transform on a float32 tensor (torch.sigmoid), .numpy(),
    MinMaxScaler.inverse_transform (float64 min_/scale_ applied in place to the
    float32 array), check_param_bounds.  The scaler is fitted, as at :232-234,
    on a synthetic (N, 29) physical-unit table that overshoots the
    ParameterLimits by 1 % on each side so the bounds check rejects some rows."""
    sys.path.insert(0, ref_dir)
    import Generate_ERT_utils as ert_utils
    from sklearn.preprocessing import MinMaxScaler
    limits = np.asarray(ert_utils.ParameterLimits().plims, dtype=np.float64)
    lo, hi = limits[:, 0], limits[:, 1]
    table = lo + (hi - lo) * (synth_uniform((400, P), 71).astype(np.float64) * 1.02 - 0.01)
    scaler = MinMaxScaler(feature_range=(0.0, 1.0))
    scaler.fit(table)
    R, B = 3, 16
    u = synth_normal((R, B, P), 72) * np.float32(2.5)
    u[0, 0, :3] = [30.0, -30.0, 0.0]        # saturated sigmoid -> data_max / data_min
    out = np.zeros((R, B, P), np.float32)
    mask = np.zeros((R, B), bool)
    n_valid = np.zeros(R, np.int64)
    import contextlib, io
    for r in range(R):
        x = ref["inverse_transform"](torch.from_numpy(u[r]), 0.0, 1.0).numpy()
        x = scaler.inverse_transform(x)
        assert x.dtype == np.float32
        out[r] = x
        mask[r] = [not any((v < mn) or (v > mx) for v, (mn, mx) in zip(row, limits)) for row in x]
        with contextlib.redirect_stdout(io.StringIO()):
            valid = ref["check_param_bounds"](x, limits)
        n_valid[r] = 0 if valid is None else len(valid)
        assert n_valid[r] == mask[r].sum()
        if valid is not None:
            assert np.array_equal(valid, x[mask[r]])
    np.savez_compressed(os.path.join(out_dir, "postproc_chain_kat.npz"), limits=limits,
                        data_min=scaler.data_min_, data_max=scaler.data_max_,
                        min_=scaler.min_, scale_=scaler.scale_, u=u, out=out, mask=mask,
                        n_valid=n_valid)


def kde_ensemble(n=40, cells=48):
    """Synthetic ensemble (n, cells): per-cell location/scale spread over a
    wide global range, every 4th cell bimodal, every 6th log-normal (skewed)."""
    z = synth_normal((n, cells), 81).astype(np.float64)
    u = synth_uniform((3, cells), 82).astype(np.float64)
    loc = 40.0 * u[0] - 20.0
    scale = 0.05 + 3.0 * u[1]
    x = loc + scale * z
    for c in range(0, cells, 4):
        x[: n // 2, c] += 6.0 * scale[c]
    for c in range(1, cells, 6):
        x[:, c] = loc[c] + np.exp(0.8 * z[:, c])
    return x


def gen_kde(ref, out_dir):
    """KDE mode (:166-181 mode_kde_calculation, called as the reference defines
    it; :747-762 the ensemble-mode loop, restated around scipy's
    gaussian_kde, the reference's dependency -- scipy 1.15.3 here)."""
    from scipy import stats
    ref["stats"] = stats          # the reference's `from scipy import stats` (its import cell)
    x = kde_ensemble()
    grid = 5000
    x_range = np.linspace(np.min(x), np.max(x), grid)
    idx = np.array([int(np.argmax(stats.gaussian_kde(x[:, c])(x_range))) for c in range(x.shape[1])])
    arrays = x[:, :8].T.copy()
    modes = np.array([ref["mode_kde_calculation"](a) for a in arrays], dtype=np.float64)
    arr_idx = np.array([int(np.argmin(np.abs(np.linspace(a.min(), a.max(), 1000) - m)))
                        for a, m in zip(arrays, modes)])
    for a, m, k in zip(arrays, modes, arr_idx):
        assert np.linspace(a.min(), a.max(), 1000)[k] == m
    np.savez_compressed(os.path.join(out_dir, "kde_kat.npz"), x=x, grid=grid,
                        lo=np.min(x), hi=np.max(x), idx_global=idx, mode_global=x_range[idx],
                        arrays=arrays, mode_arrays=modes, idx_arrays=arr_idx)


GENERATORS = ("forward", "schedule", "sampler", "train", "postproc", "postproc_chain", "kde")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default=HERE)
    ap.add_argument("--only", nargs="*", choices=GENERATORS, default=list(GENERATORS))
    args = ap.parse_args()
    torch.set_num_threads(8)
    ref = load_reference(args.ref)
    if "forward" in args.only:
        gen_forward(ref, args.out)
    if "schedule" in args.only:
        gen_schedule(ref, args.out)
    if "sampler" in args.only:
        gen_sampler(ref, args.out)
    if "train" in args.only:
        gen_train(ref, args.out)
    if "postproc" in args.only:
        gen_postproc(ref, args.ref, args.out)
    if "postproc_chain" in args.only:
        gen_postproc_chain(ref, args.ref, args.out)
    if "kde" in args.only:
        gen_kde(ref, args.out)
    for f in sorted(os.listdir(args.out)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(args.out, f)))


if __name__ == "__main__":
    main()
