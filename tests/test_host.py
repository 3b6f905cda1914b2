"""Host-side logic of the product (CPU only): API surface, C-ABI exports,
schedule tables, data transforms, checkpoint format, loud failure off-GPU."""
import os
import re

import numpy as np
import pytest
import torch

import ertdiff
from ertdiff import _lib
from conftest import ROOT


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    hdr = open(os.path.join(ROOT, "include", "ertdiff.h")).read()
    declared = set(re.findall(r"\b(ertd_[a-z_0-9]+)\s*\(", hdr))
    assert declared, "no entry points parsed from include/ertdiff.h"
    for name in sorted(declared):
        assert hasattr(lib, name), f"{name} declared in ertdiff.h but not exported"
    assert declared == set(_lib.SIGNATURES), "ctypes bindings out of sync with the header"


def test_library_host_queries():
    lib = _lib.load()
    assert lib.ertd_version() >= 1
    assert lib.ertd_packed_floats() > 0
    assert lib.ertd_error_string(-1).decode().startswith("invalid argument")
    assert lib.ertd_workspace_bytes(0, 4693, 29, 10, 1) == 0
    n64 = lib.ertd_workspace_bytes(64, 4693, 29, 1000, _lib.OP_SAMPLE)
    # partial pool sums: 64 members x 19 strips x 64 channels + U + V + cond_emb
    assert n64 >= 4 * (64 * 19 * 64 + 64 * 128 + 1000 * 128 + 64 * 128)
    assert lib.ertd_workspace_bytes(64, 4693, 29, 0, _lib.OP_FORWARD) < n64


def test_invalid_args_rejected_before_launch():
    lib = _lib.load()
    w = _lib.ErtdWeights()  # null pointers
    assert lib.ertd_pack_weights(w, None, None) == _lib.ERTD_EINVAL
    assert lib.ertd_q_sample(None, None, None, None, 4, 29, None, None) == _lib.ERTD_EINVAL
    assert lib.ertd_philox_normal(1, 0, 0, 29, 0, 0, None, None) == _lib.ERTD_EINVAL


def test_state_dict_and_init_match_reference(golden_weights):
    torch.manual_seed(42)
    m = ertdiff.ConditionalDiffusionModel(param_dim=29, hidden_dim=128)
    sd = m.state_dict()
    assert list(sd.keys()) == list(golden_weights.keys()) == ertdiff.STATE_KEYS
    for k, v in golden_weights.items():
        assert np.array_equal(sd[k].numpy(), v), k
    assert sum(p.numel() for p in m.parameters()) == 72765
    # Adam indexes parameters by position: same order as the reference module
    assert [n for n, _ in m.named_parameters()] == ertdiff.STATE_KEYS


def test_no_cpu_fallback(golden_weights):
    m = ertdiff.ConditionalDiffusionModel(29, 128)
    x = torch.zeros(2, 29)
    t = torch.zeros(2, dtype=torch.long)
    c = torch.zeros(2, 14, 50)
    with torch.no_grad(), pytest.raises(RuntimeError, match="gfx950"):
        m(x, t, c)
    with pytest.raises(RuntimeError, match="gfx950"):
        ertdiff.get_timestep_embedding(t, 128)
    with pytest.raises(RuntimeError, match="gfx950"):
        ertdiff.q_sample(x, t, x, torch.ones(10))
    b, a, ab = ertdiff.get_diffusion_schedule(10)
    with pytest.raises(RuntimeError, match="gfx950"):
        ertdiff.sample_model(m, c, 10, b, a, ab, 29, "cpu")


@pytest.mark.parametrize("T", [50, 500, 1000])
def test_schedule_and_step_tables(T, sched_kat):
    b, a, ab = ertdiff.get_diffusion_schedule(T, beta_start=1e-4, beta_end=0.02)
    assert np.array_equal(b.numpy(), sched_kat[f"T{T}_betas"])
    assert np.array_equal(ab.numpy(), sched_kat[f"T{T}_alpha_bar"])
    tab = ertdiff.step_tables(b, a, ab, T, temperature=1.0).numpy()
    assert np.array_equal(tab[0], sched_kat[f"T{T}_c1"].astype(np.float32))
    assert np.array_equal(tab[1], sched_kat[f"T{T}_c2"])
    assert np.array_equal(tab[2], sched_kat[f"T{T}_sigma"].astype(np.float32))


def test_update_rule_fp32_semantics(sched_kat):
    """The device update c1*(x - c2*eps) + sigma*z with float32 c1/sigma (one
    rounding per op) reproduces torch's scalar arithmetic bit for bit."""
    import math
    rng = np.random.default_rng(0)
    x = rng.standard_normal((64, 29)).astype(np.float32)
    eps = rng.standard_normal((64, 29)).astype(np.float32)
    z = rng.standard_normal((64, 29)).astype(np.float32)
    b, a, ab = ertdiff.get_diffusion_schedule(1000)
    tab = ertdiff.step_tables(b, a, ab, 1000, temperature=0.7).numpy()
    for t_ in (999, 500, 1):
        coef = (1 - a[t_]) / (math.sqrt(1 - ab[t_]) + 1e-8)
        ref = (1.0 / math.sqrt(a[t_])) * (torch.from_numpy(x) - coef * torch.from_numpy(eps))
        ref = ref + math.sqrt(b[t_]) * 0.7 * torch.from_numpy(z)
        c1, c2, sg = (np.float32(v) for v in tab[:, t_])
        got = c1 * (x - c2 * eps) + sg * z  # numpy float32: one rounding per op
        assert np.array_equal(got, ref.numpy())


def test_freq_table_matches_reference_expression(fwd_kat):
    f = ertdiff.schedule._freq_cpu(128)
    t = torch.from_numpy(fwd_kat["temb_t"])
    emb = torch.cat([torch.sin(t.float()[:, None] * f[None]), torch.cos(t.float()[:, None] * f[None])], 1)
    assert torch.equal(emb, torch.from_numpy(fwd_kat["temb_dim128"]))


def test_transforms_and_bounds(postproc_kat):
    k = postproc_kat
    assert np.array_equal(ertdiff.transform_to_unconstrained(k["x"], 0.0, 1.0), k["unc"])
    assert np.array_equal(ertdiff.inverse_transform(k["unc"], 0.0, 1.0), k["inv"])
    xt = torch.from_numpy(k["xt"])
    assert torch.equal(ertdiff.transform_to_unconstrained(xt, 0.0, 1.0), torch.from_numpy(k["unc_t"]))
    assert torch.equal(ertdiff.inverse_transform(torch.from_numpy(k["unc_t"]), 0.0, 1.0),
                       torch.from_numpy(k["inv_t"]))
    valid = ertdiff.check_param_bounds(k["sets"], k["limits"], verbose=False)
    assert np.array_equal(valid, k["valid"])
    assert ertdiff.check_param_bounds(k["sets"][~k["mask"]], k["limits"], verbose=False) is None


def test_dataset_contract():
    rng = np.random.default_rng(3)
    params = rng.uniform(0, 1, (5, 29, 1))
    ert = rng.uniform(0, 1, (5, 4693, 14)).astype(np.float32)
    ds = ertdiff.DiffusionDataset(params, ert)
    x0, c = ds[2]
    assert x0.shape == (29,) and c.shape == (14, 4693)
    assert torch.equal(c, torch.from_numpy(ert[2].T.copy()))
    batch = torch.utils.data.default_collate([ds[i] for i in range(3)])
    assert batch[1].is_contiguous() and batch[1].shape == (3, 14, 4693)


def test_checkpoint_roundtrip(tmp_path):
    torch.manual_seed(0)
    m = ertdiff.ConditionalDiffusionModel(29)
    opt = torch.optim.Adam(m.parameters(), lr=1e-4)
    path = tmp_path / "best_model.pt"
    ertdiff.save_checkpoint(path, m, opt, epoch=3, best_val_loss=0.25, train_history=[1.0, 0.5],
                            val_history=[0.9, 0.25], param_dim=29)
    m2 = ertdiff.ConditionalDiffusionModel(29)
    opt2 = torch.optim.Adam(m2.parameters(), lr=1e-4)
    ck = ertdiff.load_best_model(path, m2, opt2)
    assert set(ck) == {"epoch", "model_state_dict", "optimizer_state_dict", "best_val_loss",
                       "train_history", "val_history", "param_dim"}
    for k, v in m.state_dict().items():
        assert torch.equal(v, m2.state_dict()[k])


@pytest.mark.parametrize("name", ["U1", "U2", "U3", "U5"])
def test_unet_layout_matches_spec(name):
    """The library's U-Net parameter enumeration (state_dict order and
    shapes) and the module's init equal the specification
    (oracle/unet_torch.py, build-defined: parity unpinned vs the reference)."""
    from oracle import unet_torch as U
    m = ertdiff.ConditionalUNet.from_config(name, seed=0)
    spec = [(n, tuple(s)) for n, s in U.layer_shapes(U.CONFIGS[name])]
    assert [(k, tuple(v.shape)) for k, v in m.state_dict().items()] == spec
    W = U.init_weights(U.CONFIGS[name], 0)
    assert all(torch.equal(W[k], v) for k, v in m.state_dict().items())


def test_unet_host_queries_and_errors():
    import ctypes
    from ertdiff.unet import make_config
    lib = _lib.load()
    good = make_config(64, 64, (1, 2, 4), 2, False)
    assert lib.ertd_unet_packed_floats(ctypes.byref(good)) > 14_000_000
    assert lib.ertd_unet_workspace_bytes(ctypes.byref(good), 2, 4693) > 0
    for bad in (make_config(48, 64, (1, 2, 4)),            # not a power of two
                make_config(64, 64, (1, 2, 4, 8, 8)[:4]),  # 8x8 level
                make_config(64, 64, (1, 2), attn=True),    # attention needs 16x16
                make_config(64, 48, (1, 2, 4))):           # channels % groups
        assert lib.ertd_unet_n_params(ctypes.byref(bad)) == _lib.ERTD_EINVAL
        assert lib.ertd_unet_packed_floats(ctypes.byref(bad)) == 0
    assert lib.ertd_unet_forward(ctypes.byref(good), None, None, None, None, 0, 1, 1, None, None,
                                 None, 0, None) == _lib.ERTD_EINVAL


def test_unet_forward_raises_off_gpu():
    m = ertdiff.ConditionalUNet.from_config("U1", seed=0)
    with pytest.raises(RuntimeError):
        m(torch.zeros(1, 1024), torch.zeros(1, dtype=torch.long), torch.zeros(1, 14, 9))


@pytest.mark.parametrize("name", ["U1", "U3"])
def test_unet_flop_count_matches_torch(name):
    """bench.py's algorithmic FLOP per sample-step equals torch's FlopCounter
    on the spec module."""
    from torch.utils.flop_counter import FlopCounterMode
    from oracle import unet_torch as U
    from ertdiff.unet import CONFIGS, unet_flops
    cfg = U.CONFIGS[name]
    W = U.init_weights(cfg, 0)
    with FlopCounterMode(display=False) as fc:
        U.forward(torch.randn(1, cfg.param_dim), torch.tensor([3]), torch.rand(1, 14, 97), W, cfg)
    enc_97 = 2 * 14 * 3 * 32 * 49 + 2 * 32 * 3 * 64 * 25 + 2 * 64 * 128  # encoder at L=97
    f = unet_flops(**CONFIGS[name])
    assert f["total"] - f["condition_encoder"] + enc_97 == fc.get_total_flops()


def test_unet_sampler_rejects_conflicting_options():
    """sample_model on a ConditionalUNet raises (before any device work) when
    asked for a precision the model does not run or a reference-model mode,
    instead of silently ignoring them."""
    m = ertdiff.ConditionalUNet.from_config("U1", seed=0)
    sched = ertdiff.get_diffusion_schedule(4)
    cond = torch.zeros(1, 14, 9)
    with pytest.raises(RuntimeError, match="precision"):
        ertdiff.sample_model(m, cond, 4, *sched, 1024, "cpu", precision="bf16")
    with pytest.raises(RuntimeError, match="mode"):
        ertdiff.sample_model(m, cond, 4, *sched, 1024, "cpu", mode="faithful")


def test_unet_sampler_golden_fixture_shape(unet_sampler_kat):
    """tests/golden/unet_sampler_kat.npz (make_unet_golden.py): the full T = 1000
    chains the GPU tests replay; the bf16-operand spec stays within 2e-3 of the
    fp32 spec at every recorded step (the budget's basis)."""
    kat = unet_sampler_kat
    assert int(kat["T"]) == 1000 and list(kat["record"]) == [1, 10, 100, 500, 1000]
    for r in kat["record"]:
        a = kat[f"u3_bf16_x{r}"].astype(np.float64)
        b = kat[f"u3_fp32_x{r}"].astype(np.float64)
        assert np.isfinite(a).all() and np.isfinite(b).all()
        assert np.linalg.norm(a - b) / np.linalg.norm(b) < 2e-3


def test_shipped_library_has_no_diagnostic_variants():
    """The wrong-result ablation variants (ERTD_*_DBG knobs) and every schedule
    A/B knob exist only in a diagnostic build (-DERTD_DIAG, csrc/unet.h
    ERTD_KNOB): the shipped library reads no ERTD_* environment variable, so
    an inherited variable cannot move it onto an untested path.  (ERTD_LIB_PATH
    is read by the Python loader, not by the library.)"""
    data = open(_lib.LIB_PATH, "rb").read()
    names = sorted(set(re.findall(rb"ERTD_[A-Z0-9_]{2,}", data)))
    assert names == [], names
    assert b"getenv" not in data
    src = open(os.path.join(ROOT, "ert-conditional-diffusion-model_amd", "ertdiff", "unet_train.py")).read()
    assert "environ" not in src


def test_conv2d_workspace_covers_launch_scratch():
    """ertd_conv2d allocates nothing: its workspace query includes the K-split
    partial of a Winograd layer with fewer tile items than CUs and the bf16
    pre-transformed input image (caller-owned, include/ertdiff.h)."""
    lib = _lib.load()
    fp32, bf16 = _lib.PREC_FP32, _lib.PREC_BF16
    # 256 -> 256 at 16x16, B = 32: 128 register-weight F(4x4) tile items fill half
    # of 256 CUs -> K split (at B = 64 the same kernel has 256 items and no split)
    small = lib.ertd_conv2d_workspace_bytes(256, 256, 3, fp32, 64, 16, 0)
    split = lib.ertd_conv2d_workspace_bytes(256, 256, 3, fp32, 32, 16, 0)
    assert split >= 32 * 256 * 16 * 16 * 4
    assert split > small - 64 * 256 * 16 * 16 * 4     # the B = 64 layer needs no split buffer
    # bf16 3x3 stride-1 conv: the [B][C/16][H][W][16] bf16 image (C*H*W*2 bytes per sample)
    img = lib.ertd_conv2d_workspace_bytes(64, 64, 3, bf16, 8, 64, 0)
    assert img >= 8 * 64 * 64 * 64 * 2
    assert lib.ertd_conv2d_workspace_bytes(64, 64, 3, fp32, 0, 64, 0) == 0      # B < 1
    assert lib.ertd_conv2d_workspace_bytes(64, 64, 1, fp32, 2, 64, 1) == 0      # 1x1 stride 2
    assert lib.ertd_mse_loss_ws_bytes() >= 8
    assert lib.ertd_mse_loss(None, None, 4, None, None, None, 0, None) == _lib.ERTD_EINVAL


def test_bf16_unet_under_autograd_raises():
    """A bf16-operand U-Net has no backward: forward under autograd raises a
    RuntimeError that says so (before any device work) instead of returning
    a tensor that silently does not require grad."""
    m = ertdiff.ConditionalUNet.from_config("U1", seed=0, precision="bf16")
    x, t, c = torch.zeros(1, 1024), torch.zeros(1, dtype=torch.long), torch.zeros(1, 14, 9)
    with pytest.raises(RuntimeError, match="no backward"):
        m(x, t, c)
    with torch.no_grad():          # inference goes on to the device path (and raises off-GPU)
        with pytest.raises(RuntimeError, match="(?!no backward)"):
            m(x, t, c)


def test_sample_ensemble_gather_is_explicit():
    """sample_ensemble(gather=...) has no default (round 2 changed it from
    True to False, which silently changed the return shape at N > 1)."""
    from ertdiff.ensemble import sample_ensemble
    with pytest.raises(TypeError):
        sample_ensemble(None, torch.zeros(14, 5), 4, 10, None, None, None, seed=0,
                        device=torch.device("cpu"), _sampler=lambda *a, **k: None)


def test_unet_spec_random_affine_init():
    """oracle init_weights(affine="random"): distinct per-channel GroupNorm
    gamma/beta, every other tensor identical to the default init."""
    from oracle import unet_torch as U
    cfg = U.CONFIGS["U1"]
    a, r = U.init_weights(cfg, 3), U.init_weights(cfg, 3, affine="random")
    for k in a:
        if ".norm" in k or k.startswith("norm_out"):
            assert not torch.equal(a[k], r[k]) and r[k].unique().numel() == r[k].numel(), k
        else:
            assert torch.equal(a[k], r[k]), k
