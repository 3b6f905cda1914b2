"""Data contract and post-processing around the hot path (SURVEY.md 8a row a13,
8f rows 2-3).  These are host-side transforms the reference applies before
training and after sampling; they are not part of the device hot path.

  transform_to_unconstrained / inverse_transform   ERT_Conditional_Diffusion.py:26-53
  DiffusionDataset                                 :55-78
  check_param_bounds                               :183-218
  load_best_model / save_checkpoint                :345-353, :369-375
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch
from torch.utils.data import Dataset

_EPS = 1e-6


def transform_to_unconstrained(x, a, b):
    """[a,b] -> R logit with clamp eps=1e-6 (:26-40); tensor or ndarray."""
    if isinstance(x, torch.Tensor):
        xn = torch.clamp((x - a) / (b - a), min=_EPS, max=1 - _EPS)
        return torch.log(xn / (1 - xn))
    xn = np.clip((x - a) / (b - a), _EPS, 1 - _EPS)
    return np.log(xn / (1 - xn))


def inverse_transform(u, a, b):
    """Sigmoid back to [a,b] (:42-53); tensor or ndarray."""
    if isinstance(u, torch.Tensor):
        return a + (b - a) * torch.sigmoid(u)
    return a + (b - a) * (1 / (1 + np.exp(-u)))


class DiffusionDataset(Dataset):
    """(params (N,29[,1]), ert (N,4693,14)) -> (logit params (29,), cond (14,4693)).

    Same contract as the reference (:55-78).  ``a``/``b`` are explicit here
    (the reference reads module globals a, b = 0, 1 set at :230).  The
    condition is stored transposed as a view; default collation makes each
    batch a contiguous (B,14,L) tensor, which is what the kernels read.
    """

    def __init__(self, sim_param, ert_sim, a: float = 0.0, b: float = 1.0):
        if sim_param.ndim == 3 and sim_param.shape[2] == 1:
            raw = np.squeeze(sim_param, axis=2)
        else:
            raw = sim_param.copy()
        self.params = transform_to_unconstrained(torch.from_numpy(raw).float(), a, b)
        self.conditions = torch.from_numpy(np.transpose(ert_sim, (0, 2, 1))).float()

    def __len__(self):
        return self.params.shape[0]

    def __getitem__(self, idx):
        return self.params[idx], self.conditions[idx]


def bounds_mask(param: np.ndarray, limits: np.ndarray) -> np.ndarray:
    """Row validity of (n, P) parameter sets against (P, 2) [min, max] limits:
    rejected when some value is < min or > max (:205-207; a NaN passes)."""
    lo, hi = limits[:, 0], limits[:, 1]
    return ~np.any((param < lo) | (param > hi), axis=1)


def check_param_bounds(param: np.ndarray, limits: np.ndarray, verbose: bool = True) -> Optional[np.ndarray]:
    """Keep only parameter sets inside the limits (:183-218); None if none are."""
    mask = bounds_mask(param, limits)
    if verbose:
        lo, hi = limits[:, 0], limits[:, 1]
        for i in np.nonzero(~mask)[0]:
            bad = np.nonzero((param[i] < lo) | (param[i] > hi))[0][0]
            print(f"Sample {i} Parameter {bad}: {param[i, bad]:.4f} "
                  f"(out of bounds [{lo[bad]:.4f}, {hi[bad]:.4f}])")
    if not mask.any():
        return None
    return np.stack(list(param[mask]))


def save_checkpoint(path, model, optimizer, epoch: int, best_val_loss: float,
                    train_history, val_history, param_dim: int) -> None:
    """The reference's best-model dict format (:345-353)."""
    torch.save({
        "epoch": epoch,
        "model_state_dict": model.state_dict(),
        "optimizer_state_dict": optimizer.state_dict() if optimizer is not None else {},
        "best_val_loss": best_val_loss,
        "train_history": list(train_history),
        "val_history": list(val_history),
        "param_dim": param_dim,
    }, path)


def load_best_model(path, model, optimizer=None, map_location=None):
    """Restore model (+ optimizer) from a reference-format checkpoint (:369-375).
    Loaded with weights_only=True: the dict holds tensors, ints, floats, lists."""
    ckpt = torch.load(path, map_location=map_location, weights_only=True)
    model.load_state_dict(ckpt["model_state_dict"])
    if optimizer is not None and "optimizer_state_dict" in ckpt:
        optimizer.load_state_dict(ckpt["optimizer_state_dict"])
    print(f'Loaded best model from epoch {ckpt["epoch"]} with val loss {ckpt["best_val_loss"]:.6f}')
    return ckpt
