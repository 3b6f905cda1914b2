"""Ensemble KDE mode on the device.

The reference reduces an ensemble to its per-cell mode with one
scipy.stats.gaussian_kde per cell (ERT_Conditional_Diffusion.py:747-762:
65,702 KDEs over sim_data (n, 4693, 14), each evaluated on a 5000-point
linspace of the ensemble's global range) and with mode_kde_calculation
(:166-181, one array, its own range, 1000 points).  Here one kernel
(`ertd_kde_mode`, csrc/kde.hip) evaluates every cell's KDE in float64 with
scipy's formula and summation order and takes the first maximum.

    mode_kde_calculation(array)             -> float (reference name and behaviour)
    ensemble_mode(sim_data, grid=5000)      -> (cells...) modes over the global range
    kde_mode(x, grid, lo=None, hi=None, per_cell=False) -> (mode, index, density)
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch

from . import _lib

SINGULAR_MSG = ("The data appears to lie in a lower-dimensional subspace of the space in which "
                "it is expressed. This has resulted in a singular data covariance matrix, which "
                "cannot be treated using the algorithms implemented in `gaussian_kde`.")


def _as_device_f64(x, device) -> torch.Tensor:
    if isinstance(x, np.ndarray):
        dev = torch.device(device) if device is not None else torch.device("cuda", 0)
        t = torch.from_numpy(np.ascontiguousarray(x, dtype=np.float64)).to(dev)
    else:
        t = x if device is None else x.to(device)
        t = t.to(torch.float64)
    _lib.require_device(t)
    return t.contiguous()


def kde_mode(x, grid: int = 5000, lo: Optional[float] = None, hi: Optional[float] = None,
             per_cell: bool = False, device=None,
             raise_singular: bool = True) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """x: (n, *cells) ensemble (float64; float32/numpy promoted) on a gfx950
    device.  Grid = np.linspace(lo, hi, grid) with lo/hi the global min/max of
    x unless given (computed on the device), or each cell's own min/max when
    per_cell.  Returns (mode, index, density) shaped like x.shape[1:]."""
    t = _as_device_f64(x, device)
    if t.dim() < 2:
        raise ValueError("kde_mode expects (n, *cells); use mode_kde_calculation for one array")
    n = t.shape[0]
    cell_shape = tuple(t.shape[1:])
    cells = int(np.prod(cell_shape))
    dev = t.device
    mode = torch.empty(cell_shape, dtype=torch.float64, device=dev)
    index = torch.empty(cell_shape, dtype=torch.int32, device=dev)
    density = torch.empty(cell_shape, dtype=torch.float64, device=dev)
    lib = _lib.lib()
    rng = torch.empty(2, dtype=torch.float64, device=dev)
    with torch.cuda.device(dev):
        s = _lib.stream_of(dev)
        if per_cell:
            range_mode, lo_v, hi_v = 1, 0.0, 0.0
        elif lo is not None and hi is not None:
            range_mode, lo_v, hi_v = 0, float(lo), float(hi)
        else:
            work = torch.empty(2 * 1024, dtype=torch.float64, device=dev)
            _lib.check(lib.ertd_minmax_f64(t.data_ptr(), t.numel(), work.data_ptr(),
                                           rng.data_ptr(), s), "minmax")
            if lo is not None or hi is not None:   # one end given: host round trip
                r = rng.cpu().numpy()
                lo_v = float(lo) if lo is not None else float(r[0])
                hi_v = float(hi) if hi is not None else float(r[1])
                range_mode = 0
            else:
                range_mode, lo_v, hi_v = 2, 0.0, 0.0
        _lib.check(lib.ertd_kde_mode(t.data_ptr(), n, cells, cells, int(grid), range_mode, lo_v,
                                     hi_v, rng.data_ptr(), mode.data_ptr(), index.data_ptr(),
                                     density.data_ptr(), s), "kde_mode")
    if raise_singular and bool((index < 0).any()):
        raise np.linalg.LinAlgError(SINGULAR_MSG)
    return mode, index, density


def ensemble_mode(sim_data, grid: int = 5000, device=None) -> torch.Tensor:
    """The reference's ensemble_mode (:747-762): per-cell KDE mode of
    sim_data (n, *cells) over np.linspace(min(sim_data), max(sim_data), grid)."""
    return kde_mode(sim_data, grid=grid, device=device)[0]


def mode_kde_calculation(array, device=None) -> float:
    """Reference :166-181: the mode of one sample array (its own min/max,
    1000-point grid), as a Python float."""
    t = _as_device_f64(array, device).reshape(-1, 1)
    return float(kde_mode(t, grid=1000, per_cell=True)[0].item())
