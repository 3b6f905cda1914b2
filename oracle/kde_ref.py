"""ORACLE (test infrastructure only) -- the reference's KDE-mode reduction
 on the CPU, two ways:

* ``ensemble_mode_scipy`` / ``mode_kde_calculation_scipy``: the reference's
  own loops (ERT_Conditional_Diffusion.py:747-762 and :166-181) around
  scipy.stats.gaussian_kde -- the reference's dependency, pinned here at the
  version this image ships (scipy 1.15.3, numpy 2.2.6).  These are the truth
  the golden fixture tests/golden/kde_kat.npz is generated from, and the
  timed CPU baseline.
* ``kde_grid``: a vectorised float64 numpy restatement of gaussian_kde's
  1-D algorithm (scipy/stats/_kde.py: np.cov with aweights = 1/n, Cholesky
  = sqrt, Scott factor neff**(-1/5), whitened points, exp(-r^2/2) * norm
  summed over points), returning the full density on the grid so tests can
  tell a real mismatch from a near-tie between two grid points.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module.

Parity rule used by the tests: the device's grid index equals the oracle's, or
the oracle's densities at the two indices agree to 1e-9 relative (a near-tie:
scipy's BLAS-ordered covariance and glibc's exp vs the device's ordered sums
and exp may move the argmax between two grid points whose densities differ in
the last bits).
"""
from __future__ import annotations

import math

import numpy as np

TIE_RTOL = 1e-9


def mode_kde_calculation_scipy(array) -> float:
    """ERT_Conditional_Diffusion.py:166-181, restated."""
    from scipy import stats
    data_min = np.min(array)
    data_max = np.max(array)
    x_range = np.linspace(data_min, data_max, 1000)
    kde = stats.gaussian_kde(array)
    kde_values = kde(x_range)
    return x_range[np.argmax(kde_values)]


def ensemble_mode_scipy(sim_data, grid: int = 5000, cells=None):
    """ERT_Conditional_Diffusion.py:747-762, restated for sim_data (n, *cells)
    flattened to (n, C).  Returns (modes (C,), indices (C,)) for the cells
    listed in ``cells`` (all by default)."""
    from scipy import stats
    x = np.asarray(sim_data, dtype=np.float64).reshape(sim_data.shape[0], -1)
    x_range = np.linspace(np.min(x), np.max(x), grid)
    idx = range(x.shape[1]) if cells is None else cells
    modes, inds = [], []
    for c in idx:
        kde = stats.gaussian_kde(x[:, c])
        k = int(np.argmax(kde(x_range)))
        inds.append(k)
        modes.append(x_range[k])
    return np.asarray(modes), np.asarray(inds)


def kde_params(x):
    """gaussian_kde's per-cell bandwidth for x (n, C): (w, L, norm)."""
    n = x.shape[0]
    w = np.ones(n) / n
    sw = w.sum()
    avg = (x * w[:, None]).sum(0) / sw
    fact = sw - (w * w).sum() / sw
    d = x - avg
    var = (d * (d * w[:, None])).sum(0) * (1.0 / fact)
    factor = np.power(1.0 / (w ** 2).sum(), -1.0 / 5)
    L = np.sqrt(var) * factor
    norm = math.pow(2 * math.pi, -0.5) / L
    return w, L, norm


def kde_grid(x, grid: int, lo=None, hi=None, per_cell: bool = False, cells=None):
    """Densities (len(cells), grid) and grids of the cells' KDEs."""
    x = np.asarray(x, dtype=np.float64).reshape(x.shape[0], -1)
    idx = np.arange(x.shape[1]) if cells is None else np.asarray(cells)
    if not per_cell:
        lo = np.min(x) if lo is None else lo
        hi = np.max(x) if hi is None else hi
    xs = x[:, idx]
    w, L, norm = kde_params(xs)
    dens = np.empty((len(idx), grid))
    grids = np.empty((len(idx), grid))
    for k in range(len(idx)):
        g = np.linspace(xs[:, k].min(), xs[:, k].max(), grid) if per_cell else np.linspace(lo, hi, grid)
        p = xs[:, k] / L[k]
        q = g / L[k]
        r = p[:, None] - q[None, :]
        dens[k] = (w[:, None] * (np.exp(-(r * r) / 2.0) * norm[k])).sum(0)
        grids[k] = g
    return dens, grids


def same_mode(idx_a, idx_b, dens, rtol: float = TIE_RTOL):
    """Per-cell verdict of the parity rule above (dens from kde_grid)."""
    idx_a = np.asarray(idx_a).reshape(-1)
    idx_b = np.asarray(idx_b).reshape(-1)
    rows = np.arange(len(idx_a))
    va, vb = dens[rows, idx_a], dens[rows, idx_b]
    return (idx_a == idx_b) | (np.abs(va - vb) <= rtol * np.maximum(np.abs(va), np.abs(vb)))
