"""KDE-mode oracle against the golden fixture made by
the reference's own mode_kde_calculation (:166-181) and its ensemble-mode loop
(:747-762) around scipy.stats.gaussian_kde (tests/golden/make_golden.py kde).
CPU only."""
import numpy as np
import pytest

from oracle import kde_ref as K


def test_numpy_restatement_matches_reference_modes(kde_kat):
    x, G = kde_kat["x"], int(kde_kat["grid"])
    dens, grids = K.kde_grid(x, G)
    idx = dens.argmax(1)
    assert K.same_mode(idx, kde_kat["idx_global"], dens).all()
    assert np.array_equal(grids[0], np.linspace(kde_kat["lo"], kde_kat["hi"], G))


def test_numpy_restatement_per_array(kde_kat):
    arrays = kde_kat["arrays"]
    dens, grids = K.kde_grid(arrays.T, 1000, per_cell=True)
    idx = dens.argmax(1)
    assert K.same_mode(idx, kde_kat["idx_arrays"], dens).all()
    assert np.array_equal(grids[np.arange(len(idx)), kde_kat["idx_arrays"]], kde_kat["mode_arrays"])


def test_scipy_loop_reproduces_fixture(kde_kat):
    pytest.importorskip("scipy")
    modes, idx = K.ensemble_mode_scipy(kde_kat["x"], int(kde_kat["grid"]), cells=range(12))
    assert np.array_equal(idx, kde_kat["idx_global"][:12])
    assert K.mode_kde_calculation_scipy(kde_kat["arrays"][0]) == kde_kat["mode_arrays"][0]


def test_kde_bandwidth_matches_scipy(kde_kat):
    stats = pytest.importorskip("scipy.stats")
    x = kde_kat["x"][:, :6]
    _, L, _ = K.kde_params(x)
    for c in range(6):
        ref = float(stats.gaussian_kde(x[:, c]).cho_cov[0, 0])
        assert abs(L[c] - ref) <= 4e-16 * ref
