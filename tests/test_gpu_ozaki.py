"""GPU: the exact pass on the int8 matrix cores (irls_oz_impl.hpp).

In mixed mode the fit's first full-data bf16 pass records every chunk's
per-feature max |x|, and the exact pass that publishes Sig_inv (models.py:130)
then forms X^T W X from int8 digit slices with exact int32 sums.  The same fit
with DLSA_OZ=0 runs the fp64-MFMA exact pass at the SAME iterate (the bf16
passes are deterministic), so the two Sig_inv differ only by the Ozaki
scheme's error: asserted below 1e-11 relative to the largest entry (the
path's tolerance is 1e-8), per diagonal entry below 1e-10 of its own size on
columns of very different magnitudes, and bit-identical run to run (integer
accumulation is order-free).  Fallbacks (fp64 mode, chunks over 32767 rows,
P > 112) keep the fp64 pass.
"""

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

REL = 1e-8
OZ_REL = 1e-11


def _rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a visible MI355X"
    return torch


@pytest.fixture(scope="module")
def M():
    from dlsa_amd import models
    return models


def _pair(M, monkeypatch, *args, **kw):
    """The same fit with the Ozaki exact pass and with the fp64-MFMA one."""
    monkeypatch.delenv("DLSA_OZ", raising=False)
    oz = M.logistic_model_batched(*args, **kw)
    monkeypatch.setenv("DLSA_OZ", "0")
    f64 = M.logistic_model_batched(*args, **kw)
    monkeypatch.delenv("DLSA_OZ", raising=False)
    return oz, f64


@pytest.mark.parametrize("p,fi,std", [(13, True, False), (40, False, True), (64, True, True),
                                      (100, False, False), (100, True, True), (101, True, False)])
def test_ozaki_matches_fp64_exact_pass(torch_cuda, M, monkeypatch, p, fi, std):
    """NT = 1 .. 7 (NT = 1 needs P >= 12 for the in-place digit images), intercept and standardisation, ragged partitions and chunks
    (odd block counts, partial 32-row blocks): Sig_inv within 1e-11 of the
    fp64 pass at the same iterate, and the fit within 1e-8 of the oracle."""
    sizes = [3001, 1777, 6145, 2500]
    n = sum(sizes)
    X, y = O.simulate_counter(n, p, seed=11 * p + fi)
    center = scale = None
    if std:
        X = X * 3.0 - 0.7
        center, scale = X.mean(0), X.std(0)
    off = np.concatenate([[0], np.cumsum(sizes)])
    oz, f64 = _pair(M, monkeypatch, X, y, off, fit_intercept=fi, center=center, scale=scale,
                    rows_per_chunk=1000)
    assert oz.stats["passes_oz"] >= 1 and f64.stats["passes_oz"] == 0
    assert (oz.status.cpu().numpy() == 0).all()
    assert _rel(oz.sig_inv.cpu(), f64.sig_inv.cpu()) < OZ_REL
    assert _rel(oz.theta.cpu(), f64.theta.cpu()) < 1e-12
    assert _rel(oz.loglik.cpu(), f64.loglik.cpu()) < 1e-12
    th, S, St, ll, _ = O.logistic_fit_partitions(X, y, off, fit_intercept=fi, center=center,
                                                 scale=scale)
    assert _rel(oz.theta.cpu(), th) < REL
    assert _rel(oz.sig_inv.cpu(), S) < REL
    assert _rel(oz.sig_inv_theta.cpu(), St) < REL


def test_ozaki_column_scales(torch_cuda, M, monkeypatch):
    """Per-chunk, per-feature digit exponents: columns of magnitude 1e-3, 1,
    1e3, an airline-like 1500 + U(0, 900) and a rare 0/1 dummy in one design
    (with an intercept): every diagonal entry within 1e-10 of its own size."""
    rs = np.random.RandomState(3)
    n = 24000
    X = np.column_stack([
        rs.rand(n) * 1e-3, rs.rand(n) - 0.5, (rs.rand(n) - 0.5) * 1e3,
        1500.0 + 900.0 * rs.rand(n), (rs.rand(n) < 0.02).astype(np.float64),
        rs.randn(n, 9)])
    eta = X @ np.concatenate([[200.0, 1.0, 2e-3, -1e-3, 0.7], 0.1 * rs.randn(9)]) + 1.2
    y = (rs.rand(n) < 1.0 / (1.0 + np.exp(-eta))).astype(np.float64)
    off = np.array([0, 9000, n])
    oz, f64 = _pair(M, monkeypatch, X, y, off, fit_intercept=True, rows_per_chunk=2048)
    assert oz.stats["passes_oz"] >= 1
    assert (oz.status.cpu().numpy() == 0).all()
    a, b = oz.sig_inv.cpu().numpy(), f64.sig_inv.cpu().numpy()
    for k in range(2):
        d = np.abs(np.diagonal(a[k]) - np.diagonal(b[k])) / np.abs(np.diagonal(b[k]))
        assert d.max() < 1e-10, d
        assert _rel(a[k], b[k]) < OZ_REL
    th, S, _, _, _ = O.logistic_fit_partitions(X, y, off, fit_intercept=True)
    assert _rel(oz.theta.cpu(), th) < REL
    assert _rel(oz.sig_inv.cpu(), S) < REL


def test_ozaki_bit_identical_runs(torch_cuda, M):
    """Integer level sums are order-free: two fits give bitwise equal Sig_inv."""
    torch = torch_cuda
    p, sizes = 100, [8000, 5001]
    X, y = O.simulate_counter(sum(sizes), p, seed=21)
    off = np.concatenate([[0], np.cumsum(sizes)])
    f1 = M.logistic_model_batched(X, y, off, rows_per_chunk=1500)
    f2 = M.logistic_model_batched(X, y, off, rows_per_chunk=1500)
    assert f1.stats["passes_oz"] >= 1
    assert torch.equal(f1.sig_inv, f2.sig_inv) and torch.equal(f1.theta, f2.theta)


@pytest.mark.parametrize("case", ["fp64_mode", "long_chunks", "wide_p", "wide_long_groups",
                                  "wide_fp64_mode"])
def test_ozaki_fallbacks_keep_the_fp64_pass(torch_cuda, M, case):
    """hessian="fp64" (no bf16 pass records the scales), chunks or wide Gram
    row groups over 32767 rows (int32 level sums) and 112 < P <= 192: the
    fp64-MFMA exact pass / Gram, same parity."""
    p, sizes, kw = 12, [40000, 36000], {"rows_per_chunk": 40000}
    if case == "fp64_mode":
        kw = {"hessian": "fp64", "rows_per_chunk": 3000}
    elif case == "wide_p":
        p, sizes, kw = 120, [6000, 5000], {"rows_per_chunk": 2000}
    elif case == "wide_long_groups":
        p, sizes, kw = 200, [34000, 3000], {"rows_per_chunk": 34000}
    elif case == "wide_fp64_mode":
        p, sizes, kw = 200, [6000, 5000], {"hessian": "fp64", "rows_per_chunk": 2000}
    X, y = O.simulate_counter(sum(sizes), p, seed=5 + p)
    off = np.concatenate([[0], np.cumsum(sizes)])
    fit = M.logistic_model_batched(X, y, off, **kw)
    assert fit.stats["passes_oz"] == 0
    th, S, _, _, _ = O.logistic_fit_partitions(X, y, off)
    assert _rel(fit.theta.cpu(), th) < REL
    assert _rel(fit.sig_inv.cpu(), S) < REL


@pytest.mark.parametrize("p,fi,std", [(200, True, False), (300, False, True), (500, True, False)])
def test_wide_ozaki_gram_matches_fp64_gram(torch_cuda, M, monkeypatch, p, fi, std):
    """Wide path (P > 192, wide_oz.hip): the exact Gram from int8 digit records
    (exponents from the row pass's max |sqrt(w) x| per partition) against the
    fp64 Gram at the same iterate, and the fit against the oracle."""
    sizes = [6000, 5001]
    n = sum(sizes)
    X, y = O.simulate_counter(n, p, seed=13 * p + fi)
    center = scale = None
    if std:
        X = X * 3.0 - 0.7
        center, scale = X.mean(0), X.std(0)
    off = np.concatenate([[0], np.cumsum(sizes)])
    oz, f64 = _pair(M, monkeypatch, X, y, off, fit_intercept=fi, center=center, scale=scale,
                    rows_per_chunk=2000)
    assert oz.stats["passes_oz"] >= 1 and f64.stats["passes_oz"] == 0
    assert (oz.status.cpu().numpy() == 0).all()
    assert _rel(oz.sig_inv.cpu(), f64.sig_inv.cpu()) < OZ_REL
    assert _rel(oz.theta.cpu(), f64.theta.cpu()) < 1e-12
    assert _rel(oz.loglik.cpu(), f64.loglik.cpu()) < 1e-12
    th, S, St, ll, _ = O.logistic_fit_partitions(X, y, off, fit_intercept=fi, center=center,
                                                 scale=scale)
    assert _rel(oz.theta.cpu(), th) < REL
    assert _rel(oz.sig_inv.cpu(), S) < REL
    assert _rel(oz.sig_inv_theta.cpu(), St) < REL
