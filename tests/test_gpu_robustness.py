"""GPU parity beyond converged, well-conditioned fits.

* A budget that runs out (max_iter): the reference returns sklearn's coef at
  whatever point newton-cg stopped and evaluates Sig_inv = X^T W X there
  (dlsa/models.py:110-131, max_iter=500).  The product marks such partitions
  MAXITER and runs one exact pass at the returned theta, so Sig_inv,
  Sig_inv theta and the log-likelihood must be the oracle's evaluation AT THAT
  THETA (1e-8), on the fused (P <= 192), wide (P > 192) and categorical paths.
* Designs on which the bf16-steered Newton could crawl: unstandardised
  airline-like columns (the reference standardises only when data_info is
  given, models.py:99-101) and near-collinear columns.  Default (mixed) mode
  must end status ok at 1e-8 of the oracle; a stalled partition escalates
  bf16 -> fp32 -> fp64 (dlsa_internal.hpp).
* Non-finite data in one partition of a categorical fit must fail only that
  partition (the fixed-point histogram grids come from finite values).
"""

import warnings

import numpy as np
import pytest

import oracle as O
from oracle.dlsa_oracle import _expit, _loglik

pytestmark = pytest.mark.gpu

REL = 1e-8


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


def _eval_at(X, y, theta, fit_intercept=False, center=None, scale=None):
    """Oracle evaluation at a GIVEN theta (models.py:114,130-131): Sig_inv,
    Sig_inv theta and the log-likelihood."""
    X = np.asarray(X, np.float64)
    if center is not None:
        X = (X - center) / scale
    if fit_intercept:
        X = np.concatenate([np.ones((X.shape[0], 1)), X], axis=1)
    eta = X @ theta
    mu = _expit(eta)
    w = mu * (1.0 - mu)
    S = X.T @ (w[:, None] * X)
    return S, S @ theta, _loglik(eta, y)


def _check_maxiter(fit, X, y, off, fi, max_iter, expect_maxiter=True):
    st = fit.status.cpu().numpy()
    its = fit.iters.cpu().numpy()
    assert (its <= max_iter).all(), its
    if expect_maxiter:
        assert (st == 1).all(), st
    th = fit.theta.cpu().numpy()
    for k in range(len(off) - 1):
        a, b = off[k], off[k + 1]
        S, St, ll = _eval_at(X[a:b], y[a:b], th[k], fi)
        assert _rel(fit.sig_inv[k].cpu(), S) < REL, (k, _rel(fit.sig_inv[k].cpu(), S))
        assert _rel(fit.sig_inv_theta[k].cpu(), St) < REL
        assert abs(fit.loglik[k].item() - ll) <= 1e-10 * abs(ll)


@pytest.mark.parametrize("hessian", ["mixed", "fp64", "mixed_f32"])
@pytest.mark.parametrize("max_iter", [1, 2, 3])
@pytest.mark.parametrize("p,fi", [(20, True), (100, False)])
def test_maxiter_sig_inv_at_returned_theta_fused(torch_cuda, M, hessian, max_iter, p, fi):
    sizes = [6000, 7001, 5003]
    X, y = O.simulate_counter(sum(sizes), p, seed=31 + p + max_iter)
    off = np.concatenate([[0], np.cumsum(sizes)])
    fit = M.logistic_model_batched(X, y, off, fit_intercept=fi, hessian=hessian,
                                   max_iter=max_iter, rows_per_chunk=2048)
    _check_maxiter(fit, X, y, off, fi, max_iter)
    assert fit.stats["polish_partitions"] == len(sizes)
    if max_iter == 1:  # one full-data Newton step from 0 (no warm-start level)
        assert (fit.iters.cpu().numpy() == 1).all()


@pytest.mark.parametrize("max_iter", [1, 3])
@pytest.mark.parametrize("p,fi,hessian", [(200, True, "mixed"), (256, False, "mixed"),
                                          (210, False, "fp64")])
def test_maxiter_sig_inv_at_returned_theta_wide(torch_cuda, M, max_iter, p, fi, hessian):
    """The wide path (P > 192) with a budget ending in the bf16 phase: every
    MAXITER partition's Sig_inv is the exact X^T W X at its theta (advisor
    finding: it used to stay the all-zero initial frame after a backtrack)."""
    sizes = [9000, 8001]
    X, y = O.simulate_counter(sum(sizes), p, seed=7 * p + max_iter)
    off = np.concatenate([[0], np.cumsum(sizes)])
    fit = M.logistic_model_batched(X, y, off, fit_intercept=fi, hessian=hessian,
                                   max_iter=max_iter)
    assert np.abs(fit.sig_inv.cpu().numpy()).max(axis=(1, 2)).min() > 0
    _check_maxiter(fit, X, y, off, fi, max_iter)


def test_maxiter_sig_inv_at_returned_theta_categorical(torch_cuda, M):
    torch = torch_cuda
    Xn, codes, y, levels = M.simulate_categorical(3 * 6000, seed=5, numeric=3,
                                                  factors=(4, 6), device="cpu")
    off = np.array([0, 6000, 12000, 18000])
    for max_iter in (1, 2):
        fit = M.logistic_model_batched_categorical(Xn.cuda(), codes.cuda(), y.cuda(), off, levels,
                                                   fit_intercept=True, max_iter=max_iter)
        Xd = O.expand_codes(Xn.numpy(), codes.numpy(), levels)
        _check_maxiter(fit, Xd, y.numpy(), off, True, max_iter)
    del torch


def test_maxiter_partitions_enter_the_combine_with_a_warning(torch_cuda, M):
    from dlsa_amd.dlsa import reduce_partitions_device, split_reduced

    sizes = [5000, 5000]
    X, y = O.simulate_counter(sum(sizes), 8, seed=3)
    off = np.concatenate([[0], np.cumsum(sizes)])
    fit = M.logistic_model_batched(X, y, off, max_iter=1)
    assert (fit.status.cpu().numpy() == 1).all()
    with pytest.warns(UserWarning, match="max_iter"):
        buf = reduce_partitions_device(fit).cpu().numpy()
    S, v, st, K = split_reduced(buf, 8)
    assert K == 2
    assert _rel(S, fit.sig_inv.cpu().numpy().sum(0)) < 1e-14


def _airline_raw(n, seed):
    """Unstandardised airline-like design: raw DepTime ~ U(0, 2400), Distance
    ~ U(50, 3000), CRSElapsed ~ U(20, 400) and Month / DayOfWeek dummies."""
    rng = np.random.default_rng(seed)
    dep = rng.uniform(0, 2400, n)
    dist = rng.uniform(50, 3000, n)
    crs = rng.uniform(20, 400, n)
    month = rng.integers(0, 12, n)
    dow = rng.integers(0, 7, n)
    D = np.zeros((n, 11 + 6))
    D[month > 0, month[month > 0] - 1] = 1.0
    D[dow > 0, 11 + dow[dow > 0] - 1] = 1.0
    X = np.column_stack([dep, dist, crs, D])
    beta = np.concatenate([[4e-4, 2e-4, -1e-3], 0.2 * rng.standard_normal(17)])
    eta = -1.0 + X @ beta
    y = (rng.random(n) < 1.0 / (1.0 + np.exp(-eta))).astype(np.float64)
    return X, y


def _collinear(n, p, rho, seed):
    rng = np.random.default_rng(seed)
    X = rng.uniform(-0.5, 0.5, (n, p))
    z = rng.uniform(-0.5, 0.5, n)
    X[:, 1] = rho * X[:, 0] + np.sqrt(1 - rho * rho) * z
    eta = X[:, :4].sum(1)
    y = (rng.random(n) < 1.0 / (1.0 + np.exp(-eta))).astype(np.float64)
    return X, y


@pytest.mark.parametrize("case", ["airline_raw", "collinear_0.999", "collinear_1-1e-6"])
def test_default_mode_ill_conditioned_designs(torch_cuda, M, case):
    sizes = [20000, 24001]
    n = sum(sizes)
    fi = True
    if case == "airline_raw":
        X, y = _airline_raw(n, seed=11)
    elif case == "collinear_0.999":
        X, y = _collinear(n, 10, 0.999, seed=12)
    else:
        X, y = _collinear(n, 10, 1 - 1e-6, seed=13)
    off = np.concatenate([[0], np.cumsum(sizes)])
    fit = M.logistic_model_batched(X, y, off, fit_intercept=fi)  # default: hessian="mixed"
    th, S, St, ll, it = O.logistic_fit_partitions(X, y, off, fit_intercept=fi)
    assert (fit.status.cpu().numpy() == 0).all(), (fit.status, fit.stats)
    assert _rel(fit.theta.cpu(), th) < REL
    assert _rel(fit.sig_inv.cpu(), S) < REL
    assert _rel(fit.sig_inv_theta.cpu(), St) < REL
    print(case, {k: fit.stats[k] for k in ("iterations", "passes_fp32", "passes_f32x",
                                            "passes_fp64")})


def test_stalled_bf16_partition_escalates(torch_cuda, M):
    """Near-collinear columns (correlation 1 - 1e-7): bf16 rounding of the
    Z = sqrt(w) x image swamps the x0 - x1 direction of the Hessian, so the
    bf16-steered step shrinks that component every iteration (contraction
    near 1).  The stall rule moves the partition to fp32 passes; the fit
    converges (status ok) within a normal iteration count."""
    sizes = [30000]
    X, y = _collinear(sizes[0], 10, 1 - 1e-7, seed=21)
    off = np.array([0, sizes[0]])
    fit = M.logistic_model_batched(X, y, off, fit_intercept=True, max_iter=40)
    o = O.logistic_fit(X, y, fit_intercept=True)
    assert fit.status.cpu().numpy().tolist() == [0]
    assert _rel(fit.theta[0].cpu(), o["coef"]) < REL
    assert fit.stats["iterations"] < 40
    assert fit.stats["passes_f32x"] > 0 or fit.stats["passes_fp64"] >= 1


def test_categorical_inf_fails_only_its_partition(torch_cuda, M):
    """One +inf in a numeric column of partition 1 and large-magnitude values
    (x 1e3) in the other partitions: partition 1 ends nonfinite, the others
    match the oracle (advisor finding: the shared fixed-point grid used to
    come from the inf and wrap the other partitions' bins)."""
    Xn, codes, y, levels = M.simulate_categorical(4 * 5000, seed=17, numeric=3,
                                                  factors=(5, 4), device="cpu")
    Xn = Xn.numpy().copy()
    Xn[:, 1] *= 1e3
    Xn[5000 + 123, 0] = np.inf
    off = np.arange(5, dtype=np.int64) * 5000
    fit = M.logistic_model_batched_categorical(Xn, codes, y, off, levels, fit_intercept=True)
    st = fit.status.cpu().numpy()
    assert st[1] == 4, st
    Xd = O.expand_codes(Xn, codes.numpy(), levels)
    yn = y.numpy()
    for k in (0, 2, 3):
        o = O.logistic_fit(Xd[off[k]:off[k + 1]], yn[off[k]:off[k + 1]], fit_intercept=True)
        assert st[k] == 0
        assert _rel(fit.theta[k].cpu(), o["coef"]) < REL
        assert _rel(fit.sig_inv[k].cpu(), o["Sig_inv"]) < REL
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        from dlsa_amd.dlsa import reduce_partitions_device
        buf = reduce_partitions_device(fit).cpu().numpy()
    assert np.isfinite(buf).all()


@pytest.mark.parametrize("p", [8, 16, 100, 200])
def test_huge_magnitude_fails_only_its_partition(torch_cuda, M, p):
    """A value of 2^1010 in partition 1 (beyond the int8 digit grid's EMAX:
    its digits would wrap to a finite, wrong Gram): partition 1 must end in a
    failure status -- never status ok with a finite Sig_inv -- and the other
    partitions match the oracle (fused P <= 192 -- p = 16 and 100 are on the
    int8 exact pass's shapes, P >= 12 -- and wide P > 192 paths)."""
    rng = np.random.default_rng(5 + p)
    n_k, K = 3000, 3
    X = rng.normal(size=(n_k * K, p)) * 0.3
    y = (rng.random(n_k * K) < _expit(X @ (rng.normal(size=p) * 0.2))).astype(np.float64)
    X[n_k + 77, 2] = 2.0 ** 1010
    off = np.arange(K + 1, dtype=np.int64) * n_k
    fit = M.logistic_model_batched(X, y, off)
    st = fit.status.cpu().numpy()
    assert st[1] != 0, st
    for k in (0, 2):
        o = O.logistic_fit(X[off[k]:off[k + 1]], y[off[k]:off[k + 1]])
        assert st[k] == 0, st
        assert _rel(fit.theta[k].cpu(), o["coef"]) < REL
        assert _rel(fit.sig_inv[k].cpu(), o["Sig_inv"]) < REL
