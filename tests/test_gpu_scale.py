"""GPU parity at the BASELINE configs' own partition sizes.

The small-shape parity tests (test_gpu_parity.py) cover every kernel
geometry; these run the configs as the bench runs them -- config 2 at its full
K = 1024 (n = 1e8, p = 100), config 3 at ~117k rows per partition (P = 182,
categorical codes), config 4 at ~977k rows per partition (OLS, p = 64) -- with
2-4 sampled partitions against the CPU oracle and size-independent checks on
every partition (status, exact Sig_inv symmetry, the score / normal equations
evaluated on the device in fp64, the combine + DBIC selection).

Tolerance contract (BASELINE.json north_star): 1e-8 relative to the largest
entry for theta_k and Sig_inv_k; identical DBIC support.
"""

import numpy as np
import pytest

import oracle as O
from _allparts import all_partitions_independent

pytestmark = pytest.mark.gpu

REL = 1e-8


def _rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return np.abs(a - b).max() / max(np.abs(b).max(), 1e-300)


def _elem(a, b):
    """max_ij |a_ij - b_ij| / sqrt(b_ii b_jj): every entry on its own scale."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    d = np.sqrt(np.abs(np.diagonal(b)))
    return float((np.abs(a - b) / np.outer(d, d)).max())


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a visible MI355X"
    return torch


@pytest.fixture(scope="module")
def M():
    from dlsa_amd import models
    return models


def test_config2_full_K1024(torch_cuda, M):
    """BASELINE config 2 exactly: n = 1e8 rows, p = 100, K = 1024 partitions
    of 97 656 (+1) rows generated in HBM, the default mixed-Hessian fit.
    Every partition: status ok, Sig_inv exactly symmetric, score equation
    X_k^T (y_k - sigmoid(X_k theta_k)) ~ 0 (batched on the device); partitions
    0 and 1023 against the oracle; WLSE and the DBIC support of the full
    combine against the oracle's selection on the same sums."""
    torch = torch_cuda
    from dlsa_amd.dlsa import dlsa, dlsa_mapred

    n, p, K = 100_000_000, 100, 1024
    X, y = M.simulate_logistic_device(n, p, seed=2019)
    off = (np.arange(K + 1, dtype=np.int64) * n) // K
    fit = M.logistic_model_batched(X, y, off)
    assert (fit.status.cpu().numpy() == 0).all(), fit.status_counts()
    S = fit.sig_inv
    assert torch.equal(S, S.transpose(1, 2))
    # score equation on every partition: partitions hold 97 656 or 97 657 rows
    gmax = 0.0
    for k0 in range(0, K, 128):
        for k in range(k0, k0 + 128):
            a, b = int(off[k]), int(off[k + 1])
            Xk = X[a:b]
            g = Xk.T @ (y[a:b] - torch.sigmoid(Xk @ fit.theta[k]))
            gmax = max(gmax, g.abs().max().item())
    assert gmax < 1e-6, gmax
    for k in (0, K - 1):
        a, b = int(off[k]), int(off[k + 1])
        o = O.logistic_fit(X[a:b].cpu().numpy(), y[a:b].cpu().numpy())
        assert _rel(fit.theta[k].cpu(), o["coef"]) < REL
        assert _rel(fit.sig_inv[k].cpu(), o["Sig_inv"]) < REL
        assert _elem(fit.sig_inv[k].cpu(), o["Sig_inv"]) < 1e-10  # the int8 exact pass, per entry
        assert _rel(fit.sig_inv_theta[k].cpu(), o["Sig_invMcoef"]) < REL
    assert fit.stats["passes_oz"] >= 1
    comb = dlsa_mapred(fit)
    Ssum = comb.iloc[:, 2:].to_numpy()
    wlse_ref = np.linalg.lstsq(Ssum, fit.sig_inv_theta.sum(0).cpu().numpy(), rcond=None)[0]
    assert _rel(comb["beta_byOLS"], wlse_ref) < 1e-10
    sel = dlsa(Ssum, comb["beta_byOLS"], n)
    _, b_bic = O.dlsa(Ssum, comb["beta_byOLS"].to_numpy(), n)
    assert np.nonzero(sel["beta_byBIC"].to_numpy())[0].tolist() == np.nonzero(b_bic)[0].tolist()
    assert set(range(40)) <= set(np.nonzero(b_bic)[0].tolist())  # the 0.4 p true nonzeros
    all_partitions_independent(fit, X, y, n, sel)


def test_config3_partition_size(torch_cuda, M):
    """BASELINE config 3 geometry at its partition size: the airline-like
    categorical-code layout (9 numeric + 5 factors, P = 182 with the
    intercept), K = 8 partitions of ~117k rows in HBM.  Partitions 0 and 5
    against the oracle on the dense dummy expansion; every partition: status
    ok, Sig_inv symmetric, the score equation on the device-expanded design."""
    torch = torch_cuda
    K, nk = 8, 117_188
    n = K * nk + 5
    Xn, codes, y, levels = M.simulate_categorical(n, seed=2019, device="cuda")
    off = (np.arange(K + 1, dtype=np.int64) * n) // K
    fit = M.logistic_model_batched_categorical(Xn, codes, y, off, levels, fit_intercept=True)
    assert (fit.status.cpu().numpy() == 0).all(), fit.status_counts()
    assert fit.theta.shape == (K, 182)
    assert torch.equal(fit.sig_inv, fit.sig_inv.transpose(1, 2))
    Xd = M.expand_categorical(Xn, codes, levels)
    Xd = torch.cat([torch.ones((n, 1), dtype=torch.float64, device=Xd.device), Xd], 1)
    for k in range(K):
        a, b = int(off[k]), int(off[k + 1])
        g = Xd[a:b].T @ (y[a:b] - torch.sigmoid(Xd[a:b] @ fit.theta[k]))
        assert g.abs().max().item() < 1e-5  # Sum w over 117k rows ~ 2.3e4: 1e-5 ~ 1e-9 rel
    Xh = Xd.cpu().numpy()
    yh = y.cpu().numpy()
    for k in (0, 5):
        a, b = int(off[k]), int(off[k + 1])
        o = O.logistic_fit(Xh[a:b], yh[a:b])  # intercept column already in Xh
        assert _rel(fit.theta[k].cpu(), o["coef"]) < REL
        assert _rel(fit.sig_inv[k].cpu(), o["Sig_inv"]) < REL
    del Xh
    # every partition per entry, on the device-expanded dense design (the
    # check adds the intercept column itself), and the selection on those sums
    from dlsa_amd.dlsa import dlsa, dlsa_mapred
    comb = dlsa_mapred(fit)
    sel = dlsa(comb.iloc[:, 2:].to_numpy(), comb["beta_byOLS"], n, fit_intercept=True)
    Xe = Xd[:, 1:]
    all_partitions_independent(fit, Xn, y, n, sel, design=lambda a, b: Xe[a:b])


def test_config3_reference_partition_policy(torch_cuda, M):
    """Config 3 at the reference's own partition policy: K = ceil(n / 1e6)
    and row % K (projects/logistic_dlsa.py:170, 239-245), i.e. partitions of
    1e6 rows of the airline-like categorical layout (P = 182).  Partition 0
    against the oracle on its dense dummy expansion (1e6 x 182), partition 1
    through the score equation on the device."""
    torch = torch_cuda
    n = 2_000_000
    K = -(-n // 1_000_000)  # ceil(n / 1e6), logistic_dlsa.py:239-240
    Xn, codes, y, levels = M.simulate_categorical(n, seed=7, device="cuda")
    # row % K then grouped (repartition + groupby): partition k = rows k, k+K, ...
    order = torch.cat([torch.arange(k, n, K, device="cuda") for k in range(K)])
    Xn, codes, y = Xn[order].contiguous(), codes[order].contiguous(), y[order].contiguous()
    off = np.array([0] + [len(range(k, n, K)) for k in range(K)], dtype=np.int64).cumsum()
    assert (np.diff(off) == 1_000_000).all()
    fit = M.logistic_model_batched_categorical(Xn, codes, y, off, levels, fit_intercept=True)
    assert (fit.status.cpu().numpy() == 0).all(), fit.status_counts()
    # partitions of >= 2^19 rows run a 1/16-prefix warm-start level first
    # (capi.hip fit_categorical): some passes streamed fewer than all n rows
    st = fit.stats
    assert st["rows_fp64"] < st["passes_fp64"] * n, st
    Xd = M.expand_categorical(Xn, codes, levels)
    Xd = torch.cat([torch.ones((n, 1), dtype=torch.float64, device=Xd.device), Xd], 1)
    a, b = int(off[1]), int(off[2])
    g = Xd[a:b].T @ (y[a:b] - torch.sigmoid(Xd[a:b] @ fit.theta[1]))
    assert g.abs().max().item() < 1e-4  # Sum w over 1e6 rows ~ 2e5: 1e-4 ~ 5e-10 rel
    a, b = int(off[0]), int(off[1])
    Xh = Xd[a:b].cpu().numpy()
    yh = y[a:b].cpu().numpy()
    del Xd
    o = O.logistic_fit(Xh, yh)  # intercept column already in Xh
    assert _rel(fit.theta[0].cpu(), o["coef"]) < REL
    assert _rel(fit.sig_inv[0].cpu(), o["Sig_inv"]) < REL
    # both 1e6-row partitions per entry (dense rows expanded per partition)
    from dlsa_amd.dlsa import dlsa, dlsa_mapred
    comb = dlsa_mapred(fit)
    sel = dlsa(comb.iloc[:, 2:].to_numpy(), comb["beta_byOLS"], n, fit_intercept=True)
    all_partitions_independent(fit, Xn, y, n, sel,
                               design=lambda a, b: M.expand_categorical(Xn[a:b], codes[a:b],
                                                                        levels))


def test_config4_partition_size(torch_cuda, M):
    """BASELINE config 4 (OLS DLSA) at its partition size: p = 64, K = 8
    partitions of 976 563 rows in HBM (the bench's linear response).
    Partitions 0 and 7 against the oracle's closed form; every partition:
    the normal equations X_k^T (y_k - X_k theta_k) ~ 0 relative to X_k^T y_k,
    Sig_inv symmetric, rss == |y - X theta|^2."""
    torch = torch_cuda
    K, p = 8, 64
    n = K * 976_563
    X, y0 = M.simulate_logistic_device(n, p, seed=7)
    y = X[:, : int(0.4 * p)].sum(1) + 0.5 * (y0 - 0.5)
    off = (np.arange(K + 1, dtype=np.int64) * n) // K
    fit = M.ols_model_batched(X, y, off)
    assert (fit.status.cpu().numpy() == 0).all()
    assert torch.equal(fit.sig_inv, fit.sig_inv.transpose(1, 2))
    for k in range(K):
        a, b = int(off[k]), int(off[k + 1])
        r = y[a:b] - X[a:b] @ fit.theta[k]
        ne = X[a:b].T @ r
        assert ne.abs().max().item() < 1e-9 * (X[a:b].T @ y[a:b]).abs().max().item()
        rss = float((r * r).sum())
        assert abs(fit.loglik[k].item() - rss) < 1e-8 * rss
    for k in (0, K - 1):
        a, b = int(off[k]), int(off[k + 1])
        o = O.ols_fit(X[a:b].cpu().numpy(), y[a:b].cpu().numpy())
        assert _rel(fit.theta[k].cpu(), o["coef"]) < REL
        assert _rel(fit.sig_inv[k].cpu(), o["Sig_inv"]) < 1e-12
    all_partitions_independent(fit, X, y, n, None, family="ols")


def test_wide_skewed_partitions_level_plans(torch_cuda, M):
    """Wide path (P = 512) with skewed partition sizes, n_k = [5e6, 6e4, 6e4]:
    the 1/16 warm-start level then has MORE Gram row groups (258) than the
    all-rows plan (256), the case the workspace is sized for (capi.hip
    make_wide_layout over every level plan).  The small partitions against
    the oracle; the big one through the score equation."""
    torch = torch_cuda
    p = 512
    sizes = [5_000_000, 60_000, 60_000]
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    X, y = M.simulate_logistic_device(int(off[-1]), p, seed=31)
    fit = M.logistic_model_batched(X, y, off)
    assert (fit.status.cpu().numpy() == 0).all(), fit.status_counts()
    a, b = int(off[0]), int(off[1])
    g = X[a:b].T @ (y[a:b] - torch.sigmoid(X[a:b] @ fit.theta[0]))
    assert g.abs().max().item() < 1e-5
    for k in (1, 2):
        a, b = int(off[k]), int(off[k + 1])
        o = O.logistic_fit(X[a:b].cpu().numpy(), y[a:b].cpu().numpy())
        assert _rel(fit.theta[k].cpu(), o["coef"]) < REL
        assert _rel(fit.sig_inv[k].cpu(), o["Sig_inv"]) < REL
