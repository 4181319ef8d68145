"""GPU parity: the HIP path (libdlsa_hip.so through its C-ABI) against the
reference golden vectors and the pinned CPU oracle.

Tolerance contract (BASELINE.json north_star): theta_k, Sig_inv_k and the
combined estimate within 1e-8 relative (fp64); identical DBIC-selected
support.  Integer/index outputs (status, counts, generator bits) exact.
"""

import os

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

REL = 1e-8  # north_star tolerance, relative to the largest entry


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


def _golden(golden_dir, name):
    return np.load(os.path.join(golden_dir, name))


def _config1(golden_dir):
    g = _golden(golden_dir, "config1_n1e5_p10_K4.npz")
    np.random.seed(int(g["seed"]))
    pid, lab, feat = O.simulate_logistic_arrays(100000, 10, "systematic", 4)
    order, off = O.systematic_partition(pid)
    return g, feat[order], lab[order], off


@pytest.mark.parametrize("hessian", ["mixed", "fp64"])
@pytest.mark.parametrize("tag,fi", [("noint", False), ("int", True)])
def test_config1_vs_reference(golden_dir, torch_cuda, M, hessian, tag, fi):
    from dlsa_amd.dlsa import dlsa, dlsa_mapred

    g, X, y, off = _config1(golden_dir)
    fit = M.logistic_model_batched(X, y, off, fit_intercept=fi, hessian=hessian)
    outs = g["outs_" + tag]
    assert fit.status.cpu().numpy().tolist() == [0, 0, 0, 0]
    assert _rel(fit.theta.cpu(), outs[:, :, 1]) < REL
    assert _rel(fit.sig_inv.cpu(), outs[:, :, 3:]) < REL
    assert _rel(fit.sig_inv_theta.cpu(), outs[:, :, 2]) < REL
    comb = dlsa_mapred(fit)
    assert _rel(comb["beta_byOLS"], g["wlse_" + tag]) < REL
    assert _rel(comb["beta_byONESHOT"], g["oneshot_" + tag]) < REL
    if not fi:
        sel = dlsa(comb.iloc[:, 2:], comb["beta_byOLS"], 100000, fit_intercept=False, type="lasso")
        gb = g["lars_lasso_beta"][int(np.argmin(g["lars_lasso_BIC"]))]
        assert set(np.nonzero(sel["beta_byBIC"].to_numpy())[0]) == set(np.nonzero(gb)[0])


@pytest.mark.parametrize("name", ["p100_n8e4_K4.npz", "p100_n16e4_K8.npz"])
def test_p100_vs_reference(golden_dir, torch_cuda, M, name):
    """p = 100, n_k = 2e4, K = 4 and the SURVEY 8(c) K = 8 fixture."""
    from dlsa_amd.dlsa import dlsa, dlsa_mapred

    P = _golden(golden_dir, name)
    n, K = int(P["n"]), int(P["K"])
    np.random.seed(int(P["seed"]))
    pid, lab, feat = O.simulate_logistic_arrays(n, 100, "systematic", K)
    order, off = O.systematic_partition(pid)
    fit = M.logistic_model_batched(feat[order], lab[order], off)
    assert (fit.status.cpu().numpy() == 0).all()
    assert _rel(fit.theta.cpu(), P["outs"][:, :, 1]) < REL
    assert _rel(fit.sig_inv.cpu(), P["outs"][:, :, 3:]) < REL
    comb = dlsa_mapred(fit)
    assert _rel(comb["beta_byOLS"], P["wlse"]) < REL
    sel = dlsa(comb.iloc[:, 2:], comb["beta_byOLS"], n, type="lasso")
    gb = P["lars_lasso_beta"][int(np.argmin(P["lars_lasso_BIC"]))]
    assert set(np.nonzero(sel["beta_byBIC"].to_numpy())[0]) == set(np.nonzero(gb)[0])


def test_games_expand_vs_reference(golden_dir, torch_cuda, M):
    G = _golden(golden_dir, "games_expand.npz")
    X, y = G["X"].astype(float), G["y"].astype(float)
    order, off = O.systematic_partition(np.arange(len(y)) % 2)
    fit = M.logistic_model_batched(X[order], y[order], off)
    assert _rel(fit.theta.cpu(), G["outs"][:, :, 1]) < REL
    assert _rel(fit.sig_inv.cpu(), G["outs"][:, :, 3:]) < REL


def test_standardized_intercept_vs_reference(golden_dir, torch_cuda, M):
    D = _golden(golden_dir, "standardized_intercept.npz")
    order, off = O.systematic_partition(np.arange(len(D["y"])) % 3)
    fit = M.logistic_model_batched(D["X"][order], D["y"][order], off, fit_intercept=True,
                                   center=D["center"], scale=D["scale"])
    assert _rel(fit.theta.cpu(), D["outs"][:, :, 1]) < REL
    assert _rel(fit.sig_inv.cpu(), D["outs"][:, :, 3:]) < REL


def test_logistic_model_reference_signature(golden_dir, torch_cuda, M):
    """models.py:42 signature and p x (p+3) frame, one Spark group."""
    import pandas as pd

    g, X, y, off = _config1(golden_dir)
    k = 2
    df = pd.DataFrame(np.column_stack([np.full(off[k + 1] - off[k], k), y[off[k]:off[k + 1]],
                                       X[off[k]:off[k + 1]]]),
                      columns=["partition_id", "label"] + [f"x{i}" for i in range(10)])
    out = M.logistic_model(df, "label", fit_intercept=True)
    assert list(out.columns) == ["par_id", "coef", "Sig_invMcoef", "intercept"] + \
        [f"x{i}" for i in range(10)]
    assert _rel(out.to_numpy(), g["outs_int"][k]) < REL


def test_device_generator_matches_host(torch_cuda, M):
    X, y = M.simulate_logistic_device(5000, 37, seed=123, row0=777)
    Xh, yh = O.simulate_counter(5000, 37, seed=123, row0=777)
    assert np.array_equal(X.cpu().numpy(), Xh)
    assert np.array_equal(y.cpu().numpy(), yh)


@pytest.mark.parametrize("p,fi", [(1, False), (1, True), (15, True), (16, False), (16, True),
                                  (33, False), (64, True), (100, False), (127, True), (128, False),
                                  (129, False), (150, True), (181, True), (192, False)])
def test_shapes_vs_oracle(torch_cuda, M, p, fi):
    """Column-tile counts NT = 1..12 (4-wave and 8-wave pass geometries) and
    the partial-tile / intercept edges, ragged partition sizes (incl. a block
    tail of < 8 rows)."""
    sizes = [3001, 1500, 4096, 2003]
    if p > 128:  # keep n_k / P well above the MLE-existence threshold
        sizes = [4 * s + 1 for s in sizes]
    n = sum(sizes)
    X, y = O.simulate_counter(n, p, seed=p * 7 + fi)
    off = np.concatenate([[0], np.cumsum(sizes)])
    fit = M.logistic_model_batched(X, y, off, fit_intercept=fi, rows_per_chunk=1000)
    th, S, St, ll, it = O.logistic_fit_partitions(X, y, off, fit_intercept=fi)
    assert (fit.status.cpu().numpy() == 0).all()
    assert _rel(fit.theta.cpu(), th) < REL
    assert _rel(fit.sig_inv.cpu(), S) < REL
    assert _rel(fit.sig_inv_theta.cpu(), St) < REL
    assert _rel(fit.loglik.cpu(), ll) < 1e-10


def test_misaligned_x_view(torch_cuda, M):
    """X starting 8 bytes off a 16-byte boundary (LDS-DMA shift path)."""
    torch = torch_cuda
    n, p = 5000, 7
    X, y = O.simulate_counter(n, p, seed=5)
    big = torch.zeros((n * p + 1,), dtype=torch.float64, device="cuda")
    big[1:] = torch.from_numpy(X.reshape(-1)).cuda()
    Xv = big[1:].view(n, p)
    assert Xv.data_ptr() % 16 == 8
    off = np.array([0, 2500, n])
    fit = M.logistic_model_batched(Xv, y, off, rows_per_chunk=700)
    th, S, _, _, _ = O.logistic_fit_partitions(X, y, off)
    assert _rel(fit.theta.cpu(), th) < REL
    assert _rel(fit.sig_inv.cpu(), S) < REL


def test_edge_partitions(torch_cuda, M):
    """Empty partition -> zero block (models.py:84-91 semantics), tiny
    partitions -> non-ok status without disturbing the others."""
    p = 5
    sizes = [2000, 0, 3, 2500]
    n = sum(sizes)
    X, y = O.simulate_counter(n, p, seed=9)
    off = np.concatenate([[0], np.cumsum(sizes)])
    fit = M.logistic_model_batched(X, y, off, max_iter=30)
    st = fit.status.cpu().numpy()
    assert st[1] == 3  # empty
    assert np.all(fit.sig_inv[1].cpu().numpy() == 0) and np.all(fit.theta[1].cpu().numpy() == 0)
    assert st[2] != 0  # 3 rows, 5 parameters: singular / no MLE
    for k in (0, 3):
        o = O.logistic_fit(X[off[k]:off[k + 1]], y[off[k]:off[k + 1]])
        assert st[k] == 0
        assert _rel(fit.theta[k].cpu(), o["coef"]) < REL
        assert _rel(fit.sig_inv[k].cpu(), o["Sig_inv"]) < REL


def test_reduce_partitions_and_determinism(torch_cuda, M):
    from dlsa_amd.dlsa import reduce_partitions_device, split_reduced

    p = 20
    sizes = [3000] * 6
    X, y = O.simulate_counter(sum(sizes), p, seed=11)
    off = np.concatenate([[0], np.cumsum(sizes)])
    f1 = M.logistic_model_batched(X, y, off)
    f2 = M.logistic_model_batched(X, y, off)
    assert torch_cuda.equal(f1.theta, f2.theta) and torch_cuda.equal(f1.sig_inv, f2.sig_inv)
    buf = reduce_partitions_device(f1).cpu().numpy()
    S, v, st, K = split_reduced(buf, p)
    assert K == 6
    sig = f1.sig_inv.cpu().numpy()
    acc = np.zeros_like(sig[0])
    for k in range(6):
        acc = acc + sig[k]
    assert np.array_equal(S, acc)
    assert _rel(v, f1.sig_inv_theta.cpu().numpy().sum(0)) < 1e-14
    assert _rel(st, f1.theta.cpu().numpy().sum(0)) < 1e-14


def test_config2_shape_sampled_partitions(torch_cuda, M):
    """BASELINE config-2 geometry (p=100, n_k = 97 656) on 32 partitions
    generated in HBM; 4 sampled partitions against the oracle, all partitions
    through size-independent checks (status, Sig_inv symmetry / PD, score
    equation X^T(y - mu) ~ 0 at theta)."""
    torch = torch_cuda
    K, nk, p = 32, 97656, 100
    X, y = M.simulate_logistic_device(K * nk, p, seed=2019)
    off = np.arange(K + 1, dtype=np.int64) * nk
    fit = M.logistic_model_batched(X, y, off)
    assert (fit.status.cpu().numpy() == 0).all()
    S = fit.sig_inv
    assert torch.allclose(S, S.transpose(1, 2), rtol=0, atol=0)
    for k in (0, 7, 19, 31):
        Xk = X[off[k]:off[k + 1]].cpu().numpy()
        yk = y[off[k]:off[k + 1]].cpu().numpy()
        o = O.logistic_fit(Xk, yk)
        assert _rel(fit.theta[k].cpu(), o["coef"]) < REL
        assert _rel(fit.sig_inv[k].cpu(), o["Sig_inv"]) < REL
    # score equation on every partition, evaluated on the device in fp64
    th = fit.theta
    for k in range(K):
        Xk = X[off[k]:off[k + 1]]
        mu = torch.sigmoid(Xk @ th[k])
        gk = Xk.T @ (y[off[k]:off[k + 1]] - mu)
        assert gk.abs().max().item() < 1e-6


def test_config3_dummy_design_vs_oracle(torch_cuda, M):
    """BASELINE config-3 geometry: airline-like design (9 numeric + 172 dummy
    columns, intercept -> P = 182, the 8-wave NT = 12 pass) generated on the
    device; every partition (ragged sizes) against the oracle, mixed
    Hessian."""
    torch = torch_cuda
    X, y = M.simulate_dummy_design(4 * 20000 + 7, seed=7, device="cuda")
    off = np.array([0, 20000, 40003, 60001, 80007], dtype=np.int64)
    fit = M.logistic_model_batched(X, y, off, fit_intercept=True)
    Xh, yh = X.cpu().numpy(), y.cpu().numpy()
    th, S, St, ll, it = O.logistic_fit_partitions(Xh, yh, off, fit_intercept=True)
    assert (fit.status.cpu().numpy() == 0).all()
    assert fit.theta.shape == (4, 182)
    assert _rel(fit.theta.cpu(), th) < REL
    assert _rel(fit.sig_inv.cpu(), S) < REL
    assert _rel(fit.sig_inv_theta.cpu(), St) < REL
    assert _rel(fit.loglik.cpu(), ll) < 1e-10


@pytest.mark.parametrize("p,fi", [(8, True), (64, False), (100, True)])
def test_ols_vs_oracle(torch_cuda, M, p, fi):
    """Linear DLSA path (config 4 shape at small n): closed-form OLS per
    partition, Sig_inv = X^T X, rss."""
    rs = np.random.RandomState(p)
    sizes = [4000, 2501, 3333]
    n = sum(sizes)
    X = rs.rand(n, p) - 0.5
    y = X @ rs.randn(p) + 0.3 + 0.1 * rs.randn(n)
    off = np.concatenate([[0], np.cumsum(sizes)])
    fit = M.ols_model_batched(X, y, off, fit_intercept=fi, rows_per_chunk=900)
    assert (fit.status.cpu().numpy() == 0).all()
    for k in range(3):
        o = O.ols_fit(X[off[k]:off[k + 1]], y[off[k]:off[k + 1]], fit_intercept=fi)
        assert _rel(fit.theta[k].cpu(), o["coef"]) < REL
        assert _rel(fit.sig_inv[k].cpu(), o["Sig_inv"]) < 1e-12
        Xk = X[off[k]:off[k + 1]]
        if fi:
            Xk = np.column_stack([np.ones(len(Xk)), Xk])
        rss = float(((y[off[k]:off[k + 1]] - Xk @ o["coef"]) ** 2).sum())
        assert abs(fit.loglik[k].item() - rss) < 1e-6 * rss


@pytest.mark.parametrize("p,fi,std", [(63, True, False), (40, True, True), (30, False, True),
                                      (64, False, True)])
def test_ols_small_p_geometry_vs_oracle(torch_cuda, M, p, fi, std):
    """OLS at P <= 64 (16 lanes per row, 8-row blocks, x itself as the MFMA A
    operand with the ring's padded rows zeroed and the intercept column = w):
    ragged partitions and chunks (rows not a multiple of 8), with and without
    the intercept and standardisation, against the oracle on the same design."""
    rs = np.random.RandomState(100 + p)
    sizes = [3001, 2045, 4093]
    n = sum(sizes)
    X = rs.rand(n, p) * 4.0 - 1.0
    y = X @ rs.randn(p) + 0.7 + 0.1 * rs.randn(n)
    off = np.concatenate([[0], np.cumsum(sizes)])
    center = X.mean(0) if std else None
    scale = X.std(0) if std else None
    fit = M.ols_model_batched(X, y, off, fit_intercept=fi, center=center, scale=scale,
                              rows_per_chunk=1003)
    assert (fit.status.cpu().numpy() == 0).all()
    Xs = (X - center) / scale if std else X
    for k in range(3):
        o = O.ols_fit(Xs[off[k]:off[k + 1]], y[off[k]:off[k + 1]], fit_intercept=fi)
        assert _rel(fit.theta[k].cpu(), o["coef"]) < REL
        assert _rel(fit.sig_inv[k].cpu(), o["Sig_inv"]) < 1e-12


@pytest.mark.parametrize("p,fi,std", [(16, False, False), (48, False, True), (47, True, False),
                                      (33, True, True)])
def test_ols_stream_short_chunks_vs_oracle(torch_cuda, M, p, fi, std):
    """OLS stream kernel (ols_stream.hip) with chunks of 7 rows: every chunk
    ends inside a k-step group, so its rows past the chunk come from the
    bounds-checked buffer loads (read as 0, selected away under
    standardisation); P = 16 and 48 without intercept take the FULL path.
    An empty partition gives the zero frame and status 3."""
    rs = np.random.RandomState(200 + p)
    sizes = [517, 0, 96, 1031]
    n = sum(sizes)
    X = rs.rand(n, p) * 3.0 - 0.5
    y = X @ rs.randn(p) + 0.4 + 0.1 * rs.randn(n)
    off = np.concatenate([[0], np.cumsum(sizes)])
    center = X.mean(0) if std else None
    scale = X.std(0) if std else None
    fit = M.ols_model_batched(X, y, off, fit_intercept=fi, center=center, scale=scale,
                              rows_per_chunk=7)
    st = fit.status.cpu().numpy()
    assert st[1] == 3
    assert np.all(fit.sig_inv[1].cpu().numpy() == 0)
    Xs = (X - center) / scale if std else X
    for k in (0, 2, 3):
        assert st[k] == 0
        o = O.ols_fit(Xs[off[k]:off[k + 1]], y[off[k]:off[k + 1]], fit_intercept=fi)
        assert _rel(fit.theta[k].cpu(), o["coef"]) < REL
        assert _rel(fit.sig_inv[k].cpu(), o["Sig_inv"]) < 1e-12


@pytest.mark.parametrize("p,fi,std", [(10, False, False), (100, True, False), (37, True, True)])
def test_loglik_eval_vs_oracle(torch_cuda, M, p, fi, std):
    """Evaluation pass (models.py:151-225): per-partition log-likelihood of 4
    candidate vectors (AIC / BIC / WLSE / ONESHOT in the reference driver)."""
    rs = np.random.RandomState(p)
    sizes = [5000, 3001, 777]
    n = sum(sizes)
    X, y = O.simulate_counter(n, p, seed=3 * p)
    if std:
        X = X * 3.0 + 1.5
    off = np.concatenate([[0], np.cumsum(sizes)])
    P = p + fi
    betas = rs.randn(4, P) * 0.5
    center = X.mean(0) if std else None
    scale = X.std(0) if std else None
    ll = M.logistic_loglik_batched(X, y, off, betas, fit_intercept=fi, center=center,
                                   scale=scale).cpu().numpy()
    for k in range(3):
        ref = O.logistic_loglik(X[off[k]:off[k + 1]], y[off[k]:off[k + 1]], betas,
                                fit_intercept=fi, center=center, scale=scale)
        assert np.abs(ll[k] - ref).max() <= 1e-10 * np.abs(ref).max()


def test_logistic_model_eval_reference_signature(torch_cuda, M):
    import pandas as pd

    p = 6
    X, y = O.simulate_counter(4000, p, seed=17)
    df = pd.DataFrame(np.column_stack([np.zeros(4000), y, X]),
                      columns=["partition_id", "label"] + [f"x{i}" for i in range(p)])
    par = pd.DataFrame(np.random.RandomState(1).randn(p + 1, 4),
                       columns=["beta_byAIC", "beta_byBIC", "beta_byOLS", "beta_byONESHOT"])
    out = M.logistic_model_eval(df, "label", par, fit_intercept=True)
    ref = O.logistic_loglik(X, y, par.to_numpy().T, fit_intercept=True)
    assert list(out.columns) == list(par.columns)
    assert np.abs(out.to_numpy()[0] - ref).max() <= 1e-10 * np.abs(ref).max()


# ---- wide P (DLSA_MAX_P_FUSED < P <= DLSA_MAX_P): row pass + tiled Gram pass
# + blocked Cholesky in HBM (BASELINE config 5 path) ---------------------------

@pytest.mark.parametrize("p,fi,std", [(193, False, False), (200, True, False), (256, False, False),
                                      (300, True, True), (383, True, False), (450, False, False),
                                      (499, True, False), (512, False, False)])
def test_wide_shapes_vs_oracle(torch_cuda, M, p, fi, std):
    """NB = 2..4 column blocks of 128, partial last block / intercept edges,
    several row chunks and Gram row groups per partition (row-group count not
    a multiple of 8), ragged partitions."""
    sizes = [10 * p + 7, 12 * p + 1001, 11 * p]
    n = sum(sizes)
    X, y = O.simulate_counter(n, p, seed=p * 3 + fi)
    center = scale = None
    if std:
        X = X * 2.0 + 0.25
        center, scale = X.mean(0), X.std(0)
    off = np.concatenate([[0], np.cumsum(sizes)])
    fit = M.logistic_model_batched(X, y, off, fit_intercept=fi, center=center, scale=scale,
                                   rows_per_chunk=1000)
    th, S, St, ll, it = O.logistic_fit_partitions(X, y, off, fit_intercept=fi, center=center,
                                                  scale=scale)
    assert (fit.status.cpu().numpy() == 0).all()
    assert _rel(fit.theta.cpu(), th) < REL
    assert _rel(fit.sig_inv.cpu(), S) < REL
    assert _rel(fit.sig_inv_theta.cpu(), St) < REL
    assert _rel(fit.loglik.cpu(), ll) < 1e-10
    S_ = fit.sig_inv.cpu().numpy()
    assert np.array_equal(S_, np.transpose(S_, (0, 2, 1)))


@pytest.mark.parametrize("p,fi,std", [(300, True, False), (301, False, True), (450, True, True)])
def test_wide_fused_pass_gradient_fixed_point(torch_cuda, M, p, fi, std):
    """The fused bf16 pass's fp64 gradient / log-lik: run the approximate
    phase to a step of 1e-12 (switch_tol), so it stops at the zero of ITS
    gradient; if that gradient is the true X^T (y - mu), the exact phase then
    accepts the point in ONE fp64 pass and the fit matches the oracle.
    Even / odd p (16-byte / 8-byte row loads), intercept, standardisation."""
    n = 14 * p + 333
    X, y = O.simulate_counter(n, p, seed=p + 11)
    center = scale = None
    if std:
        X = X * 1.5 - 0.2
        center, scale = X.mean(0), X.std(0)
    off = np.array([0, n], dtype=np.int64)
    fit = M.logistic_model_batched(X, y, off, fit_intercept=fi, center=center, scale=scale,
                                   switch_tol=1e-12, rows_per_chunk=1500)
    assert fit.stats["passes_fp32"] >= 3
    assert fit.stats["passes_fp64"] == 1
    th, S, St, ll, it = O.logistic_fit_partitions(X, y, off, fit_intercept=fi, center=center,
                                                  scale=scale)
    assert int(fit.status[0]) == 0
    assert _rel(fit.theta.cpu(), th) < REL
    assert _rel(fit.sig_inv.cpu(), S) < REL
    assert _rel(fit.loglik.cpu(), ll) < 1e-10


def test_wide_auto_chunking_and_determinism(torch_cuda, M):
    """Default (automatic) row-chunk / row-group plan, and bit-identical
    results across two runs (fixed-order reductions everywhere)."""
    torch = torch_cuda
    p, K, nk = 260, 5, 6000
    X, y = M.simulate_logistic_device(K * nk, p, seed=77)
    off = np.arange(K + 1, dtype=np.int64) * nk
    f1 = M.logistic_model_batched(X, y, off, fit_intercept=True)
    f2 = M.logistic_model_batched(X, y, off, fit_intercept=True)
    assert torch.equal(f1.theta, f2.theta) and torch.equal(f1.sig_inv, f2.sig_inv)
    Xh, yh = X.cpu().numpy(), y.cpu().numpy()
    for k in (0, 4):
        o = O.logistic_fit(Xh[off[k]:off[k + 1]], yh[off[k]:off[k + 1]], fit_intercept=True)
        assert _rel(f1.theta[k].cpu(), o["coef"]) < REL
        assert _rel(f1.sig_inv[k].cpu(), o["Sig_inv"]) < REL


def test_wide_edge_partitions(torch_cuda, M):
    """Empty partition -> zero block; a partition with fewer rows than
    parameters -> singular, the others unaffected."""
    p = 220
    sizes = [4000, 0, 150, 3500]
    n = sum(sizes)
    X, y = O.simulate_counter(n, p, seed=19)
    off = np.concatenate([[0], np.cumsum(sizes)])
    fit = M.logistic_model_batched(X, y, off, max_iter=30, rows_per_chunk=700)
    st = fit.status.cpu().numpy()
    assert st[1] == 3
    assert np.all(fit.sig_inv[1].cpu().numpy() == 0)
    assert st[2] != 0
    for k in (0, 3):
        o = O.logistic_fit(X[off[k]:off[k + 1]], y[off[k]:off[k + 1]])
        assert st[k] == 0
        assert _rel(fit.theta[k].cpu(), o["coef"]) < REL
        assert _rel(fit.sig_inv[k].cpu(), o["Sig_inv"]) < REL


@pytest.mark.parametrize("p,fi", [(300, True), (500, False)])
def test_wide_ols_vs_oracle(torch_cuda, M, p, fi):
    rs = np.random.RandomState(p)
    sizes = [4 * p, 3 * p + 11]
    n = sum(sizes)
    X = rs.rand(n, p) - 0.5
    y = X @ rs.randn(p) + 0.3 + 0.1 * rs.randn(n)
    off = np.concatenate([[0], np.cumsum(sizes)])
    fit = M.ols_model_batched(X, y, off, fit_intercept=fi, rows_per_chunk=900)
    assert (fit.status.cpu().numpy() == 0).all()
    for k in range(2):
        o = O.ols_fit(X[off[k]:off[k + 1]], y[off[k]:off[k + 1]], fit_intercept=fi)
        assert _rel(fit.theta[k].cpu(), o["coef"]) < 1e-8
        assert _rel(fit.sig_inv[k].cpu(), o["Sig_inv"]) < 1e-12


def test_config5_shape_sampled_partitions(torch_cuda, M):
    """BASELINE config 5 exactly (p = 500, n = 5e6, K = 32 partitions of
    156 250 rows generated in HBM, the default mixed fit: bf16 fused passes +
    the int8 exact Gram): partitions 0 and 31 against the oracle, every
    partition through the score equation X^T (y - mu) ~ 0 and Sig_inv
    symmetry; then the combine, whose DBIC support must EQUAL the oracle's
    selection on the same sums (dlsa/dlsa.py:70-100)."""
    torch = torch_cuda
    from dlsa_amd.dlsa import dlsa, dlsa_mapred

    K, nk, p = 32, 156250, 500
    X, y = M.simulate_logistic_device(K * nk, p, seed=2019)
    off = np.arange(K + 1, dtype=np.int64) * nk
    fit = M.logistic_model_batched(X, y, off)
    assert (fit.status.cpu().numpy() == 0).all()
    assert fit.stats["passes_oz"] >= 1
    S = fit.sig_inv
    assert torch.equal(S, S.transpose(1, 2))
    for k in (0, K - 1):
        o = O.logistic_fit(X[off[k]:off[k + 1]].cpu().numpy(),
                           y[off[k]:off[k + 1]].cpu().numpy())
        assert _rel(fit.theta[k].cpu(), o["coef"]) < REL
        assert _rel(fit.sig_inv[k].cpu(), o["Sig_inv"]) < REL
        assert _rel(fit.sig_inv_theta[k].cpu(), o["Sig_invMcoef"]) < REL
    th = fit.theta
    for k in range(K):
        Xk = X[off[k]:off[k + 1]]
        gk = Xk.T @ (y[off[k]:off[k + 1]] - torch.sigmoid(Xk @ th[k]))
        assert gk.abs().max().item() < 1e-5
    comb = dlsa_mapred(fit)
    Ssum = comb.iloc[:, 2:].to_numpy()
    sel = dlsa(Ssum, comb["beta_byOLS"], K * nk)
    _, b_bic = O.dlsa(Ssum, comb["beta_byOLS"].to_numpy(), K * nk)
    sup = np.nonzero(sel["beta_byBIC"].to_numpy())[0].tolist()
    assert sup == np.nonzero(b_bic)[0].tolist()
    assert set(range(200)) <= set(sup)  # the 0.4 p true nonzeros are all kept
    from _allparts import all_partitions_independent
    all_partitions_independent(fit, X, y, K * nk, sel)  # all 32 partitions, per entry


# ---------------------------------------------------------------------------
# categorical-code layout (dummy branch, BASELINE config 3)
# ---------------------------------------------------------------------------


def test_logistic_model_dummy_branch_vs_reference(golden_dir, torch_cuda, M):
    """The reference-signature logistic_model with dummy_info / baseline /
    data_info (models.py:42-147) runs the categorical-code HIP pass and
    reproduces the reference's frames; the partition missing a selected level
    returns the all-zero frame with the reference's warning."""
    from test_oracle_golden import _dummy_fixture

    g, df, dinfo, base, info = _dummy_fixture(golden_dir)
    outs = g["outs"]
    for k in range(outs.shape[0]):
        part = df[df["partition_id"] == k].reset_index(drop=True)
        if k == 4:
            with pytest.warns(UserWarning, match="missing in this data chunk"):
                o = M.logistic_model(part, "label", True, dinfo, base, info)
            assert list(o.columns) == [str(c) for c in g["cols"]]
            assert not np.abs(o.to_numpy(dtype=np.float64)).any()
            continue
        o = M.logistic_model(part, "label", True, dinfo, base, info)
        assert list(o.columns) == [str(c) for c in g["cols"]]
        got, ref = o.to_numpy(dtype=np.float64), outs[k]
        assert _rel(got[:, 1], ref[:, 1]) < REL
        assert _rel(got[:, 3:], ref[:, 3:]) < REL
        assert _rel(got[:, 2], ref[:, 2]) < REL


def _cat_case(q, levels, n_parts, seed, center=False):
    rs = np.random.RandomState(seed)
    sizes = [int(s) for s in rs.randint(3000, 9000, size=n_parts)]
    n = sum(sizes)
    Xn = rs.randn(n, q) * 2.0 + 1.0 if center else rs.rand(n, q) - 0.5
    codes = np.stack([np.minimum((L * rs.rand(n) ** 2).astype(np.int64), L - 1)
                      for L in levels], 1).astype(np.uint8) if levels else \
        np.zeros((n, 0), np.uint8)
    D = sum(L - 1 for L in levels)
    beta = np.concatenate([rs.uniform(-1, 1, q) * (0.5 if center else 1.0), 0.4 * rs.randn(D)])
    Xs = (Xn - 1.0) / 2.0 if center else Xn
    X = O.expand_codes(Xs, codes, levels)
    y = (rs.rand(n) < 1 / (1 + np.exp(-(X @ beta - 0.2)))).astype(np.float64)
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    return Xn, codes, y, off


@pytest.mark.parametrize("q,levels,fi,std,rpc", [
    (3, [4, 3], False, False, 0),                 # QN 4 bucket, no intercept
    (7, [5, 5, 9], True, True, 1500),             # QN 8, standardised, multi-chunk partitions
    (9, [12, 7, 20, 30, 30], True, False, 0),     # QN 10 (airline-like numeric block)
    (11, [3] * 10, True, False, 0),               # QN 12, F = 10 (16-factor kernel)
    (15, [4, 6], True, True, 2000),               # QN 16, 256-thread kernel
])
def test_categorical_vs_oracle(torch_cuda, M, q, levels, fi, std, rpc):
    """Categorical-code pass (LDS histograms for the one-hot blocks) against
    the oracle on the dense dummy expansion: every kernel bucket, replicated
    and unreplicated histograms, standardisation, ragged partitions."""
    Xn, codes, y, off = _cat_case(q, levels, 3, seed=q, center=std)
    c = np.full(q, 1.0) if std else None
    s = np.full(q, 2.0) if std else None
    fit = M.logistic_model_batched_categorical(Xn, codes, y, off, levels, fit_intercept=fi,
                                               center=c, scale=s, rows_per_chunk=rpc)
    D = sum(L - 1 for L in levels)
    X = O.expand_codes(Xn, codes, levels)
    kw = {}
    if std:
        kw = dict(center=np.concatenate([c, np.zeros(D)]), scale=np.concatenate([s, np.ones(D)]))
    th, S, St, ll, it = O.logistic_fit_partitions(X, y, off, fit_intercept=fi, **kw)
    assert (fit.status.cpu().numpy() == 0).all(), fit.status
    assert fit.theta.shape == (3, int(fi) + q + D)
    assert _rel(fit.theta.cpu(), th) < REL
    assert _rel(fit.sig_inv.cpu(), S) < REL
    assert _rel(fit.sig_inv_theta.cpu(), St) < REL
    assert _rel(fit.loglik.cpu(), ll) < 1e-10


def test_categorical_config3_geometry_vs_oracle_and_dense(torch_cuda, M):
    """BASELINE config-3 shape (9 numeric + 5 factors -> P = 182) generated on
    the device: categorical path vs the oracle and vs the dense mixed-Hessian
    path on the expanded design; an empty partition (status empty) and a
    partition missing a level (status missing_level, zero outputs)."""
    torch = torch_cuda
    Xn, codes, y, levels = M.simulate_categorical(4 * 20000 + 7, seed=7, device="cuda")
    off = np.array([0, 20000, 40003, 40003, 60001, 80007], dtype=np.int64)
    # partition 4: drop Dest level 5 (-> baseline) so that column has no rows
    sl = slice(60001, 80007)
    c4 = codes[sl, 4]
    codes[sl, 4] = torch.where(c4 == 5, torch.zeros_like(c4), c4)
    fit = M.logistic_model_batched_categorical(Xn, codes, y, off, levels, fit_intercept=True)
    st = fit.status.cpu().numpy().tolist()
    assert st == [0, 0, 3, 0, 5], st
    X = O.expand_codes(Xn.cpu().numpy(), codes.cpu().numpy(), levels)
    keep = [0, 1, 3]
    yh = y.cpu().numpy()
    ref = [O.logistic_fit(X[off[k]:off[k + 1]], yh[off[k]:off[k + 1]], fit_intercept=True)
           for k in keep]
    assert fit.theta.shape == (5, 182)
    assert _rel(fit.theta.cpu()[keep], np.stack([r["coef"] for r in ref])) < REL
    assert _rel(fit.sig_inv.cpu()[keep], np.stack([r["Sig_inv"] for r in ref])) < REL
    assert _rel(fit.sig_inv_theta.cpu()[keep], np.stack([r["Sig_invMcoef"] for r in ref])) < REL
    for k in (2, 4):
        assert not fit.theta[k].abs().max().item() and not fit.sig_inv[k].abs().max().item()
    dense = M.logistic_model_batched(torch.from_numpy(X).cuda(), y, off, fit_intercept=True)
    assert _rel(fit.theta.cpu()[keep], dense.theta.cpu()[keep]) < REL
    assert _rel(fit.sig_inv.cpu()[keep], dense.sig_inv.cpu()[keep]) < REL


def test_categorical_bit_identical_runs_and_column_ranges(torch_cuda, M):
    """The one-hot histograms are fixed-point int64 sums (order-free), so two
    runs are bit-identical; numeric columns of very different magnitudes
    (x 1e3, x 1e-3, an offset column) get their own grids and still match the
    oracle to the parity tolerance."""
    torch = torch_cuda
    Xn, codes, y, levels = M.simulate_categorical(3 * 30000, seed=11, device="cuda")
    Xn = Xn.clone()
    Xn[:, 0] *= 1e3
    Xn[:, 1] *= 1e-3
    Xn[:, 2] += 50.0
    off = np.array([0, 30000, 60000, 90000], dtype=np.int64)
    f1 = M.logistic_model_batched_categorical(Xn, codes, y, off, levels, fit_intercept=True)
    f2 = M.logistic_model_batched_categorical(Xn, codes, y, off, levels, fit_intercept=True)
    assert torch.equal(f1.theta, f2.theta) and torch.equal(f1.sig_inv, f2.sig_inv)
    assert torch.equal(f1.loglik, f2.loglik)
    assert (f1.status.cpu().numpy() == 0).all(), f1.status
    X = O.expand_codes(Xn.cpu().numpy(), codes.cpu().numpy(), levels)
    yh = y.cpu().numpy()
    for k in (0, 2):
        o = O.logistic_fit(X[off[k]:off[k + 1]], yh[off[k]:off[k + 1]], fit_intercept=True)
        assert _rel(f1.theta[k].cpu(), o["coef"]) < REL
        assert _rel(f1.sig_inv[k].cpu(), o["Sig_inv"]) < REL


def _per_entry(S, R):
    """max |S_ij - R_ij| / sqrt(R_ii R_jj) (the Sig_inv metric of the Ozaki tests)"""
    S, R = np.asarray(S, np.float64), np.asarray(R, np.float64)
    d = np.sqrt(np.abs(np.diag(R)))
    return float((np.abs(S - R) / np.maximum(np.outer(d, d), 1e-300)).max())


def test_categorical_outlier_and_rare_level_per_entry(torch_cuda, M):
    """Per-partition fixed-point grids: one numeric value 1e6 x the column's
    range in partition 1 coarsens only partition 1's grid of that column, and
    a level with 25 rows per partition keeps its small blocks exact.  Every
    partition's Sig_inv per entry (|dH_ij| / sqrt(H_ii H_jj)) is within 1e-10
    of the oracle on the dense expansion, and theta within the parity
    tolerance."""
    torch = torch_cuda
    n_k, K = 25000, 4
    Xn, codes, y, levels = M.simulate_categorical(K * n_k, seed=23, device="cuda")
    Xn, codes = Xn.clone(), codes.clone()
    Xn[n_k + 777, 3] = 5e5                  # outlier row in partition 1 (column range 1)
    c = codes[:, 2]
    lv = int(levels[2]) - 1                 # factor 2's last dummy level ...
    c[c == lv] = 1                          # ... made rare: 25 rows per partition
    rs = np.random.RandomState(5)
    rows = np.concatenate([k * n_k + rs.choice(n_k, 25, replace=False) for k in range(K)])
    c[torch.from_numpy(rows).cuda()] = lv
    off = np.arange(K + 1, dtype=np.int64) * n_k
    fit = M.logistic_model_batched_categorical(Xn, codes, y, off, levels, fit_intercept=True)
    assert (fit.status.cpu().numpy() == 0).all(), fit.status
    X = O.expand_codes(Xn.cpu().numpy(), codes.cpu().numpy(), levels)
    yh = y.cpu().numpy()
    for k in range(K):
        o = O.logistic_fit(X[off[k]:off[k + 1]], yh[off[k]:off[k + 1]], fit_intercept=True)
        assert _rel(fit.theta[k].cpu(), o["coef"]) < REL, k
        assert _per_entry(fit.sig_inv[k].cpu().numpy(), o["Sig_inv"]) < 1e-10, k


def test_categorical_invalid_code_fails_loudly(torch_cuda, M):
    from dlsa_amd._hip import DlsaHipError

    Xn, codes, y, off = _cat_case(2, [3, 4], 2, seed=1)
    codes[17, 1] = 4  # levels[1] = 4 -> valid codes 0..3
    with pytest.raises(DlsaHipError, match="level codes"):
        M.logistic_model_batched_categorical(Xn, codes, y, off, [3, 4], fit_intercept=True)


def test_dlsa_fit_sharded_dense_and_categorical(torch_cuda, M):
    """The one-rank path of dlsa_fit_sharded (fit -> HBM pre-reduction -> WLSE
    -> LARS/DBIC) for both layouts: WLSE and the DBIC support match the oracle
    on the dense expansion."""
    from dlsa_amd.distributed import dlsa_fit_sharded

    Xn, codes, y, off = _cat_case(4, [5, 7], 4, seed=21)
    levels = [5, 7]
    X = O.expand_codes(Xn, codes, levels)
    th, S, St, ll, it = O.logistic_fit_partitions(X, y, off, fit_intercept=True)
    wlse, oneshot, Ssum = O.dlsa_mapred(th, S, St)
    for kw in (dict(X=X), dict(X=Xn, codes=codes, levels=levels)):
        Xa = kw.pop("X")
        res = dlsa_fit_sharded(Xa, y, off, fit_intercept=True, **kw)
        assert _rel(res["wlse"], wlse) < REL
        assert _rel(res["oneshot"], oneshot) < REL
        _, b_bic = O.dlsa(Ssum, wlse, int(off[-1]), fit_intercept=True)
        sup_ref = np.nonzero(np.asarray(b_bic)[1:])[0] + 1
        assert res["dbic_support"].tolist() == sup_ref.tolist()


@pytest.mark.parametrize("q,levels,fi", [(0, [6, 4], True), (5, [], True), (3, [1, 5], False)])
def test_categorical_edge_layouts(torch_cuda, M, q, levels, fi):
    """Factors only (q = 0), no factors (F = 0: the numeric block alone), and a
    one-level factor (no dummy columns): same estimates as the oracle on the
    dense expansion."""
    Xn, codes, y, off = _cat_case(q, levels, 2, seed=5 + q)
    fit = M.logistic_model_batched_categorical(Xn, codes, y, off, levels, fit_intercept=fi)
    X = O.expand_codes(Xn, codes, levels)
    th, S, St, ll, it = O.logistic_fit_partitions(X, y, off, fit_intercept=fi)
    assert (fit.status.cpu().numpy() == 0).all(), fit.status
    assert _rel(fit.theta.cpu(), th) < REL
    assert _rel(fit.sig_inv.cpu(), S) < REL


# ---------------------------------------------------------------------------
# boundary, modes and failure handling
# ---------------------------------------------------------------------------


def test_plain_c_abi_entry_as_integration_binds_it(golden_dir, torch_cuda):
    """dlsa_logistic_fit_batched exactly as INTEGRATION.md section 2 binds it
    (a fresh ctypes.CDLL, its argtypes, K = 1 per call, the caller's stream)
    reproduces the reference's config-1 partitions (models.py:42)."""
    import ctypes

    torch = torch_cuda
    from dlsa_amd import _hip

    lib = ctypes.CDLL(_hip.LIB_PATH)
    v = ctypes.c_void_p
    lib.dlsa_logistic_fit_batched.argtypes = [
        v, v, v, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, v, v,
        ctypes.c_int32, ctypes.c_double, v, v, v, v, v, v, v]
    lib.dlsa_last_error.restype = ctypes.c_char_p
    g, X, y, off = _config1(golden_dir)
    for fi, tag in ((False, "noint"), (True, "int")):
        for k in range(4):
            xk = X[off[k]:off[k + 1]]
            n, p = xk.shape
            P = p + int(fi)
            Xd = torch.from_numpy(np.ascontiguousarray(xk)).cuda()
            Yd = torch.from_numpy(np.ascontiguousarray(y[off[k]:off[k + 1]])).cuda()
            th = torch.empty(1, P, dtype=torch.float64, device="cuda")
            S = torch.empty(1, P, P, dtype=torch.float64, device="cuda")
            St = torch.empty(1, P, dtype=torch.float64, device="cuda")
            ll = torch.empty(1, dtype=torch.float64, device="cuda")
            it = torch.empty(1, dtype=torch.int32, device="cuda")
            st = torch.empty(1, dtype=torch.int32, device="cuda")
            offs = np.array([0, n], dtype=np.int64)
            rc = lib.dlsa_logistic_fit_batched(
                Xd.data_ptr(), Yd.data_ptr(), offs.ctypes.data, 1, p, int(fi), None, None, 100,
                1e-10, th.data_ptr(), S.data_ptr(), St.data_ptr(), ll.data_ptr(), it.data_ptr(),
                st.data_ptr(), torch.cuda.current_stream().cuda_stream)
            assert rc == 0, lib.dlsa_last_error()
            torch.cuda.synchronize()
            ref = g["outs_" + tag][k]
            assert int(st.item()) == 0
            assert _rel(th[0].cpu(), ref[:, 1]) < REL
            assert _rel(S[0].cpu(), ref[:, 3:]) < REL
            assert _rel(St[0].cpu(), ref[:, 2]) < REL


@pytest.mark.parametrize("p,fi", [(10, True), (100, False), (150, True), (300, False)])
def test_hessian_mixed_f32_vs_oracle(torch_cuda, M, p, fi):
    """hessian="mixed_f32" (fp32-MFMA approximate Hessian, fp64 gradient and
    final pass) reaches the same MLE and Sig_inv as the oracle -- fused
    (4- and 8-wave) and wide geometries."""
    sizes = [4000 + 13 * p, 3000 + 11 * p]
    n = sum(sizes)
    X, y = O.simulate_counter(n, p, seed=p + 100 * fi)
    off = np.concatenate([[0], np.cumsum(sizes)])
    fit = M.logistic_model_batched(X, y, off, fit_intercept=fi, hessian="mixed_f32",
                                   rows_per_chunk=1500)
    th, S, St, ll, it = O.logistic_fit_partitions(X, y, off, fit_intercept=fi)
    assert (fit.status.cpu().numpy() == 0).all()
    assert fit.stats["passes_fp32"] > 0 and fit.stats["passes_fp64"] > 0
    assert _rel(fit.theta.cpu(), th) < REL
    assert _rel(fit.sig_inv.cpu(), S) < REL
    assert _rel(fit.sig_inv_theta.cpu(), St) < REL


@pytest.mark.parametrize("w", ["1", "2"])
@pytest.mark.parametrize("p,fi,std", [(17, False, False), (64, True, True), (100, False, False),
                                      (111, True, False)])
def test_exact_pass_wave_split_vs_oracle(torch_cuda, M, monkeypatch, w, p, fi, std):
    """The per-wave exact pass in both geometries (exact_waves: all tiles in
    one wave, or the tile rows split over two waves with the rows of a block
    split in the row phase): fp64 fits and OLS against the oracle, with
    standardisation, intercept and ragged partitions (block tails)."""
    sizes = [3001, 1777, 4096 + 9]
    n = sum(sizes)
    X, y = O.simulate_counter(n, p, seed=3 * p + fi)
    center = scale = None
    if std:
        X = X * 3.0 - 0.7
        center, scale = X.mean(0), X.std(0)
    off = np.concatenate([[0], np.cumsum(sizes)])
    fit = M.logistic_model_batched(X, y, off, fit_intercept=fi, center=center, scale=scale,
                                   hessian="fp64", rows_per_chunk=1000, exact_waves=int(w))
    th, S, St, ll, it = O.logistic_fit_partitions(X, y, off, fit_intercept=fi, center=center,
                                                  scale=scale)
    assert (fit.status.cpu().numpy() == 0).all()
    assert _rel(fit.theta.cpu(), th) < REL
    assert _rel(fit.sig_inv.cpu(), S) < REL
    assert _rel(fit.loglik.cpu(), ll) < 1e-10
    yl = X[:, :3].sum(1) + 0.1 * y
    ols = M.ols_model_batched(X, yl, off, fit_intercept=fi, rows_per_chunk=1000,
                              exact_waves=int(w))
    for k in range(3):
        o = O.ols_fit(X[off[k]:off[k + 1]], yl[off[k]:off[k + 1]], fit_intercept=fi)
        assert _rel(ols.theta[k].cpu(), o["coef"]) < REL
        assert _rel(ols.sig_inv[k].cpu(), o["Sig_inv"]) < 1e-12


def test_nonfinite_partition_is_excluded_from_the_combine(torch_cuda, M):
    """A partition with a NaN in X ends "nonfinite" with a finite theta (the
    last finite iterate) and is summed as the reference's zero frame, with a
    warning: WLSE / ONESHOT / DBIC of the others stay finite and equal to the
    oracle's combine with that frame zeroed."""
    from dlsa_amd.dlsa import dlsa_mapred

    p = 6
    sizes = [3000, 2500, 2800]
    n = sum(sizes)
    X, y = O.simulate_counter(n, p, seed=41)
    off = np.concatenate([[0], np.cumsum(sizes)])
    Xb = X.copy()
    Xb[off[1] + 17, 2] = np.nan
    fit = M.logistic_model_batched(Xb, y, off)
    st = fit.status.cpu().numpy()
    assert st.tolist() == [0, 4, 0]
    assert np.isfinite(fit.theta.cpu().numpy()).all()
    with pytest.warns(UserWarning, match=r"partitions \[1\] ended \['nonfinite'\]"):
        comb = dlsa_mapred(fit)
    th, S, St, _, _ = O.logistic_fit_partitions(X, y, off)
    th[1] = 0.0
    S[1] = 0.0
    St[1] = 0.0
    wlse, oneshot, Ssum = O.dlsa_mapred(th, S, St)
    assert _rel(comb["beta_byOLS"], wlse) < REL
    assert _rel(comb["beta_byONESHOT"], oneshot) < REL
    assert _rel(comb.iloc[:, 2:].to_numpy(), Ssum) < REL


# ---------------------------------------------------------------------------
# evaluation pass against the reference's logistic_model_eval (eval.npz)
# ---------------------------------------------------------------------------


@pytest.mark.parametrize("fi", [False, True])
@pytest.mark.parametrize("std", [False, True])
def test_logistic_model_eval_vs_reference(golden_dir, torch_cuda, M, fi, std):
    """models.py:151-225 with the reference's own signature and frames:
    config-1 partitions, 4 candidate columns, intercept / data_info."""
    import pandas as pd

    from test_oracle_golden import _eval_inputs

    E, pid, lab, feat, info = _eval_inputs(golden_dir)
    tag = f"{'int' if fi else 'noint'}_{'std' if std else 'raw'}"
    names = ["beta_byAIC", "beta_byBIC", "beta_byOLS", "beta_byONESHOT"]
    par = pd.DataFrame(E["par_" + tag], columns=names)
    for k in range(4):
        m = pid == k
        df = pd.DataFrame(np.column_stack([pid[m], lab[m], feat[m]]),
                          columns=["partition_id", "label"] + [f"x{i}" for i in range(10)])
        out = M.logistic_model_eval(df, "label", par, fit_intercept=fi,
                                    data_info=info if std else [])
        assert list(out.columns) == names and out.shape == (1, 4)
        ref = E["ll_" + tag][k]
        assert np.abs(out.to_numpy()[0] - ref).max() <= 1e-10 * np.abs(ref).max()


def test_logistic_model_eval_dummy_branch_vs_reference(golden_dir, torch_cuda, M):
    """The dummy branch of logistic_model_eval (models.py:161-205): every
    level present (partitions 0-3 of the dummy fixture) -- the reference's
    values; partition 4 (a selected level missing) -- the reference raises
    (pandas 2, see test_oracle_golden), the product evaluates with that dummy
    column = 0, checked against the oracle on that design."""
    import pandas as pd

    from test_oracle_golden import _dummy_fixture

    E = np.load(os.path.join(golden_dir, "eval.npz"))
    g, df, dinfo, base, info = _dummy_fixture(golden_dir)
    names = ["beta_byAIC", "beta_byBIC", "beta_byOLS", "beta_byONESHOT"]
    par = pd.DataFrame(E["par_dummy"], columns=names)
    df = df[["partition_id", "label", "DepTime", "Distance", "Month", "UniqueCarrier", "Origin"]]
    for k in range(4):
        part = df[df["partition_id"] == k].reset_index(drop=True)
        out = M.logistic_model_eval(part, "label", par, True, dinfo, base, info)
        ref = E["ll_dummy"][k]
        assert np.abs(out.to_numpy()[0] - ref).max() <= 1e-10 * np.abs(ref).max()
    part = df[df["partition_id"] == 4].reset_index(drop=True)
    with pytest.warns(UserWarning, match="missing in this data chunk"):
        out = M.logistic_model_eval(part, "label", par, True, dinfo, base, info)
    num = {c: part[c].to_numpy() for c in ("Distance", "DepTime")}
    fac = {c: part[c].to_numpy() for c in ("Month", "UniqueCarrier", "Origin")}
    X, cols, missing = O.dummy_design(num, fac, dinfo, base)
    assert missing
    center = np.array([float(info[c][1]) if c in num else 0.0 for c in cols])
    scale = np.array([float(info[c][2]) if c in num else 1.0 for c in cols])
    ref = O.logistic_loglik(X, part["label"].to_numpy(), par.to_numpy().T, fit_intercept=True,
                            center=center, scale=scale)
    assert np.isfinite(out.to_numpy()).all()
    assert np.abs(out.to_numpy()[0] - ref).max() <= 1e-10 * np.abs(ref).max()


@pytest.mark.parametrize("p,fi,std", [(20, False, False), (24, False, False), (36, True, False),
                                      (87, True, True), (100, True, False), (116, False, False)])
def test_exact_pass_edge_strip_vs_oracle(torch_cuda, M, p, fi, std):
    """The exact pass's last tile row as 4x4x4_4b sub-blocks (irls_wave_impl.hpp
    edge strip): one sub-block (P - 16 (NT - 1) <= 4: P = 20, 116) and two
    (<= 8: P = 24, 37, 88, 101), in the two-wave and the one-wave (NT = 8)
    geometry, fp64 fits and OLS against the oracle."""
    sizes = [2999, 1781, 4096 + 13]
    n = sum(sizes)
    X, y = O.simulate_counter(n, p, seed=5 * p + fi)
    center = scale = None
    if std:
        X = X * 2.0 + 0.3
        center, scale = X.mean(0), X.std(0)
    off = np.concatenate([[0], np.cumsum(sizes)])
    fit = M.logistic_model_batched(X, y, off, fit_intercept=fi, center=center, scale=scale,
                                   hessian="fp64", rows_per_chunk=1000)
    th, S, St, ll, it = O.logistic_fit_partitions(X, y, off, fit_intercept=fi, center=center,
                                                  scale=scale)
    assert (fit.status.cpu().numpy() == 0).all()
    assert _rel(fit.theta.cpu(), th) < REL
    assert _rel(fit.sig_inv.cpu(), S) < REL
    assert _rel(fit.sig_inv_theta.cpu(), St) < REL
    assert _rel(fit.loglik.cpu(), ll) < 1e-10
    yl = X[:, :3].sum(1) + 0.1 * y
    ols = M.ols_model_batched(X, yl, off, fit_intercept=fi, rows_per_chunk=1000)
    for k in range(3):
        o = O.ols_fit(X[off[k]:off[k + 1]], yl[off[k]:off[k + 1]], fit_intercept=fi)
        assert _rel(ols.theta[k].cpu(), o["coef"]) < REL
        assert _rel(ols.sig_inv[k].cpu(), o["Sig_inv"]) < 1e-12
