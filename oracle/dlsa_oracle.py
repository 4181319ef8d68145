"""numpy restatement of the reference DLSA path -- TEST INFRASTRUCTURE ONLY.

Every function cites the reference file:line it restates
(/root/reference = Vicky-Lamperouge/dlsa).  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg may import
this module; the product package ``dlsa_amd`` never does.

Pinned against the reference's own outputs: ``tests/golden/make_golden.py``
runs the reference (through a compatibility shim) and the
``tests/test_oracle_golden.py`` suite checks this restatement against those
vectors.
"""

from __future__ import annotations

import math

import numpy as np

# --------------------------------------------------------------------------
# a1: synthetic data generator
# --------------------------------------------------------------------------


def simulate_logistic_arrays(sample_size, p, partition_method="systematic",
                             partition_num=1):
    """Vectorised restatement of ``simulate_logistic`` (dlsa/models.py:6-40).

    The reference draws ``np.random.rand(n, p)`` (models.py:22) and then, row
    by row, ``np.random.binomial(n=1, p=prob[i], size=1)`` (models.py:30).
    One vectorised ``np.random.binomial(1, prob)`` call consumes the legacy
    RNG stream in the same order, so for the same ``np.random.seed`` the
    arrays are bit-identical (pinned by tests/golden/simulate_*.npz).

    Returns ``(partition_id[n], label[n], features[n, p])`` as float64.
    """
    n = int(sample_size)
    p1 = int(p * 0.4)                              # models.py:12
    beta = np.zeros((p, 1))                        # models.py:18-19
    beta[:p1] = 1
    features = np.random.rand(n, p) - 0.5          # models.py:22
    prob = 1 / (1 + np.exp(-features.dot(beta)))   # models.py:23
    label = np.random.binomial(1, prob[:, 0]).astype(np.float64)  # models.py:28-30
    if partition_method != "systematic":           # models.py:32-35
        raise Exception("No such partition method implemented!")
    partition_id = (np.arange(n) % partition_num).astype(np.float64)
    return partition_id, label, features


def simulate_logistic(sample_size, p, partition_method="systematic",
                      partition_num=1):
    """DataFrame form of :func:`simulate_logistic_arrays` (models.py:37-38)."""
    import pandas as pd

    pid, label, features = simulate_logistic_arrays(sample_size, p,
                                                    partition_method,
                                                    partition_num)
    data_np = np.concatenate((pid[:, None], label[:, None], features), 1)
    return pd.DataFrame(data_np, columns=["partition_id", "label"] +
                        ["x" + str(x) for x in range(p)])


_M64 = (1 << 64) - 1
_Y_SALT = 0x5DEECE66D


def _u01_counter(seed, ctr):
    """splitmix64 finaliser of (seed + (ctr+1) * golden) -> U[0,1) with 53 bits
    (dlsa_amd/csrc/aux_kernels.hip:u01), vectorised over uint64 counters."""
    with np.errstate(over="ignore"):
        z = np.uint64(seed & _M64) + (ctr.astype(np.uint64) + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)


def simulate_counter(n, p, seed=2019, row0=0):
    """Host restatement of the device generator ``dlsa_simulate_logistic``
    (SURVEY 8(d) large-config input): same distribution as
    ``simulate_logistic`` (X ~ U(-1/2, 1/2), beta* = 1 on the first
    floor(0.4 p) columns, y ~ Bernoulli(sigmoid(X beta*))) from counter-based
    streams, so the GPU can generate 80 GB in place and the host can
    regenerate any rows bit for bit."""
    rows = np.arange(row0, row0 + n, dtype=np.uint64)
    ctr = rows[:, None] * np.uint64(p) + np.arange(p, dtype=np.uint64)[None, :]
    X = _u01_counter(seed, ctr) - 0.5
    p1 = int(p * 0.4)
    eta = np.zeros(n)
    for j in range(p1):  # sequential order, as the device loop
        eta = eta + X[:, j]
    prob = 1.0 / (1.0 + np.exp(-eta))
    y = (_u01_counter(seed ^ _Y_SALT, rows) < prob).astype(np.float64)
    return X, y


def systematic_partition(partition_id):
    """Stable grouping of rows by partition id (Spark ``groupby`` at
    projects/logistic_dlsa.py:325 hands each group to the UDF in row order).

    Returns ``(order, offsets)``: ``order`` permutes rows so that each
    partition is contiguous; ``offsets[k]:offsets[k+1]`` is partition k.
    """
    pid = np.asarray(partition_id).astype(np.int64)
    order = np.argsort(pid, kind="stable")
    K = int(pid.max()) + 1 if pid.size else 0
    counts = np.bincount(pid, minlength=K)
    offsets = np.zeros(K + 1, dtype=np.int64)
    np.cumsum(counts, out=offsets[1:])
    return order, offsets


# --------------------------------------------------------------------------
# a4-a9: per-partition logistic fit (the map stage)
# --------------------------------------------------------------------------


def _expit(t):
    out = np.empty_like(t)
    pos = t >= 0
    out[pos] = 1.0 / (1.0 + np.exp(-t[pos]))
    e = np.exp(t[~pos])
    out[~pos] = e / (1.0 + e)
    return out


def _loglik(eta, y):
    # sum_i y_i eta_i - log(1 + exp(eta_i)), stable softplus
    sp = np.maximum(eta, 0) + np.log1p(np.exp(-np.abs(eta)))
    return float(np.sum(y * eta - sp))


def logistic_fit(X, y, fit_intercept=False, center=None, scale=None,
                 tol=1e-12, max_iter=100):
    """Restates the body of ``logistic_model`` (dlsa/models.py:94-131).

    * standardise ``(x - mean) / stddev`` with the caller's vectors
      (models.py:99-101, data_info rows 1 and 2);
    * unpenalised logistic MLE (sklearn ``LogisticRegression(solver=
      'newton-cg', penalty='none')``, models.py:110-113).  The MLE does not
      depend on the solver; this restatement uses full Newton (IRLS) with
      step halving, iterated to ``max|step| <= tol * (1 + max|theta|)`` so it
      matches the reference run at a tight tolerance (golden vectors use
      sklearn ``tol=1e-12``);
    * intercept first, implicit ones column (models.py:116-122);
    * ``Sig_inv = X^T diag(p(1-p)) X`` at the estimate (models.py:114,130);
    * ``Sig_invMcoef = Sig_inv @ coef`` (models.py:131).

    Returns dict(coef[p], Sig_inv[p,p], Sig_invMcoef[p], loglik, iters,
    converged).
    """
    X = np.asarray(X, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64).reshape(-1)
    if center is not None:
        X = (X - np.asarray(center, np.float64)) / np.asarray(scale, np.float64)
    if fit_intercept:
        X = np.concatenate([np.ones((X.shape[0], 1)), X], axis=1)
    n, p = X.shape
    theta = np.zeros(p)
    eta = X @ theta
    ll = _loglik(eta, y)
    converged = False
    it = 0
    for it in range(1, max_iter + 1):
        mu = _expit(eta)
        w = mu * (1.0 - mu)
        g = X.T @ (y - mu)
        H = X.T @ (w[:, None] * X)
        step = np.linalg.solve(H, g)
        t = 1.0
        for _ in range(60):  # step halving on a log-likelihood decrease
            cand = theta + t * step
            eta_c = X @ cand
            ll_c = _loglik(eta_c, y)
            if ll_c >= ll - 1e-12 * abs(ll) or t < 1e-12:
                break
            t *= 0.5
        theta, eta, ll = cand, eta_c, ll_c
        if np.max(np.abs(t * step)) <= tol * (1.0 + np.max(np.abs(theta))):
            converged = True
            break
    mu = _expit(eta)
    w = mu * (1.0 - mu)
    Sig_inv = X.T @ (w[:, None] * X)               # models.py:130
    return dict(coef=theta, Sig_inv=Sig_inv, Sig_invMcoef=Sig_inv @ theta,
                loglik=ll, iters=it, converged=converged)


def logistic_fit_partitions(X, y, offsets, **kw):
    """The Spark map stage: ``groupby('partition_id').apply(logistic_model_udf)``
    (projects/logistic_dlsa.py:314-325), one ``logistic_fit`` per partition.
    Returns stacked arrays theta[K,p], sig_inv[K,p,p], sig_inv_theta[K,p]."""
    K = len(offsets) - 1
    outs = [logistic_fit(X[offsets[k]:offsets[k + 1]],
                         y[offsets[k]:offsets[k + 1]], **kw) for k in range(K)]
    return (np.stack([o["coef"] for o in outs]),
            np.stack([o["Sig_inv"] for o in outs]),
            np.stack([o["Sig_invMcoef"] for o in outs]),
            np.array([o["loglik"] for o in outs]),
            np.array([o["iters"] for o in outs]))


def dummy_design(numeric, factors, dummy_info, dummy_factors_baseline=()):
    """Dense design of one data chunk in the reference's dummy branch,
    dlsa/models.py:56-91, restated without pandas:
    dropped levels -> "000_OTHERS" (:59); a dummy per level (:62-65) named
    "<factor>_<value>", baselines dropped (:67, :77); columns = sorted numeric
    names (:70) then each factor's sorted selected names (:72-75).  Returns
    (X [n, p], column names, missing) where ``missing`` is the reference's
    column-set check (:84): the chunk lacks a selected column or has a value
    outside the selected names -> the caller returns the all-zero frame.

    numeric: {name: [n] array}; factors: {name: [n] values} (any order)."""
    base = set(dummy_factors_baseline)
    names_num = sorted(numeric)
    cols = list(names_num)
    blocks = [np.column_stack([np.asarray(numeric[c], dtype=np.float64) for c in names_num])] \
        if names_num else []
    n = len(next(iter(numeric.values()))) if numeric else len(next(iter(factors.values())))
    present = set(names_num)
    for f in dummy_info["factor_selected"]:
        dropped = set(str(v) for v in dummy_info["factor_dropped"].get(f, []))
        vals = ["000_OTHERS" if str(v) in dropped else str(v) for v in factors[f]]
        names = [f"{f}_{v}" for v in vals]
        present |= set(names) - base
        sel = [c for c in sorted(dummy_info["factor_selected_names"][f]) if c not in base]
        cols.extend(sel)
        idx = {c: j for j, c in enumerate(sel)}
        B = np.zeros((n, len(sel)))
        for i, nm in enumerate(names):
            j = idx.get(nm)
            if j is not None:
                B[i, j] = 1.0
        blocks.append(B)
    X = np.hstack(blocks) if blocks else np.zeros((n, 0))
    return X, cols, present != set(cols)


def expand_codes(Xn, codes, levels):
    """Dense dummy design of a categorical-code layout: numeric columns, then
    per factor f the levels[f] - 1 indicator columns of codes 1..L-1 (code 0
    = the dropped baseline level)."""
    Xn = np.asarray(Xn, dtype=np.float64)
    codes = np.asarray(codes)
    blocks = [Xn]
    for f, L in enumerate(levels):
        B = np.zeros((Xn.shape[0], int(L) - 1))
        c = codes[:, f].astype(np.int64)
        m = c > 0
        B[np.nonzero(m)[0], c[m] - 1] = 1.0
        blocks.append(B)
    return np.hstack(blocks)


def logistic_loglik(X, y, betas, fit_intercept=False, center=None, scale=None):
    """Restates the likelihood loop of ``logistic_model_eval``
    (dlsa/models.py:196-225): for each candidate column beta,
    sum(y log p + (1 - y) log(1 - p)), p = sigmoid(x . beta), after the same
    standardisation / intercept handling as the fit (models.py:195-205),
    evaluated in the stable form y eta - softplus(eta)."""
    X = np.asarray(X, dtype=np.float64)
    if center is not None:
        X = (X - np.asarray(center, np.float64)) / np.asarray(scale, np.float64)
    if fit_intercept:
        X = np.concatenate([np.ones((X.shape[0], 1)), X], axis=1)
    y = np.asarray(y, np.float64).reshape(-1)
    betas = np.atleast_2d(np.asarray(betas, np.float64))
    return np.array([_loglik(X @ b, y) for b in betas])


def ols_fit(X, y, fit_intercept=False):
    """Closed-form OLS local fit for the linear DLSA path (SURVEY 8(d) config
    4; the reference only has a statsmodels demo,
    projects/results/linear_regression_dc.py:27-37): theta=(X^T X)^-1 X^T y,
    Sig_inv = X^T X."""
    X = np.asarray(X, np.float64)
    if fit_intercept:
        X = np.concatenate([np.ones((X.shape[0], 1)), X], axis=1)
    G = X.T @ X
    theta = np.linalg.solve(G, X.T @ np.asarray(y, np.float64))
    return dict(coef=theta, Sig_inv=G, Sig_invMcoef=G @ theta)


def column_moments(X):
    """[5, p] count, mean, M2, min, max per column, NaNs skipped -- the
    numbers Spark's ``describe()`` reports (count, mean, stddev = sqrt(M2 /
    (count - 1)), min, max) for the reference's data_info
    (projects/logistic_dlsa.py:287-298), as numpy's two-pass mean /
    variance."""
    X = np.asarray(X, np.float64)
    if X.ndim == 1:
        X = X[:, None]
    if X.shape[0] == 0:
        return np.stack([np.zeros(X.shape[1])] + [np.full(X.shape[1], np.nan)] * 4)
    ok = ~np.isnan(X)
    cnt = ok.sum(0).astype(np.float64)
    with np.errstate(invalid="ignore", divide="ignore"):
        mean = np.where(ok, X, 0.0).sum(0) / cnt
        m2 = (np.where(ok, X - mean, 0.0) ** 2).sum(0)
        mn = np.where(cnt > 0, np.nanmin(np.where(ok, X, np.inf), 0), np.nan)
        mx = np.where(cnt > 0, np.nanmax(np.where(ok, X, -np.inf), 0), np.nan)
    m2 = np.where(cnt > 0, m2, np.nan)
    return np.stack([cnt, mean, m2, mn, mx])


# --------------------------------------------------------------------------
# a11: combine
# --------------------------------------------------------------------------


def dlsa_mapred(theta, sig_inv, sig_inv_theta=None, num_partitions=None):
    """Restates ``dlsa_mapred`` (dlsa/dlsa.py:21-61) on stacked arrays.

    Group-sum over partitions (dlsa.py:30-34), WLSE = lstsq(sum Sig_inv,
    sum Sig_inv@coef, rcond=None) (dlsa.py:44-49) and ONESHOT = sum(coef) /
    number of partitions (dlsa.py:51-52).
    Returns (beta_byOLS[p], beta_byONESHOT[p], Sig_inv_sum[p,p]).
    """
    theta = np.asarray(theta, np.float64)
    sig_inv = np.asarray(sig_inv, np.float64)
    if sig_inv_theta is None:
        sig_inv_theta = np.einsum("kij,kj->ki", sig_inv, theta)
    if theta.shape[0] == 0:
        raise Exception(
            "Zero-length grouped pandas DataFrame obtained, check the input.")
    S = sig_inv.sum(0)
    v = np.asarray(sig_inv_theta, np.float64).sum(0)
    wlse = np.linalg.lstsq(S, v, rcond=None)[0]
    K = theta.shape[0] if num_partitions is None else num_partitions
    return wlse, theta.sum(0) / K, S


# --------------------------------------------------------------------------
# a13: LARS / adaptive lasso on the quadratic form (LSA)
# --------------------------------------------------------------------------


def _backsolvet(R, x):
    # lsa.py:8-9
    return np.linalg.solve(np.triu(R).T, x)


def _update_r(xnew, xold, R, rank, eps):
    # lsa.py:12-32 (np.matrix column/row stacking restated on ndarrays)
    if R is None:
        return np.array([[math.sqrt(xnew)]]), 1
    r = _backsolvet(R, xold)
    rpp = xnew - float(np.sum(r ** 2))
    if rpp <= eps:
        rpp = eps
    else:
        rpp = math.sqrt(rpp)
        rank = rank + 1
    m = R.shape[0]
    Rn = np.zeros((m + 1, m + 1))
    Rn[:m, :m] = R
    Rn[:m, m] = r
    Rn[m, m] = rpp
    return Rn, rank


def _delcol(r, k):
    # lsa.py:35-71: drop column k, restore triangularity by Givens rotations
    p = r.shape[0]
    r = np.delete(r, k, axis=1)
    for i in range(k + 1, p):
        a = r[i - 1, i - 1]
        b = r[i, i - 1]
        if b != 0:
            if not abs(b) > abs(a):
                tau = -b / a
                c = 1 / math.sqrt(1 + tau * tau)
                s = c * tau
            else:
                tau = -a / b
                s = 1 / math.sqrt(1 + tau * tau)
                c = s * tau
            ri = r[i - 1, i - 1:].copy()
            rj = r[i, i - 1:].copy()
            r[i - 1, i - 1:] = c * ri - s * rj
            r[i, i - 1:] = s * ri + c * rj
    return r


def _downdate_r(R, k):
    # lsa.py:74-80
    p = R.shape[1]
    if p == 1:
        return None
    return np.delete(_delcol(R, k), p - 1, axis=0)


def lars_lsa(Sigma0, b0, intercept, n, type="lar", eps=np.finfo(float).eps,
             max_steps=None):
    """Restates ``lars_lsa`` (dlsa/lsa.py:90-212) on plain ndarrays.

    Reference defects fixed here: ``np.float``/``np.NAN``
    (lsa.py:12,23,90) are plain float/nan; the intercept branch slices with
    the parameter count instead of the sample size ``n`` (lsa.py:100,101,196);
    the singular back-out keeps the leading sub-block of R (lsa.py:141-142
    indexes a diagonal by mistake).  ``Sigma0`` may be any 2-D array (the port
    required ``np.matrix``).
    """
    Sigma0 = np.asarray(Sigma0, dtype=np.float64)
    b0 = np.asarray(b0, dtype=np.float64).reshape(-1)
    P = Sigma0.shape[0]
    if intercept:                                   # lsa.py:98-104
        a11 = Sigma0[0, 0]
        a12 = Sigma0[1:P, 0].copy()
        a22 = Sigma0[1:P, 1:P]
        Sigma = a22 - np.outer(a12, a12) / a11
        b = b0[1:].copy()
        beta0_init = float(a12 @ b) / a11
    else:
        Sigma = Sigma0.copy()
        b = b0.copy()
    absb = np.abs(b)
    Sigma = absb[:, None] * Sigma * absb[None, :]   # lsa.py:108
    b = np.sign(b)                                   # lsa.py:109
    m = Sigma.shape[1]
    im = np.arange(1, m + 1)
    inactive = im.copy()
    Cvec = b @ Sigma                                 # lsa.py:114
    if max_steps is None:                            # lsa.py:116-117
        max_steps = 8 * m
    beta = np.zeros((max_steps + 1, m))
    first = np.zeros(m)
    active = np.array([], dtype=int)
    drops = np.array([False])
    Sign = np.array([])
    R, rank = None, 0
    k = 0
    ignores = np.array([], dtype=int)
    C = np.array([])
    Cmax = 0.0
    while k < max_steps and len(active) < m:        # lsa.py:126
        k += 1
        C = Cvec[inactive - 1]
        Cmax = float(np.max(np.abs(C)))
        if not np.any(drops):                        # lsa.py:130-149
            new = inactive[np.abs(C) >= Cmax - eps]
            C = C[np.abs(C) < Cmax - eps]
            for inew in new:
                R, rank = _update_r(Sigma[inew - 1, inew - 1],
                                    Sigma[inew - 1, active - 1], R, rank, eps)
                if rank == len(active):
                    na = len(active)
                    R = R[:na, :na]
                    rank = na
                    ignores = np.append(ignores, inew).astype(int)
                else:
                    if first[inew - 1] == 0:
                        first[inew - 1] = k
                    active = np.append(active, inew).astype(int)
                    Sign = np.append(Sign, np.sign(Cvec[inew - 1]))
        Gi1 = np.linalg.solve(np.triu(R), _backsolvet(R, Sign))   # lsa.py:151
        A = 1 / math.sqrt(float(np.sum(Gi1 * Sign)))
        w = A * Gi1
        if len(active) >= m:                         # lsa.py:154-162
            gamhat = Cmax / A
        else:
            keep = np.setdiff1d(np.arange(m),
                                np.append(active, ignores) - 1)
            a = w @ Sigma[np.ix_(active - 1, keep)]
            gam = np.append((Cmax - C) / (A - a), (Cmax + C) / (A + a))
            gamhat = float(np.min(np.append(gam[gam > eps], Cmax / A)))
        if type == "lasso":                          # lsa.py:164-173
            b1 = beta[k - 1, active - 1]
            z1 = -b1 / w
            zmin = float(np.min(np.append(z1[z1 > eps], gamhat)))
            if zmin < gamhat:
                gamhat = zmin
                drops = z1 == zmin
            else:
                drops = np.array([False])
        beta[k] = beta[k - 1]                        # lsa.py:175-177
        beta[k, active - 1] += gamhat * w
        Cvec = Cvec - gamhat * (Sigma[:, active - 1] @ w)
        if type == "lasso" and np.any(drops):        # lsa.py:179-186
            for did in np.where(drops)[0][::-1]:
                R = _downdate_r(R, did)
                rank = 0 if R is None else R.shape[1]
            dropid = active[drops]
            beta[k, dropid - 1] = 0
            active = active[~drops]
            Sign = Sign[~drops]
        inactive = np.delete(im, active - 1)         # lsa.py:188
    beta = beta[:k + 1]                              # lsa.py:190-192
    dff = b[:, None] - beta.T
    RSS = np.einsum("ij,ik,kj->j", dff, Sigma, dff)
    if intercept:                                    # lsa.py:194-201
        beta = beta * np.abs(b0[1:P])[None, :]
        beta0 = beta0_init - (beta @ a12) / a11      # lsa.py:203-204
    else:
        beta = beta * np.abs(b0)[None, :]
        beta0 = np.zeros(k + 1)                      # lsa.py:206
    dof = np.sum(np.abs(beta) > eps, axis=1)         # lsa.py:208-210
    BIC = RSS + math.log(n) * dof
    AIC = RSS + 2 * dof
    return {"AIC": AIC, "BIC": BIC, "beta": beta, "beta0": beta0}


def dlsa(Sig_inv_, beta_, sample_size, fit_intercept=False, type="lasso"):
    """Restates ``dlsa`` (dlsa/dlsa.py:70-100): LSA path, argmin AIC/BIC
    (dlsa.py:83-86), intercept restored as ``beta0 + WLSE[0]``
    (dlsa.py:88-95).  The reference calls R ``lars.lsa`` (dlsa.py:77-80; the
    R submodule is absent here) whose ``type`` argument defaults to the first
    element of ``c("lasso", "lar")``; ``type`` is exposed so either path can
    be checked.  Returns (beta_byAIC, beta_byBIC)."""
    Sig = np.asarray(Sig_inv_, np.float64)
    b = np.asarray(beta_, np.float64).reshape(-1)
    fit = lars_lsa(Sig, b, intercept=fit_intercept, n=sample_size, type=type)
    ia = int(np.argmin(fit["AIC"]))
    ib = int(np.argmin(fit["BIC"]))
    beta = fit["beta"]
    if fit_intercept:
        beta0 = fit["beta0"] + b[0]
        return (np.hstack([beta0[ia], beta[ia]]),
                np.hstack([beta0[ib], beta[ib]]))
    return beta[ia].copy(), beta[ib].copy()
