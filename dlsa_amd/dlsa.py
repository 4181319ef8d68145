"""Combine and selection steps of DLSA (drop-in for dlsa/dlsa.py).

* ``dlsa_mapred`` -- dlsa/dlsa.py:21-61: sum the per-partition outputs,
  WLSE = lstsq(sum Sig_inv, sum Sig_inv theta), ONESHOT = sum theta / K.  For
  a GPU ``BatchedFit`` the sum runs in HBM (``dlsa_reduce_partitions``); the
  pandas forms mirror the Spark ``groupby('par_id').sum()``.
* ``dlsa`` -- dlsa/dlsa.py:70-100: adaptive-lasso LSA path and the AIC / BIC
  (DBIC) argmin, through the native ``lars_lsa`` instead of R via rpy2.
"""

from __future__ import annotations

import ctypes

import numpy as np

from . import _hip


def wlse(S, v):
    """WLSE = (sum Sig_inv)^-1 (sum Sig_inv theta) (dlsa.py:48-49).

    The reference calls ``np.linalg.lstsq`` (an SVD).  ``sum Sig_inv`` is a sum
    of positive-definite information matrices, so a Cholesky solve gives the
    same solution (to rounding) at a fraction of the host time (P = 182: 0.3 ms
    instead of 6 ms); a matrix that is not numerically positive definite
    (e.g. an all-zero dummy column) falls back to the reference's lstsq,
    whose minimum-norm solution is then the defined result."""
    import scipy.linalg as sla

    S = np.asarray(S, dtype=np.float64)
    v = np.asarray(v, dtype=np.float64)
    try:
        c = sla.cho_factor(S, lower=True, check_finite=True)
        x = sla.cho_solve(c, v, check_finite=False)
        if np.all(np.isfinite(x)):
            return x
    except (np.linalg.LinAlgError, ValueError):
        pass
    return np.linalg.lstsq(S, v, rcond=None)[0]


def _frame(S, v, sum_theta, K, columns):
    import pandas as pd

    p = v.size
    beta_ols = wlse(S, v)                                      # dlsa.py:48-49
    beta_oneshot = sum_theta / K                               # dlsa.py:51-52
    if columns is None:
        columns = [f"x{j}" for j in range(p)]
    return pd.DataFrame(np.concatenate((beta_ols.reshape(p, 1), beta_oneshot.reshape(p, 1), S), 1),
                        columns=["beta_byOLS", "beta_byONESHOT"] + list(columns))


#: statuses whose outputs are not usable estimates: their Sig_inv / theta are
#: replaced by the reference's zero frame (models.py:84-91) in the reduce
EXCLUDED_STATUS = {2: "singular", 4: "nonfinite"}


def reduce_partitions_device(fit, n_rows=False):
    """[sum Sig_inv | sum Sig_inv theta | sum theta | K] of a BatchedFit, as a
    device tensor of P*P + 2P + 1 fp64 (the buffer the RCCL all-reduce sums);
    with ``n_rows`` one more entry holds the fitted row count, so the sharded
    path's single collective also carries N for the DBIC.

    Partitions that reached max_iter are summed as they are (last iterate,
    Sig_inv = X^T W X at it: what the reference sums after sklearn's
    ConvergenceWarning) with a warning.  Partitions whose status is singular
    or nonfinite are summed as the reference's all-zero frame (models.py:84-91)
    with a warning naming them:
    the reference's sklearn fit would not have produced a usable estimate
    either, and one NaN block would otherwise turn WLSE, ONESHOT and the
    LARS/DBIC path into NaN.  Empty / missing-level partitions already are
    zero frames."""
    import warnings

    import torch

    P, K = fit.P, fit.K
    sig, sigt, th = fit.sig_inv, fit.sig_inv_theta, fit.theta
    st = fit.status.cpu().numpy()
    slow = np.nonzero(st == 1)[0]
    if slow.size:
        # the reference sums whatever sklearn returns at max_iter (it only
        # warns, ConvergenceWarning): such a partition is summed with its
        # last iterate and the exact X^T W X at that iterate
        warnings.warn("partitions " + str(slow.tolist()) + " reached max_iter before "
                      "converging: summed with their last iterate and Sig_inv at it")
    bad = np.nonzero(np.isin(st, list(EXCLUDED_STATUS)))[0]
    if bad.size:
        warnings.warn("partitions " + str(bad.tolist()) + " ended "
                      + str(sorted({EXCLUDED_STATUS[int(v)] for v in st[bad]}))
                      + ": summed as zero frames (excluded from WLSE / ONESHOT / DBIC)")
        keep = torch.from_numpy(~np.isin(st, list(EXCLUDED_STATUS))).to(th.device)
        zero = torch.zeros((), dtype=th.dtype, device=th.device)
        sig = torch.where(keep[:, None, None], sig, zero).contiguous()
        sigt = torch.where(keep[:, None], sigt, zero).contiguous()
        th = torch.where(keep[:, None], th, zero).contiguous()
    out = torch.empty((P * P + 2 * P + 1 + (1 if n_rows else 0),), dtype=torch.float64,
                      device=th.device)
    lib = _hip.load()
    stream = ctypes.c_void_p(torch.cuda.current_stream(th.device).cuda_stream)
    rc = lib.dlsa_reduce_partitions(ctypes.c_void_p(sig.data_ptr()),
                                    ctypes.c_void_p(sigt.data_ptr()),
                                    ctypes.c_void_p(th.data_ptr()), K, P,
                                    ctypes.c_void_p(out.data_ptr()), stream)
    _hip.check(rc, "dlsa_reduce_partitions")
    if n_rows:
        out[-1] = float(fit.n_rows)
    return out


def split_reduced(buf, P):
    """Split a reduced buffer (host array) into (S, v, sum_theta, K)."""
    b = np.asarray(buf, dtype=np.float64)
    S = b[:P * P].reshape(P, P)
    v = b[P * P:P * P + P]
    st = b[P * P + P:P * P + 2 * P]
    return S, v, st, float(b[P * P + 2 * P])


def dlsa_mapred(model_mapped_sdf, columns=None, num_partitions=None):
    """MapReduce combine for partitioned fits (dlsa/dlsa.py:21).

    Accepts a ``BatchedFit`` (GPU), a stacked pandas frame shaped like the
    Spark map output (``par_id, coef, Sig_invMcoef, <cols>``), or a list of
    per-partition frames.  Returns the reference frame
    ``[beta_byOLS, beta_byONESHOT, <sum Sig_inv columns>]``.
    """
    import pandas as pd

    from .models import BatchedFit

    if isinstance(model_mapped_sdf, BatchedFit):
        buf = reduce_partitions_device(model_mapped_sdf).cpu().numpy()
        S, v, st, K = split_reduced(buf, model_mapped_sdf.P)
        if columns is None:
            p = model_mapped_sdf.P - (1 if model_mapped_sdf.fit_intercept else 0)
            columns = (["intercept"] if model_mapped_sdf.fit_intercept else []) + \
                [f"x{j}" for j in range(p)]
        return _frame(S, v, st, num_partitions or K, columns)
    if isinstance(model_mapped_sdf, (list, tuple)):
        model_mapped_sdf = pd.concat(list(model_mapped_sdf), axis=0, ignore_index=True)
    df = model_mapped_sdf
    grouped = df.groupby("par_id").sum().sort_index()          # dlsa.py:30-34
    if grouped.shape[0] == 0:
        raise Exception("Zero-length grouped pandas DataFrame obtained, check the input.")
    p = grouped.shape[0]
    K = num_partitions if num_partitions is not None else len(df) // p
    S = grouped.iloc[:, 2:].to_numpy(dtype=np.float64)
    v = grouped["Sig_invMcoef"].to_numpy(dtype=np.float64)
    st = grouped["coef"].to_numpy(dtype=np.float64)
    return _frame(S, v, st, K, list(df.columns[3:]) if columns is None else columns)


def dlsa(Sig_inv_, beta_, sample_size, fit_intercept=False, type="lasso"):
    """Distributed Least Squares Approximation selection step (dlsa/dlsa.py:70).

    Runs the LSA path on (Sig_inv_, beta_) and returns the frame
    ``{beta_byAIC, beta_byBIC}`` (BIC here is the paper's DBIC with
    n = sample_size).  With ``fit_intercept`` the intercept (entry 0) is
    restored as ``beta0 + beta_[0]`` (dlsa.py:88-95).  ``type`` defaults to
    "lasso", the first choice of the R ``lars.lsa`` signature the reference
    calls without a type argument (dlsa.py:77-80).
    """
    import pandas as pd

    from .lsa import lars_lsa

    b = np.asarray(beta_, dtype=np.float64).reshape(-1)
    fit = lars_lsa(np.asarray(Sig_inv_, dtype=np.float64), b, intercept=fit_intercept,
                   n=sample_size, type=type)
    ia = int(np.argmin(fit["AIC"]))
    ib = int(np.argmin(fit["BIC"]))
    beta = fit["beta"]
    if fit_intercept:
        beta0 = fit["beta0"] + b[0]
        b_aic = np.hstack([beta0[ia], beta[ia, :]])
        b_bic = np.hstack([beta0[ib], beta[ib, :]])
    else:
        b_aic = beta[ia, :]
        b_bic = beta[ib, :]
    return pd.DataFrame({"beta_byAIC": b_aic, "beta_byBIC": b_bic})
