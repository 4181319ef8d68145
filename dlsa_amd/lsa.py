"""LARS / adaptive lasso on the LSA quadratic form (drop-in for dlsa/lsa.py).

``lars_lsa`` keeps the reference signature and return value
(dlsa/lsa.py:90-212: dict with ``AIC``, ``BIC``, ``beta`` [steps x m] and
``beta0``).  The path is computed by native host code in libdlsa_hip.so
(``dlsa_lars_lsa``, dlsa_amd/csrc/lars_host.cpp) -- O(p^3) work on the
driver, as in the reference; it needs no GPU.
"""

from __future__ import annotations

import ctypes

import numpy as np

from . import _hip


def lars_lsa(Sigma0, b0, intercept, n, type="lar", eps=np.finfo(float).eps, max_steps=None):
    """Least Angle Regression / Lasso path for LSA (dlsa/lsa.py:90).

    Sigma0: P x P positive-definite matrix (any 2-D array; the reference
    required ``np.matrix``); b0: length-P estimate; intercept: treat entry 0 as
    an unpenalised intercept (profiled out through the Schur complement);
    n: sample size for BIC = RSS + log(n) dof; type: 'lar' or 'lasso'.
    """
    S = np.ascontiguousarray(np.asarray(Sigma0, dtype=np.float64))
    b = np.ascontiguousarray(np.asarray(b0, dtype=np.float64).reshape(-1))
    if S.ndim != 2 or S.shape[0] != S.shape[1] or S.shape[0] != b.size:
        raise ValueError("Sigma0 must be P x P and b0 length P")
    if type not in ("lar", "lasso"):
        raise ValueError("type must be 'lar' or 'lasso'")
    P = S.shape[0]
    m = P - (1 if intercept else 0)
    ms = 8 * m if max_steps is None else int(max_steps)
    beta = np.zeros((ms + 1) * m)
    beta0 = np.zeros(ms + 1)
    aic = np.zeros(ms + 1)
    bic = np.zeros(ms + 1)
    nst = ctypes.c_int32(0)
    vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    lib = _hip.load()
    rc = lib.dlsa_lars_lsa(vp(S), vp(b), P, int(bool(intercept)), float(n),
                           1 if type == "lasso" else 0, float(eps), ms, vp(beta), vp(beta0),
                           vp(aic), vp(bic), ctypes.byref(nst))
    _hip.check(rc, "dlsa_lars_lsa")
    k1 = nst.value
    return {"AIC": aic[:k1].copy(), "BIC": bic[:k1].copy(),
            "beta": beta.reshape(ms + 1, m)[:k1].copy(), "beta0": beta0[:k1].copy()}
