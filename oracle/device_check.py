"""Independent device restatement of Sig_inv for EVERY partition -- TEST
INFRASTRUCTURE ONLY (the checker, never the product).

The numpy oracle (``dlsa_oracle.logistic_fit``) refits a partition on the CPU,
which is affordable for 2 sampled partitions of a full-size config but not
for all 1024.  This module evaluates the reference's own formulas at the
product's returned coefficients, for every partition, on the GPU through
torch's fp64 library GEMM (hipBLASLt / rocBLAS) -- a code path that shares
nothing with the HIP kernels under test:

* ``predict_proba`` and the weights ``p (1 - p)``: dlsa/models.py:114;
* ``Sig_inv = X^T diag(p (1 - p)) X``: dlsa/models.py:130 (OLS: ``X^T X``);
* ``Sig_invMcoef = Sig_inv @ coef``: dlsa/models.py:131;
* the combine sums ``sum_k Sig_inv_k`` and ``sum_k Sig_inv_k coef_k`` and
  WLSE = lstsq(sum Sig_inv, sum Sig_invMcoef): dlsa/dlsa.py:30-49.

Only ``tests/`` and ``bench.py`` (after its timed region) use it.  Nothing
under ``dlsa_amd/`` imports it.
"""

from __future__ import annotations

import numpy as np


def partition_hessians(X, y, offsets, theta, family="logistic", fit_intercept=False,
                       design=None):
    """[K, P, P] fp64 on X's device: X_k^T diag(w_k) X_k with w from theta[k]
    (logistic) or w = 1 (OLS), one library GEMM per partition.

    ``design(a, b)`` (optional) returns the dense design rows [a, b) -- used
    for the categorical-code layout, whose dense dummy expansion of a whole
    full-size data set would not fit HBM.  ``fit_intercept`` prepends the
    ones column (models.py:104-108)."""
    import torch

    K = len(offsets) - 1
    P = int(theta.shape[1])
    H = torch.zeros((K, P, P), dtype=torch.float64, device=theta.device)
    for k in range(K):
        a, b = int(offsets[k]), int(offsets[k + 1])
        if b <= a:
            continue
        Xk = design(a, b) if design is not None else X[a:b]
        if fit_intercept:
            Xk = torch.cat([torch.ones((b - a, 1), dtype=Xk.dtype, device=Xk.device), Xk], 1)
        if family == "ols":
            H[k] = Xk.T @ Xk
        else:
            mu = torch.sigmoid(Xk @ theta[k])
            H[k] = Xk.T @ ((mu * (1.0 - mu))[:, None] * Xk)
    return H


def per_entry_error(S, H):
    """Per partition max_ij |S_ij - H_ij| / sqrt(H_ii H_jj) (every entry on its
    own scale, the metric of tests/test_gpu_ozaki.py).  Returns a [K] numpy
    array."""
    import torch

    d = torch.sqrt(torch.diagonal(H, dim1=1, dim2=2).abs()).clamp_min(1e-300)
    e = (S - H).abs() / (d[:, :, None] * d[:, None, :])
    return e.amax(dim=(1, 2)).cpu().numpy()


def combine_from(H, theta, mask=None):
    """The combine of dlsa/dlsa.py:30-49 on the independent matrices: returns
    (sum H_k [P, P], sum H_k theta_k [P], WLSE [P]) as numpy fp64."""
    import torch

    if mask is not None:
        H = H[mask]
        theta = theta[mask]
    S = H.sum(0)
    v = torch.einsum("kij,kj->i", H, theta)
    S, v = S.cpu().numpy(), v.cpu().numpy()
    return S, v, np.linalg.lstsq(S, v, rcond=None)[0]


def check_all_partitions(fit, X, y, family="logistic", design=None):
    """Every partition of ``fit`` against the independent restatement.
    Returns a dict: per-entry Sig_inv error (max and worst partition),
    Sig_invMcoef relative error, WLSE of the independent sums and its
    relative distance to the WLSE of the product's own sums."""
    import torch

    H = partition_hessians(X, y, fit.offsets, fit.theta, family=family,
                           fit_intercept=fit.fit_intercept, design=design)
    ok = fit.status == 0
    e = per_entry_error(fit.sig_inv, H)
    e_ok = np.where(ok.cpu().numpy(), e, 0.0)
    mt = torch.einsum("kij,kj->ki", H, fit.theta)
    st_rel = ((fit.sig_inv_theta - mt).abs().amax(1) /
              mt.abs().amax(1).clamp_min(1e-300)).cpu().numpy()
    st_rel = np.where(ok.cpu().numpy(), st_rel, 0.0)
    S_i, v_i, w_i = combine_from(H, fit.theta, ok)
    S_p = fit.sig_inv[ok].sum(0).cpu().numpy()
    v_p = fit.sig_inv_theta[ok].sum(0).cpu().numpy()
    w_p = np.linalg.lstsq(S_p, v_p, rcond=None)[0]
    return {"partitions": int(len(e)), "max_elem_err": float(e_ok.max()) if len(e) else 0.0,
            "worst_partition": int(np.argmax(e_ok)) if len(e) else -1,
            "sig_inv_theta_rel": float(st_rel.max()) if len(e) else 0.0,
            "wlse_rel": float(np.abs(w_i - w_p).max() / max(np.abs(w_i).max(), 1e-300)),
            "Ssum": S_i, "vsum": v_i, "wlse": w_i}
