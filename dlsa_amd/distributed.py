"""Multi-GPU DLSA: partitions sharded over ranks, one collective.

The reference's only exchange is the Spark shuffle + collect of every
partition's p x (p+3) frame to the driver (dlsa/dlsa.py:30-34; K*p*(p+3)
doubles over the network).  Here each rank (one process per GPU) fits its own
partitions in HBM, pre-reduces them on the device into
``[sum Sig_inv | sum Sig_inv theta | sum theta | K]`` (P^2 + 2P + 1 fp64,
81.6 KB at P = 100) and ONE ``all_reduce(SUM)`` over RCCL/xGMI combines the
ranks.  Every rank then holds the global sums and can solve the WLSE and run
the LARS/DBIC path locally (dlsa/dlsa.py:44-52, :70-100).  The global row
count N (for the DBIC) rides in the same buffer: one collective in all.
"""

from __future__ import annotations

import numpy as np

from .dlsa import reduce_partitions_device, split_reduced


def combine(buf, group=None):
    """Sum the per-rank reduced buffers in place (RCCL when the process group
    backend is "nccl", gloo on CPU tensors).  No-op without a process group;
    with one (even of one rank) the all-reduce runs, so a single-GPU job under
    ``torch.distributed`` takes the same collective path as the 8-GPU one."""
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        if buf.is_cuda and dist.get_backend(group) == "gloo":
            # gloo (CPU test / fallback transport): reduce a host copy
            tmp = buf.cpu()
            dist.all_reduce(tmp, op=dist.ReduceOp.SUM, group=group)
            buf.copy_(tmp)
        else:
            dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
    return buf


def finish(S, v, sum_theta, K, n_global, fit_intercept=False, lars_type="lasso"):
    """Host tail of DLSA from the global sums: WLSE (lstsq as dlsa.py:48),
    ONESHOT (dlsa.py:51-52), LSA path and the AIC/BIC argmin (dlsa.py:83-98).
    """
    from .lsa import lars_lsa

    wlse = np.linalg.lstsq(S, v, rcond=None)[0]
    oneshot = sum_theta / K
    path = lars_lsa(S, wlse, intercept=fit_intercept, n=n_global, type=lars_type)
    ia = int(np.argmin(path["AIC"]))
    ib = int(np.argmin(path["BIC"]))
    if fit_intercept:
        b0 = path["beta0"] + wlse[0]
        b_aic = np.hstack([b0[ia], path["beta"][ia]])
        b_bic = np.hstack([b0[ib], path["beta"][ib]])
        support = np.nonzero(path["beta"][ib])[0] + 1
    else:
        b_aic = path["beta"][ia].copy()
        b_bic = path["beta"][ib].copy()
        support = np.nonzero(b_bic)[0]
    return {"wlse": wlse, "oneshot": oneshot, "beta_byAIC": b_aic, "beta_byBIC": b_bic,
            "dbic_support": support, "path": path, "Sig_inv_sum": S}


def combine_and_finish(buf, P, fit_intercept=False, lars_type="lasso", group=None):
    """The exchange step and the host tail of the sharded path: ONE
    all-reduce of this rank's ``[sum Sig_inv | sum Sig_inv theta | sum theta |
    K | N]`` buffer (P^2 + 2P + 2 fp64, the layout of
    ``reduce_partitions_device(fit, n_rows=True)``), then WLSE / ONESHOT /
    LARS / DBIC from the global sums on every rank."""
    combine(buf, group)
    b = buf.cpu().numpy() if hasattr(buf, "cpu") else np.asarray(buf)
    S, v, st, K = split_reduced(b[:-1], P)
    return finish(S, v, st, K, int(round(float(b[-1]))), fit_intercept, lars_type)


def dlsa_fit_sharded(X, y, offsets, fit_intercept=False, lars_type="lasso",
                     group=None, codes=None, levels=None, **fit_kw):
    """Fit this rank's partitions on its GPU and return the global DLSA result.

    X, y, offsets describe the LOCAL shard (rows already on this rank's
    device).  With ``codes``/``levels`` X holds the numeric columns of the
    categorical-code layout (``logistic_model_batched_categorical``).  The
    row count N of the DBIC is summed in the same single collective as the
    partition sums (reference: the shuffle + collect of dlsa/dlsa.py:30-34).
    """
    from .models import logistic_model_batched, logistic_model_batched_categorical

    if codes is not None:
        fit = logistic_model_batched_categorical(X, codes, y, offsets, levels,
                                                 fit_intercept=fit_intercept, **fit_kw)
    else:
        fit = logistic_model_batched(X, y, offsets, fit_intercept=fit_intercept, **fit_kw)
    buf = reduce_partitions_device(fit, n_rows=True)
    out = combine_and_finish(buf, fit.P, fit_intercept, lars_type, group)
    out["fit"] = fit
    return out
