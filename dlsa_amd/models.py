"""Map stage of DLSA on MI355X: per-partition logistic fits.

Drop-in for dlsa/models.py of the reference (Vicky-Lamperouge/dlsa):

* ``simulate_logistic``      -- models.py:6-40 (same legacy-RNG stream);
* ``logistic_model``         -- models.py:42-147, same signature and output
  frame; the fit itself runs on the GPU through ``logistic_model_batched``;
* ``logistic_model_batched`` -- K partitions in one batched Newton/IRLS run
  (the Spark ``groupby("partition_id").apply(udf)`` of
  projects/logistic_dlsa.py:314-325, without Spark);
* ``simulate_logistic_device`` -- synthetic data generated directly in HBM.

There is no CPU implementation of the fit: without libdlsa_hip.so or a GPU
these functions raise ``DlsaHipError``.
"""

from __future__ import annotations

import ctypes
import warnings
from dataclasses import dataclass, field

import numpy as np

from . import _hip
from ._hip import DlsaHipError

try:  # torch is the HBM allocator / stream provider only
    import torch
except ImportError:  # pragma: no cover
    torch = None


# ---------------------------------------------------------------------------
# device helpers
# ---------------------------------------------------------------------------


def _require_gpu(device=None):
    if torch is None or not torch.cuda.is_available():
        raise DlsaHipError(
            "no ROCm GPU visible: the DLSA map stage runs only as HIP kernels on "
            "MI355X; there is no CPU fallback")
    _hip.load()
    return torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _dev_f64(a, device):
    if isinstance(a, torch.Tensor):
        t = a.to(device=device, dtype=torch.float64)
    else:
        t = torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).to(device)
    return t.contiguous()


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


# ---------------------------------------------------------------------------
# synthetic data
# ---------------------------------------------------------------------------


def simulate_logistic(sample_size, p, partition_method, partition_num):
    """Simulate data based on the logistic model (dlsa/models.py:6-40).

    Same draws as the reference for the same ``np.random.seed``: ``rand(n, p)``
    then one Bernoulli draw per row in row order (the reference's per-row
    ``binomial(n=1, p=prob[i], size=1)`` loop, models.py:28-30, consumes the
    legacy stream exactly like one vectorised call).  Unlike the reference the
    frame is built once (the reference rebuilds it inside the row loop,
    models.py:37-38, which is O(n^2)).
    """
    import pandas as pd

    if partition_method != "systematic":
        raise Exception("No such partition method implemented!")
    n = int(sample_size)
    n_true = int(p * 0.4)
    coef_true = np.zeros((p, 1))
    coef_true[:n_true] = 1.0
    feats = np.random.rand(n, p) - 0.5
    prob = 1 / (1 + np.exp(-feats.dot(coef_true)))
    label = np.random.binomial(1, prob[:, 0])
    pid = np.arange(n) % partition_num
    data = np.column_stack([pid.astype(np.float64), label.astype(np.float64), feats])
    return pd.DataFrame(data, columns=["partition_id", "label"] + [f"x{i}" for i in range(p)])


def simulate_logistic_device(n, p, seed=2019, row0=0, device=None):
    """Synthetic logistic data written straight into HBM:
    X[i, j] ~ U(-1/2, 1/2), beta* = 1 on the first floor(0.4 p) columns,
    y ~ Bernoulli(sigmoid(X beta*)), from counter-based streams (seed, row0 +
    i).  Returns (X [n, p] fp64, y [n] fp64) on ``device``."""
    dev = _require_gpu(device)
    X = torch.empty((int(n), int(p)), dtype=torch.float64, device=dev)
    y = torch.empty((int(n),), dtype=torch.float64, device=dev)
    lib = _hip.load()
    _hip.check(lib.dlsa_simulate_logistic(_ptr(X), _ptr(y), int(n), int(p), int(seed) & (2**64 - 1),
                                          int(row0), _stream(dev)), "dlsa_simulate_logistic")
    return X, y


#: airline-like design of BASELINE config 3: numeric columns + dummy-coded
#: factors (levels per factor; the first level of each is the dropped baseline,
#: models.py:65-69 with ``dummy_factors_baseline``) -> 9 + 11 + 6 + 19 + 68 + 68
#: = 181 columns, 182 parameters with the intercept.
AIRLINE_NUMERIC = 9
AIRLINE_FACTORS = (12, 7, 20, 69, 69)  # Month, DayOfWeek, UniqueCarrier, Origin, Dest


def simulate_categorical(n, seed=2019, numeric=AIRLINE_NUMERIC, factors=AIRLINE_FACTORS,
                         device=None):
    """Synthetic airline-like logistic data (BASELINE config 3) in the
    categorical-code layout, generated with torch ops on ``device`` ("cpu"
    allowed: test and baseline plumbing).

    ``numeric`` U(-1/2, 1/2) columns and, per factor with L levels, a uint8 code
    skewed towards low levels (code = floor(L u^2), like airport and carrier
    frequencies; code 0 is the baseline level).  y ~ Bernoulli(sigmoid(-0.3 +
    x beta*_num + sum_f beta*_f[code_f])) with beta*_num ~ U(-1, 1) and dummy
    effects ~ 0.3 N(0, 1) (fixed by ``seed``; the rows by ``seed`` too).
    Returns (Xn [n, numeric] fp64, codes [n, F] uint8, y [n] fp64, levels
    [F] int32 numpy); fit with ``fit_intercept=True``."""
    dev = torch.device(device) if device is not None else torch.device("cuda")
    n = int(n)
    D = sum(L - 1 for L in factors)
    gb = torch.Generator(device="cpu").manual_seed(int(seed) ^ 0x5EED)
    beta = torch.cat([torch.rand(numeric, generator=gb, dtype=torch.float64) * 2 - 1,
                      0.3 * torch.randn(D, generator=gb, dtype=torch.float64)]).to(dev)
    g = torch.Generator(device=dev).manual_seed(int(seed))
    Xn = torch.rand((n, numeric), generator=g, dtype=torch.float64, device=dev) - 0.5
    codes = torch.empty((n, len(factors)), dtype=torch.uint8, device=dev)
    eta = Xn @ beta[:numeric] - 0.3
    col = numeric
    for f, L in enumerate(factors):
        u = torch.rand((n,), generator=g, dtype=torch.float64, device=dev)
        code = torch.clamp((L * u * u).long(), max=L - 1)
        codes[:, f] = code.to(torch.uint8)
        eff = torch.cat([torch.zeros(1, dtype=torch.float64, device=dev), beta[col:col + L - 1]])
        eta = eta + eff[code]
        col += L - 1
    y = (torch.rand((n,), generator=g, dtype=torch.float64, device=dev) < torch.sigmoid(eta)).double()
    return Xn, codes, y, np.asarray(factors, dtype=np.int32)


def expand_categorical(Xn, codes, levels):
    """Dense dummy design [n, q + sum(L_f - 1)] of a categorical-code layout
    (the columns pd.get_dummies + the baseline drop of models.py:62-69 give).
    Works on torch tensors (any device) -- the dense baseline layout, not the
    product path."""
    n, q = Xn.shape
    levels = [int(L) for L in levels]
    X = torch.zeros((n, q + sum(L - 1 for L in levels)), dtype=torch.float64, device=Xn.device)
    X[:, :q] = Xn
    rows = torch.arange(n, device=Xn.device)
    col = q
    for f, L in enumerate(levels):
        c = codes[:, f].long()
        m = c > 0
        X[rows[m], col + c[m] - 1] = 1.0
        col += L - 1
    return X


def simulate_dummy_design(n, seed=2019, numeric=AIRLINE_NUMERIC, factors=AIRLINE_FACTORS,
                          device=None):
    """The same data as ``simulate_categorical`` as a dense dummy-coded design
    (the reference's layout after models.py:56-91).  Returns (X [n, p] fp64,
    y [n] fp64); fit it with ``fit_intercept=True``."""
    Xn, codes, y, levels = simulate_categorical(n, seed, numeric, factors, device)
    return expand_categorical(Xn, codes, levels), y


def encode_categorical(sample_df, Y_name, dummy_info, dummy_factors_baseline=()):
    """Categorical-code layout of one data chunk with the reference's dummy
    semantics (dlsa/models.py:56-91): dropped levels -> "000_OTHERS"
    (models.py:59), one column per sorted selected dummy name except the
    baselines (models.py:66-79), numeric columns sorted by name (models.py:70).

    Returns a dict: ``Xn`` [n, q] fp64, ``codes`` [n, F] uint8 (0 = baseline),
    ``levels`` [F] int32 (= dummy columns + 1), ``numeric`` / ``cols`` (the
    reference's column names, intercept excluded), ``unknown`` (a value outside
    the selected and baseline names: the reference's column-set check fails,
    models.py:84), ``unknown_rows`` ([n] bool: the rows holding such a value)
    and ``counts`` (rows per dummy column)."""
    factors = list(dummy_info["factor_selected"].keys())
    dropped = {k: v for k, v in dummy_info["factor_dropped"].items() if len(v) > 0}
    df = sample_df.replace(dropped, "000_OTHERS") if dropped else sample_df
    numeric = sorted(set(df.columns.drop(["partition_id", Y_name])) - set(factors))
    base = set(dummy_factors_baseline)
    n = len(df)
    codes = np.zeros((n, len(factors)), dtype=np.uint8)
    levels = np.zeros(len(factors), dtype=np.int32)
    cols = list(numeric)
    unknown = False
    unknown_rows = np.zeros(n, dtype=bool)
    counts = []
    for fi, f in enumerate(factors):
        names = [c for c in sorted(dummy_info["factor_selected_names"][f]) if c not in base]
        if len(names) > 255:
            raise ValueError(f"factor {f}: {len(names)} dummy columns > 255 (uint8 codes)")
        lut = {nm: j + 1 for j, nm in enumerate(names)}
        for b in base:
            if b.startswith(f + "_"):
                lut.setdefault(b, 0)
        import pandas as pd

        inv, uniq = pd.factorize(df[f], sort=False)  # one name per distinct value
        # a missing value (factorize code -1) has no dummy column in
        # pd.get_dummies (dummy_na=False): all-zero block = code 0
        mapped = np.array([lut.get(f"{f}_{u}", -1) for u in uniq] + [0], dtype=np.int64)
        c = mapped[inv] if n else np.zeros(0, dtype=np.int64)
        if (c < 0).any():
            unknown = True
            unknown_rows |= c < 0
            c = np.where(c < 0, 0, c)
        codes[:, fi] = c
        levels[fi] = len(names) + 1
        counts.append(np.bincount(c, minlength=len(names) + 1)[1:])
        cols.extend(names)
    Xn = np.ascontiguousarray(df[numeric].to_numpy(dtype=np.float64)) if numeric else \
        np.zeros((n, 0), dtype=np.float64)
    return {"Xn": Xn, "codes": codes, "levels": levels, "numeric": numeric, "cols": cols,
            "unknown": unknown, "unknown_rows": unknown_rows,
            "counts": np.concatenate(counts) if counts else np.zeros(0, dtype=np.int64)}


def partition_offsets(partition_id, num_partitions=None):
    """Group rows by partition id: returns (order, offsets) so that rows
    ``order[offsets[k]:offsets[k+1]]`` are partition k in their original order
    (what Spark's repartition + groupby hand to each UDF call,
    projects/logistic_dlsa.py:303-325)."""
    pid = np.asarray(partition_id).astype(np.int64)
    K = int(num_partitions) if num_partitions is not None else (int(pid.max()) + 1 if pid.size else 0)
    order = np.argsort(pid, kind="stable")
    offsets = np.zeros(K + 1, dtype=np.int64)
    np.cumsum(np.bincount(pid, minlength=K), out=offsets[1:])
    return order, offsets


# ---------------------------------------------------------------------------
# batched fit (the hot path)
# ---------------------------------------------------------------------------


@dataclass
class BatchedFit:
    """Result of one batched fit; tensors live in HBM."""
    theta: "torch.Tensor"          # [K, P]  coef (intercept first)
    sig_inv: "torch.Tensor"        # [K, P, P] X^T W X at theta
    sig_inv_theta: "torch.Tensor"  # [K, P]  Sig_inv @ theta
    loglik: "torch.Tensor"         # [K]
    iters: "torch.Tensor"          # [K] int32
    status: "torch.Tensor"         # [K] int32 (0 ok, 1 maxiter, 2 singular, 3 empty, 4 nonfinite)
    offsets: np.ndarray            # [K+1] host
    fit_intercept: bool
    stats: dict = field(default_factory=dict)

    @property
    def K(self):
        return int(self.theta.shape[0])

    @property
    def P(self):
        return int(self.theta.shape[1])

    @property
    def n_rows(self):
        return int(self.offsets[-1])

    def status_counts(self):
        s = self.status.cpu().numpy()
        return {_hip.STATUS_NAMES.get(int(v), str(v)): int((s == v).sum()) for v in np.unique(s)}


def logistic_model_batched(X, y, offsets, fit_intercept=False, center=None, scale=None,
                           max_iter=100, tol=1e-10, hessian="mixed", switch_tol=1e-6,
                           record_timing=False, rows_per_chunk=0, workspace=None,
                           device=None, exact="auto", exact_waves=0, oz_max_bytes=0):
    """Fit K row partitions at once on the GPU (batched Newton/IRLS).

    Per partition k (rows ``offsets[k]:offsets[k+1]`` of X) this computes what
    ``logistic_model`` returns for one Spark group (models.py:94-131): the
    unpenalised MLE ``theta_k`` (intercept first when ``fit_intercept``),
    ``Sig_inv_k = X_k^T diag(p(1-p)) X_k`` at theta_k and
    ``Sig_inv_k theta_k``.  ``center``/``scale`` standardise the columns like
    models.py:99-101.

    X: [n, p] fp64 (torch tensor on the GPU, or array-like, copied once);
    y: [n] 0/1; offsets: K+1 host ints.  ``hessian`` = "mixed" (bf16-MFMA
    Hessian until the Newton step is below ``switch_tol``, then fp64-MFMA
    passes; the gradient and the returned Sig_inv are always fp64),
    "mixed_f32" (fp32-MFMA approximate Hessian) or "fp64".  ``exact`` =
    "auto" (the exact pass that publishes Sig_inv on the int8 matrix cores,
    as int8 digit slices, wherever it applies; ~1e-12 per entry) or "fp64"
    (fp64 MFMA); ``exact_waves`` (0, 1, 2) the fp64 exact pass's geometry
    for P <= 128 and ``oz_max_bytes`` a cap on the wide path's int8 digit
    records (include/dlsa_hip.h, dlsa_fit_options).
    """
    dev = _require_gpu(device)
    Xd = _dev_f64(X, dev)
    yd = _dev_f64(y, dev).reshape(-1)
    if Xd.dim() != 2:
        raise ValueError("X must be 2-D [n, p]")
    n, p = Xd.shape
    offs = np.ascontiguousarray(np.asarray(offsets, dtype=np.int64))
    K = offs.size - 1
    if K < 1 or offs[0] != 0 or offs[-1] != n or np.any(np.diff(offs) < 0):
        raise ValueError("offsets must be non-decreasing, start at 0 and end at n")
    if yd.numel() != n:
        raise ValueError("y must have n entries")
    P = p + (1 if fit_intercept else 0)
    if P > _hip.MAX_P:
        raise DlsaHipError(f"P = {P} > {_hip.MAX_P} is not supported")
    cd = sd = None
    if center is not None or scale is not None:
        cd = _dev_f64(center, dev).reshape(-1)
        sd = _dev_f64(scale, dev).reshape(-1)
        if cd.numel() != p or sd.numel() != p:
            raise ValueError("center/scale must have p entries")
    theta = torch.empty((K, P), dtype=torch.float64, device=dev)
    sig = torch.empty((K, P, P), dtype=torch.float64, device=dev)
    sigt = torch.empty((K, P), dtype=torch.float64, device=dev)
    ll = torch.empty((K,), dtype=torch.float64, device=dev)
    iters = torch.empty((K,), dtype=torch.int32, device=dev)
    status = torch.empty((K,), dtype=torch.int32, device=dev)

    lib = _hip.load()
    opt = _hip.default_options()
    opt.hessian_mode = {"mixed": _hip.HESSIAN_MIXED, "fp64": _hip.HESSIAN_FP64,
                        "mixed_f32": _hip.HESSIAN_MIXED_F32}[hessian]
    opt.switch_tol = float(switch_tol)
    opt.record_timing = 1 if record_timing else 0
    opt.rows_per_chunk = int(rows_per_chunk)
    opt.exact_pass = {"auto": _hip.EXACT_AUTO, "fp64": _hip.EXACT_FP64}[exact]
    opt.exact_waves = int(exact_waves)
    opt.oz_max_bytes = int(oz_max_bytes)
    offs_p = offs.ctypes.data_as(ctypes.c_void_p)
    need = lib.dlsa_logistic_workspace_bytes(offs_p, K, p, int(bool(fit_intercept)),
                                             opt.rows_per_chunk)
    if need < 0:
        raise DlsaHipError(_hip.last_error())
    if workspace is None or workspace.numel() < need:
        workspace = torch.empty((max(int(need), 1),), dtype=torch.uint8, device=dev)
    opt.workspace = workspace.data_ptr()
    opt.workspace_bytes = workspace.numel()
    rc = lib.dlsa_logistic_fit_batched_ex(
        _ptr(Xd), _ptr(yd), offs_p, K, p, int(bool(fit_intercept)), _ptr(cd), _ptr(sd),
        int(max_iter), float(tol), _ptr(theta), _ptr(sig), _ptr(sigt), _ptr(ll), _ptr(iters),
        _ptr(status), ctypes.byref(opt), _stream(dev))
    _hip.check(rc, "dlsa_logistic_fit_batched_ex")
    stats = _hip.last_fit_stats()
    stats["workspace_bytes"] = int(need)
    return BatchedFit(theta, sig, sigt, ll, iters, status, offs, bool(fit_intercept), stats)


def logistic_model_batched_categorical(Xn, codes, y, offsets, levels, fit_intercept=False,
                                       center=None, scale=None, max_iter=100, tol=1e-10,
                                       record_timing=False, rows_per_chunk=0, zero_partitions=None,
                                       device=None):
    """Batched local logistic fit on the categorical-code layout (the dummy
    branch of dlsa/models.py:56-91, BASELINE config 3) without materialising
    the dummy matrix: the one-hot blocks of X^T W X are LDS histograms in the
    HIP pass (``dlsa_logistic_fit_categorical``).

    Xn: [n, q] fp64 numeric columns; codes: [n, F] uint8 level codes (0 =
    baseline, c = dummy column c of the factor); levels: F ints (dummy columns
    + 1); ``center``/``scale`` [q] standardise the numeric columns only
    (models.py:99-101).  Parameters: [intercept] [numeric] [factor 0 dummies]
    ...  A partition with a dummy column that has no rows gets status
    "missing_level" and all-zero outputs (the reference's zero frame), and so
    does every partition listed in ``zero_partitions`` (the partitions holding
    a factor value outside dummy_info, ``read_csv_partitioned``'s
    ``zero_partitions``: the reference's column-set check fails there too,
    models.py:84-91)."""
    dev = _require_gpu(device)
    Xd = _dev_f64(Xn, dev)
    if Xd.dim() != 2:
        raise ValueError("Xn must be 2-D [n, q]")
    n, q = Xd.shape
    if isinstance(codes, torch.Tensor):
        cd8 = codes.to(device=dev, dtype=torch.uint8).contiguous()
    else:
        cd8 = torch.from_numpy(np.ascontiguousarray(np.asarray(codes, dtype=np.uint8))).to(dev)
    if cd8.dim() != 2 or cd8.shape[0] != n:
        raise ValueError("codes must be [n, F]")
    F = cd8.shape[1]
    lv = np.ascontiguousarray(np.asarray(levels, dtype=np.int32).reshape(-1))
    if lv.size != F:
        raise ValueError("levels must have F entries")
    yd = _dev_f64(y, dev).reshape(-1)
    offs = np.ascontiguousarray(np.asarray(offsets, dtype=np.int64))
    K = offs.size - 1
    if K < 1 or offs[0] != 0 or offs[-1] != n or np.any(np.diff(offs) < 0) or yd.numel() != n:
        raise ValueError("offsets must be non-decreasing, start at 0 and end at n; y has n rows")
    P = int(bool(fit_intercept)) + q + int((lv - 1).sum())
    cen = sca = None
    if center is not None or scale is not None:
        cen = _dev_f64(center, dev).reshape(-1)
        sca = _dev_f64(scale, dev).reshape(-1)
        if cen.numel() != q or sca.numel() != q:
            raise ValueError("center/scale must have q entries (numeric columns)")
    theta = torch.empty((K, P), dtype=torch.float64, device=dev)
    sig = torch.empty((K, P, P), dtype=torch.float64, device=dev)
    sigt = torch.empty((K, P), dtype=torch.float64, device=dev)
    ll = torch.empty((K,), dtype=torch.float64, device=dev)
    iters = torch.empty((K,), dtype=torch.int32, device=dev)
    status = torch.empty((K,), dtype=torch.int32, device=dev)
    lib = _hip.load()
    opt = _hip.default_options()
    opt.record_timing = 1 if record_timing else 0
    opt.rows_per_chunk = int(rows_per_chunk)
    rc = lib.dlsa_logistic_fit_categorical(
        _ptr(Xd), _ptr(cd8), _ptr(yd), offs.ctypes.data_as(ctypes.c_void_p), K, q, F,
        lv.ctypes.data_as(ctypes.c_void_p), int(bool(fit_intercept)), _ptr(cen), _ptr(sca),
        int(max_iter), float(tol), _ptr(theta), _ptr(sig), _ptr(sigt), _ptr(ll), _ptr(iters),
        _ptr(status), ctypes.byref(opt), _stream(dev))
    _hip.check(rc, "dlsa_logistic_fit_categorical")
    stats = _hip.last_fit_stats()
    if zero_partitions is not None and len(zero_partitions):
        idx = torch.as_tensor(np.asarray(zero_partitions, dtype=np.int64), device=dev)
        for t in (theta, sig, sigt, ll):
            t[idx] = 0
        status[idx] = 5
    return BatchedFit(theta, sig, sigt, ll, iters, status, offs, bool(fit_intercept), stats)


def ols_model_batched(X, y, offsets, fit_intercept=False, center=None, scale=None,
                      rows_per_chunk=0, record_timing=False, device=None, exact_waves=0):
    """Batched local OLS (linear DLSA path): per
    partition theta_k = (X_k^T X_k)^-1 X_k^T y_k and Sig_inv_k = X_k^T X_k from
    one fused fp64 pass.  Returns a BatchedFit whose ``loglik`` field holds the
    residual sum of squares of each partition."""
    dev = _require_gpu(device)
    Xd = _dev_f64(X, dev)
    yd = _dev_f64(y, dev).reshape(-1)
    n, p = Xd.shape
    offs = np.ascontiguousarray(np.asarray(offsets, dtype=np.int64))
    K = offs.size - 1
    if K < 1 or offs[0] != 0 or offs[-1] != n or np.any(np.diff(offs) < 0) or yd.numel() != n:
        raise ValueError("offsets must be non-decreasing, start at 0 and end at n; y has n rows")
    P = p + (1 if fit_intercept else 0)
    if P > _hip.MAX_P:
        raise DlsaHipError(f"P = {P} > {_hip.MAX_P} is not supported")
    cd = sd = None
    if center is not None or scale is not None:
        cd = _dev_f64(center, dev).reshape(-1)
        sd = _dev_f64(scale, dev).reshape(-1)
    theta = torch.empty((K, P), dtype=torch.float64, device=dev)
    sig = torch.empty((K, P, P), dtype=torch.float64, device=dev)
    sigt = torch.empty((K, P), dtype=torch.float64, device=dev)
    rss = torch.empty((K,), dtype=torch.float64, device=dev)
    status = torch.empty((K,), dtype=torch.int32, device=dev)
    lib = _hip.load()
    opt = _hip.default_options()
    opt.rows_per_chunk = int(rows_per_chunk)
    opt.record_timing = 1 if record_timing else 0
    opt.exact_waves = int(exact_waves)
    rc = lib.dlsa_ols_fit_batched(_ptr(Xd), _ptr(yd), offs.ctypes.data_as(ctypes.c_void_p), K, p,
                                  int(bool(fit_intercept)), _ptr(cd), _ptr(sd), _ptr(theta),
                                  _ptr(sig), _ptr(sigt), _ptr(rss), _ptr(status),
                                  ctypes.byref(opt), _stream(dev))
    _hip.check(rc, "dlsa_ols_fit_batched")
    iters = torch.ones((K,), dtype=torch.int32, device=dev)
    return BatchedFit(theta, sig, sigt, rss, iters, status, offs, bool(fit_intercept),
                      _hip.last_fit_stats())


def logistic_loglik_batched(X, y, offsets, betas, fit_intercept=False, center=None, scale=None,
                            device=None):
    """Per-partition log-likelihood of candidate coefficient vectors in one
    pass over X (the evaluation step of dlsa/models.py:151-225 /
    dlsa/model_eval.py:10-42).  betas: [B, P] (B <= 16), intercept first.
    Returns a [K, B] fp64 tensor on the device."""
    dev = _require_gpu(device)
    Xd = _dev_f64(X, dev)
    yd = _dev_f64(y, dev).reshape(-1)
    n, p = Xd.shape
    offs = np.ascontiguousarray(np.asarray(offsets, dtype=np.int64))
    K = offs.size - 1
    if K < 1 or offs[0] != 0 or offs[-1] != n or np.any(np.diff(offs) < 0) or yd.numel() != n:
        raise ValueError("offsets must be non-decreasing, start at 0 and end at n; y has n rows")
    bd = _dev_f64(betas, dev)
    if bd.dim() == 1:
        bd = bd.reshape(1, -1)
    B, P = bd.shape
    if P != p + (1 if fit_intercept else 0):
        raise ValueError("betas must have P = p + fit_intercept columns")
    cd = sd = None
    if center is not None or scale is not None:
        cd = _dev_f64(center, dev).reshape(-1)
        sd = _dev_f64(scale, dev).reshape(-1)
    out = torch.empty((K, B), dtype=torch.float64, device=dev)
    lib = _hip.load()
    rc = lib.dlsa_logistic_loglik_batched(_ptr(Xd), _ptr(yd), offs.ctypes.data_as(ctypes.c_void_p),
                                          K, p, int(bool(fit_intercept)), _ptr(cd), _ptr(sd),
                                          _ptr(bd), B, _ptr(out), _stream(dev))
    _hip.check(rc, "dlsa_logistic_loglik_batched")
    return out


# ---------------------------------------------------------------------------
# reference-signature wrapper (one Spark group)
# ---------------------------------------------------------------------------


def _describe_row(data_info, col, row):
    # Spark DataFrame.describe().toPandas(): rows count/mean/stddev/min/max,
    # values as strings (models.py:99-101 reads rows 1 and 2)
    return float(data_info[col][row])


def _design(sample_df, Y_name, dummy_info, dummy_factors_baseline):
    """Host-side design matrix of one partition, models.py:56-104.  Returns
    (x_train DataFrame, usecols_x0 numeric columns, usecols_x all columns,
    zero_frame_or_None)."""
    import pandas as pd

    if len(dummy_info) > 0:
        factors = list(dummy_info["factor_selected"].keys())
        dropped = {k: v for k, v in dummy_info["factor_dropped"].items() if len(v) > 0}
        df = sample_df.replace(dropped, "000_OTHERS")
        wide = pd.get_dummies(data=df, drop_first=False, columns=factors, sparse=True)
        x_train = wide.drop(["partition_id", Y_name] + list(dummy_factors_baseline), axis=1)
        numeric = sorted(set(df.columns.drop(["partition_id", Y_name])) - set(factors))
        cols = list(numeric)
        for f in factors:
            cols.extend(sorted(dummy_info["factor_selected_names"][f]))
        cols = [c for c in cols if c not in dummy_factors_baseline]
        if set(x_train.columns) != set(cols):
            return x_train, numeric, cols, True
        return x_train, numeric, cols, False
    x_train = sample_df.drop(["partition_id", Y_name] + list(dummy_factors_baseline), axis=1)
    return x_train, list(x_train.columns), list(x_train.columns), False


def _logistic_model_codes(sample_df, Y_name, fit_intercept, dummy_info, dummy_factors_baseline,
                          data_info):
    """Dummy branch of logistic_model on the categorical-code layout (no dense
    dummy matrix).  None when the design exceeds the kernel's limits (F <= 16
    factors, intercept + numeric <= 16, P <= 192): the caller then builds the
    dense design."""
    import pandas as pd

    icpt = ["intercept"] if fit_intercept else []
    enc = encode_categorical(sample_df, Y_name, dummy_info, dummy_factors_baseline)
    q, F = enc["Xn"].shape[1], enc["codes"].shape[1]
    P = len(icpt) + len(enc["cols"])
    if F > 16 or len(icpt) + q > 16 or P > _hip.MAX_P_FUSED:
        return None
    cols = enc["cols"]
    if enc["unknown"] or (enc["counts"] == 0).any():
        absent = [c for c, m in zip(cols[q:], enc["counts"]) if m == 0]
        warnings.warn("Dummies:" + str(set(absent)) + "missing in this data chunk "
                      + str((len(sample_df), len(cols))) + "Skip modeling this part of data.")
        return pd.DataFrame(0, index=np.arange(P),
                            columns=["par_id", "coef", "Sig_invMcoef"] + icpt + cols)
    center = scale = None
    if len(data_info) > 0 and q > 0:
        center = np.array([_describe_row(data_info, c, 1) for c in enc["numeric"]])
        scale = np.array([_describe_row(data_info, c, 2) for c in enc["numeric"]])
    y = np.asarray(sample_df[Y_name], dtype=np.float64)
    fit = logistic_model_batched_categorical(enc["Xn"], enc["codes"], y, np.array([0, y.size]),
                                             enc["levels"], fit_intercept=fit_intercept,
                                             center=center, scale=scale)
    coef = fit.theta[0].cpu().numpy()
    sig = fit.sig_inv[0].cpu().numpy()
    sigt = fit.sig_inv_theta[0].cpu().numpy()
    out = pd.DataFrame(np.column_stack([coef, sigt, sig]),
                       columns=pd.Index(["coef", "Sig_invMcoef"] + icpt + cols))
    out.insert(0, "par_id", np.arange(P))
    if out.isna().values.any():
        warnings.warn("NAs appear in the final output")
    return out


def logistic_model(sample_df, Y_name, fit_intercept=False, dummy_info=[], dummy_factors_baseline=[],
                   data_info=[]):
    """Run the logistic model on one partition (dlsa/models.py:42-147).

    Same inputs and the same p x (p+3) output frame as the reference:
    ``par_id | coef | Sig_invMcoef | <Sig_inv columns>``, intercept first.
    A partition that lacks a selected dummy level returns the reference's
    all-zero frame (models.py:84-91).  The estimate is the converged MLE (the
    reference stops sklearn at its default tol=1e-4); the fit runs on the GPU.
    """
    import pandas as pd

    icpt = ["intercept"] if fit_intercept else []
    if len(dummy_info) > 0:
        out = _logistic_model_codes(sample_df, Y_name, fit_intercept, dummy_info,
                                    dummy_factors_baseline, data_info)
        if out is not None:
            return out
    x_train, numeric, cols, missing = _design(sample_df, Y_name, dummy_info, dummy_factors_baseline)
    if missing:
        warnings.warn("Dummies:" + str(set(cols) - set(x_train.columns))
                      + "missing in this data chunk " + str(x_train.shape)
                      + "Skip modeling this part of data.")
        return pd.DataFrame(0, index=np.arange(len(icpt + cols)),
                            columns=["par_id", "coef", "Sig_invMcoef"] + icpt + cols)
    x_train = x_train.reindex(columns=cols)
    X = np.ascontiguousarray(x_train.to_numpy(dtype=np.float64))
    y = np.asarray(sample_df[Y_name], dtype=np.float64)
    center = scale = None
    if len(data_info) > 0:
        center = np.zeros(len(cols))
        scale = np.ones(len(cols))
        for j, c in enumerate(cols):
            if c in numeric:
                center[j] = _describe_row(data_info, c, 1)
                scale[j] = _describe_row(data_info, c, 2)
    fit = logistic_model_batched(X, y, np.array([0, X.shape[0]]), fit_intercept=fit_intercept,
                                 center=center, scale=scale)
    coef = fit.theta[0].cpu().numpy()
    sig = fit.sig_inv[0].cpu().numpy()
    sigt = fit.sig_inv_theta[0].cpu().numpy()
    P = coef.size
    out = pd.DataFrame(np.column_stack([coef, sigt, sig]),
                       columns=pd.Index(["coef", "Sig_invMcoef"] + icpt + cols))
    out.insert(0, "par_id", np.arange(P))
    if out.isna().values.any():
        warnings.warn("NAs appear in the final output")
    return out


def logistic_model_eval(sample_df, Y_name, par, fit_intercept=False, dummy_info=[],
                        dummy_factors_baseline=[], data_info=[]):
    """Log-likelihood of each coefficient column of ``par`` on one partition
    (dlsa/models.py:151-225).  ``par`` is a P-row DataFrame (one column per
    method, e.g. beta_byAIC / beta_byBIC / beta_byOLS / beta_byONESHOT).
    Returns a one-row DataFrame with the same columns.  A partition missing a
    dummy level is evaluated with that dummy column set to 0, as the
    reference does (models.py:185-193).  The pass runs on the GPU."""
    import pandas as pd

    x_train, numeric, cols, missing = _design(sample_df, Y_name, dummy_info, dummy_factors_baseline)
    if missing:
        warnings.warn("Dummies:" + str(set(cols) - set(x_train.columns))
                      + "missing in this data chunk " + str(x_train.shape))
    x_train = x_train.reindex(columns=cols, fill_value=0)
    X = np.ascontiguousarray(x_train.to_numpy(dtype=np.float64))
    y = np.asarray(sample_df[Y_name], dtype=np.float64)
    center = scale = None
    if len(data_info) > 0:
        center = np.zeros(len(cols))
        scale = np.ones(len(cols))
        for j, c in enumerate(cols):
            if c in numeric:
                center[j] = _describe_row(data_info, c, 1)
                scale[j] = _describe_row(data_info, c, 2)
    betas = np.ascontiguousarray(np.asarray(par, dtype=np.float64).T)
    ll = logistic_loglik_batched(X, y, np.array([0, X.shape[0]]), betas,
                                 fit_intercept=fit_intercept, center=center, scale=scale)
    return pd.DataFrame(ll.cpu().numpy(), columns=list(par.columns))
