"""GPU: the exact pass on the int8 matrix cores (irls_oz_impl.hpp).

In mixed mode every full-data bf16 pass records, per chunk and feature, max
|x| and max |sqrt(w) x| at the theta it saw, and the exact pass that publishes
Sig_inv (models.py:130) then forms X^T W X from int8 digit slices with exact
int32 sums, its digit exponents from that record (grown by the bound on how
far sqrt(w) can have moved since).  The same fit
with exact="fp64" (DLSA_EXACT_FP64) runs the fp64-MFMA exact pass at the SAME iterate (the bf16
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


def _elem(a, b):
    """max_ij |a_ij - b_ij| / sqrt(b_ii b_jj) over partitions [K, P, P]: the
    per-entry error on the scale of the entry's own rows and columns (a
    relative-to-the-largest-entry metric cannot see errors in small entries)."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    worst = 0.0
    for k in range(b.shape[0]):
        d = np.sqrt(np.abs(np.diagonal(b[k])))
        scale = np.outer(d, d)
        m = scale > 0
        worst = max(worst, float((np.abs(a[k] - b[k])[m] / scale[m]).max()))
    return worst


def heavy_design(kind, n, chunk=4096, seed=0, p_extra=0):
    """Designs where one digit exponent per chunk column is weakest:
    lognormal: a lognormal(0, 2) column (max/median ~ 1e3);
    outlier: a U(-1/2, 1/2) column with one 1e4 entry per `chunk` rows, whose
      coefficient 0.8 makes eta ~ 8000 there (w = 0: the row's z is 0 while
      its |x| is 2e4 times the column's others);
    separable: |eta| ~ N(0, 12^2) (median 7.6, most rows |eta| < 20: weights
      down to e^-20).
    p_extra U(-1/2, 1/2) columns with zero coefficients are appended."""
    rs = np.random.RandomState(seed)
    if kind == "lognormal":
        X = np.column_stack([rs.randn(n, 6), rs.lognormal(0.0, 2.0, n)])
        beta = np.array([0.5, -0.4, 0.3, 0.2, -0.1, 0.3, 0.05])
    elif kind == "outlier":
        c = rs.rand(n) - 0.5
        c[chunk // 2::chunk] = 1e4
        X = np.column_stack([rs.randn(n, 6), c])
        beta = np.array([0.5, -0.4, 0.3, 0.2, -0.1, 0.3, 0.8])
    else:
        X = rs.randn(n, 6)
        beta = np.array([6.0, -5.0, 4.0, 5.0, -3.0, 4.0])
    eta = X @ beta
    y = (rs.rand(n) < 1.0 / (1.0 + np.exp(-eta))).astype(np.float64)
    if p_extra:
        X = np.column_stack([X, rs.rand(n, p_extra) - 0.5])
    return X, y


def _pair(M, monkeypatch, *args, **kw):
    """The same fit with the Ozaki exact pass and with the fp64-MFMA one
    (dlsa_fit_options.exact_pass)."""
    oz = M.logistic_model_batched(*args, exact="auto", **kw)
    f64 = M.logistic_model_batched(*args, exact="fp64", **kw)
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


ELEM = 1e-10


@pytest.mark.parametrize("kind", ["lognormal", "outlier", "separable"])
@pytest.mark.parametrize("p_extra", [6, 93])
def test_ozaki_heavy_tails_per_entry(torch_cuda, M, monkeypatch, kind, p_extra):
    """Default mode, fused int8 exact pass (P = 13-14 and 100-101, NT 1 and 7):
    the designs of heavy_design against the fp64 exact pass at the same
    iterate and against the oracle, entry by entry: max |dH_ij| / sqrt(H_ii
    H_jj) < 1e-10, theta within 1e-8.  (Digit exponents from the chunk's max
    |x| / 2 -- the round-3 rule -- miss this by 5 orders of magnitude on the
    outlier column, tests/test_cpu_ozaki_numerics.py.)"""
    n, chunk = 40000, 4096
    X, y = heavy_design(kind, n, chunk=chunk, p_extra=p_extra)
    off = np.array([0, 20000, n])
    oz, f64 = _pair(M, monkeypatch, X, y, off, fit_intercept=True, rows_per_chunk=chunk)
    assert oz.stats["passes_oz"] >= 1 and f64.stats["passes_oz"] == 0
    assert (oz.status.cpu().numpy() == 0).all()
    assert _elem(oz.sig_inv.cpu(), f64.sig_inv.cpu()) < ELEM
    assert _rel(oz.theta.cpu(), f64.theta.cpu()) < 1e-12
    th, S, St, _, _ = O.logistic_fit_partitions(X, y, off, fit_intercept=True)
    assert _rel(oz.theta.cpu(), th) < REL
    assert _elem(oz.sig_inv.cpu(), S) < ELEM
    assert _rel(oz.sig_inv_theta.cpu(), St) < REL


@pytest.mark.parametrize("kind", ["lognormal", "outlier", "separable"])
def test_wide_ozaki_heavy_tails_per_entry(torch_cuda, M, monkeypatch, kind):
    """The same designs on the wide path (P = 208: row pass + int8 Gram with
    per-row-group digit exponents, wide_oz.hip)."""
    n, chunk = 24000, 4096
    X, y = heavy_design(kind, n, chunk=chunk, p_extra=200)
    off = np.array([0, 12000, n])
    oz, f64 = _pair(M, monkeypatch, X, y, off, fit_intercept=True, rows_per_chunk=chunk)
    assert oz.stats["passes_oz"] >= 1 and f64.stats["passes_oz"] == 0
    assert (oz.status.cpu().numpy() == 0).all()
    assert _elem(oz.sig_inv.cpu(), f64.sig_inv.cpu()) < ELEM
    assert _rel(oz.theta.cpu(), f64.theta.cpu()) < 1e-12
    th, S, _, _, _ = O.logistic_fit_partitions(X, y, off, fit_intercept=True)
    assert _rel(oz.theta.cpu(), th) < REL
    assert _elem(oz.sig_inv.cpu(), S) < ELEM


def _wide_problem(p, seed):
    sizes = [6000, 5001, 4000]
    X, y = O.simulate_counter(sum(sizes), p, seed=seed)
    return X, y, np.concatenate([[0], np.cumsum(sizes)])


def test_wide_ozaki_concurrent_fits_two_threads(torch_cuda, M):
    """Two wide mixed-mode fits (P = 300, then the larger P = 500) on two Python
    threads, each on its own torch stream: the digit records live in each
    fit's own workspace (no process-wide buffer), so both equal the sequential
    fits bit for bit, with the int8 Gram used in both."""
    import threading

    torch = torch_cuda
    probs = {p: _wide_problem(p, 40 + p) for p in (300, 500)}
    seq = {}
    for p, (X, y, off) in probs.items():
        seq[p] = M.logistic_model_batched(X, y, off, rows_per_chunk=2000)
        assert seq[p].stats["passes_oz"] >= 1
    Xd = {p: (torch.from_numpy(X).cuda(), torch.from_numpy(y).cuda()) for p, (X, y, _) in
          probs.items()}
    torch.cuda.synchronize()
    out, err = {}, []
    go = threading.Barrier(2)

    def run(p):
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                go.wait()
                f = M.logistic_model_batched(Xd[p][0], Xd[p][1], probs[p][2],
                                             rows_per_chunk=2000)
                s.synchronize()
                out[p] = f
        except Exception as e:  # pragma: no cover - reported below
            err.append(e)

    ts = [threading.Thread(target=run, args=(p,)) for p in (300, 500)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not err, err
    for p in (300, 500):
        assert out[p].stats["passes_oz"] >= 1
        assert torch.equal(out[p].theta, seq[p].theta)
        assert torch.equal(out[p].sig_inv, seq[p].sig_inv)
        assert torch.equal(out[p].loglik, seq[p].loglik)


def _abi_fit(torch, X, y, off, p, workspace_bytes, guard=0, pattern=0xA5, rows_per_chunk=2000,
             oz_max_bytes=0):
    """dlsa_logistic_fit_batched_ex through ctypes with a caller workspace of
    exactly `workspace_bytes` (plus `guard` bytes of `pattern` after it, or a
    NULL workspace when workspace_bytes is None)."""
    import ctypes

    from dlsa_amd import _hip

    lib = _hip.load()
    K = len(off) - 1
    Xd = torch.from_numpy(np.ascontiguousarray(X)).cuda()
    yd = torch.from_numpy(np.ascontiguousarray(y)).cuda()
    th = torch.empty(K, p, dtype=torch.float64, device="cuda")
    S = torch.empty(K, p, p, dtype=torch.float64, device="cuda")
    St = torch.empty(K, p, dtype=torch.float64, device="cuda")
    ll = torch.empty(K, dtype=torch.float64, device="cuda")
    it = torch.empty(K, dtype=torch.int32, device="cuda")
    st = torch.empty(K, dtype=torch.int32, device="cuda")
    opt = _hip.default_options()
    opt.rows_per_chunk = rows_per_chunk
    opt.oz_max_bytes = oz_max_bytes
    ws = None
    if workspace_bytes is not None:
        ws = torch.full((workspace_bytes + guard,), pattern, dtype=torch.uint8, device="cuda")
        opt.workspace = ws.data_ptr()
        opt.workspace_bytes = workspace_bytes
    offs = np.ascontiguousarray(off, dtype=np.int64)
    rc = lib.dlsa_logistic_fit_batched_ex(
        Xd.data_ptr(), yd.data_ptr(), offs.ctypes.data_as(ctypes.c_void_p), K, p, 0, None, None,
        100, 1e-10, th.data_ptr(), S.data_ptr(), St.data_ptr(), ll.data_ptr(), it.data_ptr(),
        st.data_ptr(), ctypes.byref(opt), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    _hip.check(rc, "dlsa_logistic_fit_batched_ex")
    return th.cpu(), S.cpu(), _hip.last_fit_stats(), ws


def test_wide_ozaki_workspace_ownership_and_fallback(torch_cuda, M, monkeypatch):
    """The digit records are part of the workspace dlsa_logistic_workspace_bytes
    reports.  A workspace of exactly that size runs the int8 Gram and writes
    nothing past its end (a guard band of 1 MiB keeps its fill pattern); one
    byte less cannot hold the records and runs the fp64 Gram (oz_fallbacks =
    1, no error); a NULL workspace is allocated and freed inside the call;
    dlsa_fit_options.oz_max_bytes below the records' size falls back the same way."""
    import ctypes

    torch = torch_cuda
    from dlsa_amd import _hip

    p = 300
    X, y, off = _wide_problem(p, 77)
    lib = _hip.load()
    offs = np.ascontiguousarray(off, dtype=np.int64)
    need = lib.dlsa_logistic_workspace_bytes(offs.ctypes.data_as(ctypes.c_void_p), len(off) - 1,
                                             p, 0, 2000)
    assert need > 0
    guard = 1 << 20
    th, S, st, ws = _abi_fit(torch, X, y, off, p, need, guard=guard)
    assert st["passes_oz"] >= 1 and st["oz_fallbacks"] == 0
    tail = ws[need:].cpu().numpy()
    assert (tail == 0xA5).all(), "the fit wrote past the end of its workspace"
    th_f, S_f, st_f, _ = _abi_fit(torch, X, y, off, p, need - 1)
    assert st_f["passes_oz"] == 0 and st_f["oz_fallbacks"] == 1
    th_n, S_n, st_n, _ = _abi_fit(torch, X, y, off, p, None)
    assert st_n["passes_oz"] >= 1 and st_n["oz_fallbacks"] == 0
    assert torch.equal(th_n, th) and torch.equal(S_n, S)
    th_c, S_c, st_c, _ = _abi_fit(torch, X, y, off, p, need, oz_max_bytes=4096)
    assert st_c["passes_oz"] == 0 and st_c["oz_fallbacks"] == 1
    assert torch.equal(th_c, th_f) and torch.equal(S_c, S_f)
    thr, Sr, _, _, _ = O.logistic_fit_partitions(X, y, off)
    for t_, s_ in ((th, S), (th_f, S_f)):
        assert _rel(t_, thr) < REL
        assert _rel(s_, Sr) < REL
    assert _elem(S, S_f) < ELEM


@pytest.mark.parametrize("p,rows", [(201, 2000), (300, 1000), (500, 4096), (384, 32767)])
def test_wide_ozaki_digit_records_stay_in_bounds(torch_cuda, M, p, rows):
    """Ragged row groups (partial 32-row blocks, groups of 1 .. 32767 rows,
    PP = 256 / 384 / 512) with a 1 MiB guard band after the workspace: the
    digits kernel's records and every other workspace region stay inside it,
    and the fit matches the oracle."""
    torch = torch_cuda
    sizes = [rows + 17, 3, 1001, 40] if rows < 32767 else [32767, 5]
    X, y = O.simulate_counter(sum(sizes), p, seed=p + rows)
    off = np.concatenate([[0], np.cumsum(sizes)])
    import ctypes

    from dlsa_amd import _hip

    lib = _hip.load()
    offs = np.ascontiguousarray(off, dtype=np.int64)
    need = lib.dlsa_logistic_workspace_bytes(offs.ctypes.data_as(ctypes.c_void_p), len(off) - 1,
                                             p, 0, rows)
    th, S, st, ws = _abi_fit(torch, X, y, off, p, need, guard=1 << 20, rows_per_chunk=rows)
    assert st["passes_oz"] >= 1
    assert (ws[need:].cpu().numpy() == 0xA5).all()


@pytest.mark.parametrize("kind", ["separable", "outlier"])
def test_ozaki_polish_pass_per_entry(torch_cuda, M, monkeypatch, kind):
    """A budget that runs out (max_iter = 4) on heavy designs: the polish
    pass publishes Sig_inv at the returned theta.  A partition stopped in an
    approximate phase took a full Newton step after its last max |z| record,
    so the growth bound exp(|dtheta|_1 max|x| / 2) would be the only margin
    (advisor finding, r4) -- on the outlier design that left 8e-5 per entry
    (round-5 run r05k).  The exact pass therefore runs on the int8 cores only
    when every partition in it has a record from its last approximate pass
    (capi.hip zfresh), else on the fp64 MFMA.  Per entry within 1e-10 of the
    fp64-MFMA pass at the same iterate."""
    X, y = heavy_design(kind, 24000, seed=4, p_extra=6)  # P = 13: the in-place images fit
    off = np.array([0, 7000, 15000, 24000])
    oz, f64 = _pair(M, monkeypatch, X, y, off, max_iter=4, rows_per_chunk=2048)
    assert oz.stats["polish_partitions"] >= 1, oz.stats
    print(kind, {k: oz.stats[k] for k in ("passes_oz", "oz_stale_partitions",
                                          "polish_partitions", "passes_fp64")})
    assert _rel(oz.theta.cpu(), f64.theta.cpu()) < 1e-10
    assert _elem(oz.sig_inv.cpu(), f64.sig_inv.cpu()) < 1e-10
