#!/usr/bin/env python3
"""Generate golden vectors by running the REFERENCE implementation.

Run in the build container only (needs /root/reference, read-only):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports the reference package ``dlsa`` from /root/reference through a
minimal compatibility shim (the reference targets numpy<1.24, pandas<2 and
sklearn<1.2; SURVEY.md 8(c) "Oracle recipe"):

* ``dlsa.models.LogisticRegression``  -> factory mapping ``penalty='none'``
  to ``None`` and forcing ``tol`` (1e-12 for parity; 1e-4 = sklearn default
  also recorded);
* ``dlsa.models.pd``                  -> proxy whose ``concat(objs, 1)``
  forwards ``axis=1``;
* ``np.float = float; np.NAN = np.nan`` before ``import dlsa.lsa``.

Nothing of the reference is copied: only inputs and the reference's outputs
are written, as ``tests/golden/*.npz``.  Large inputs are not stored; they are
regenerated from the recorded seed by the vectorised generator, which this
script first checks to be bit-identical with the reference's
``simulate_logistic``.
"""

import os
import sys
import warnings

sys.dont_write_bytecode = True
REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REF)
sys.path.insert(0, os.path.abspath(os.path.join(OUT, "..", "..")))

import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402
from sklearn.linear_model import LogisticRegression as _SkLR  # noqa: E402
from sklearn.linear_model import lars_path_gram  # noqa: E402

warnings.filterwarnings("ignore")

import dlsa.models as RM  # noqa: E402  (reference)

np.float = float  # shim for dlsa/lsa.py:12,90
np.NAN = np.nan   # shim for dlsa/lsa.py:23
import dlsa.lsa as RL  # noqa: E402  (reference)

from oracle.dlsa_oracle import simulate_logistic_arrays  # noqa: E402

_TOL = [1e-12]


def _lr_factory(**kw):
    if kw.get("penalty") == "none":
        kw["penalty"] = None
    kw["tol"] = _TOL[0]
    return _SkLR(**kw)


class _PdProxy:
    def __getattr__(self, name):
        return getattr(pd, name)

    @staticmethod
    def concat(objs, *args, **kw):
        if args:
            kw["axis"] = args[0]
        return pd.concat(objs, **kw)


RM.LogisticRegression = _lr_factory
RM.pd = _PdProxy()


def ref_map(df, y_name, fit_intercept, data_info=None, tol=1e-12):
    """Reference map stage: logistic_model per partition group, in partition
    order (projects/logistic_dlsa.py:325)."""
    _TOL[0] = tol
    outs = []
    for _, g in df.groupby("partition_id", sort=True):
        # Spark's GROUPED_MAP pandas_udf builds each group from Arrow with a
        # fresh RangeIndex; models.py:119-120 relies on it.
        g = g.reset_index(drop=True)
        kw = {}
        if data_info is not None:
            kw["data_info"] = data_info
        o = RM.logistic_model(g, y_name, fit_intercept=fit_intercept, **kw)
        outs.append(o.to_numpy(dtype=np.float64))
    return np.stack(outs)  # [K, p, p+3]: par_id, coef, Sig_invMcoef, Sig_inv


def combine(outs, K):
    """dlsa_mapred restated (Spark absent): group-sum + lstsq (dlsa.py:30-52)."""
    S = outs[:, :, 3:].sum(0)
    v = outs[:, :, 2].sum(0)
    wlse = np.linalg.lstsq(S, v, rcond=None)[0]
    oneshot = outs[:, :, 1].sum(0) / K
    return wlse, oneshot, S


def ref_lars(S, b, n, typ):
    r = RL.lars_lsa(np.matrix(S), np.asarray(b, float), intercept=False, n=n,
                    type=typ)
    return (np.asarray(r["AIC"]).ravel(), np.asarray(r["BIC"]).ravel(),
            np.asarray(r["beta"]), np.asarray(r["beta0"]).ravel())


def sk_lars(S, b, typ):
    """Independent oracle: sklearn lars_path_gram on the scaled problem."""
    D = np.abs(b)
    G = D[:, None] * S * D[None, :]
    Xy = G @ np.sign(b)
    _, _, coefs = lars_path_gram(Xy=Xy, Gram=G, n_samples=10 ** 6,
                                 method=typ, eps=np.finfo(float).eps)
    return (coefs * D[:, None]).T


def main():
    rng_report = {}

    # ---- A. simulate_logistic bit-identity ---------------------------------
    for (seed, n, p, K) in [(2019, 3000, 10, 4), (7, 600, 7, 3)]:
        np.random.seed(seed)
        ref_df = RM.simulate_logistic(n, p, "systematic", K)
        np.random.seed(seed)
        pid, lab, feat = simulate_logistic_arrays(n, p, "systematic", K)
        mine = np.concatenate([pid[:, None], lab[:, None], feat], 1)
        ref = ref_df.to_numpy(np.float64)
        assert np.array_equal(ref, mine), "vectorised generator differs"
        np.savez_compressed(os.path.join(OUT, f"simulate_s{seed}_n{n}_p{p}_K{K}.npz"),
                            seed=seed, n=n, p=p, K=K, data=ref)
        rng_report[(seed, n, p)] = "bit-identical"
    print("simulate: bit-identical", rng_report)

    # ---- B. config 1 (n=1e5, p=10, K=4, seed 2019) -------------------------
    np.random.seed(2019)
    pid, lab, feat = simulate_logistic_arrays(100000, 10, "systematic", 4)
    cols = ["x" + str(i) for i in range(10)]
    df = pd.DataFrame(np.concatenate([pid[:, None], lab[:, None], feat], 1),
                      columns=["partition_id", "label"] + cols)
    rec = dict(seed=2019, n=100000, p=10, K=4,
               checksum_X=float(feat.sum()), checksum_y=float(lab.sum()))
    for fi in (False, True):
        outs = ref_map(df, "label", fi, tol=1e-12)
        outs_def = ref_map(df, "label", fi, tol=1e-4)
        wlse, oneshot, S = combine(outs, 4)
        tag = "int" if fi else "noint"
        rec[f"outs_{tag}"] = outs
        rec[f"outs_deftol_{tag}"] = outs_def
        rec[f"wlse_{tag}"] = wlse
        rec[f"oneshot_{tag}"] = oneshot
        if not fi:
            for typ in ("lar", "lasso"):
                AIC, BIC, beta, beta0 = ref_lars(S, wlse, 100000, typ)
                rec[f"lars_{typ}_AIC"] = AIC
                rec[f"lars_{typ}_BIC"] = BIC
                rec[f"lars_{typ}_beta"] = beta
                sk = sk_lars(S, wlse, typ)
                m = min(sk.shape[0], beta.shape[0])
                print(f"config1 lars {typ}: ref vs sklearn max|d|",
                      np.abs(sk[:m] - beta[:m]).max())
        else:
            try:
                RL.lars_lsa(np.matrix(S), wlse, intercept=True, n=100000)
                rec["ref_intercept_lars_error"] = "none"
            except Exception as e:  # lsa.py:100 indexes range(1, n)
                rec["ref_intercept_lars_error"] = type(e).__name__
                print("reference lars_lsa(intercept=True) raises", type(e).__name__)
    np.savez_compressed(os.path.join(OUT, "config1_n1e5_p10_K4.npz"), **rec)
    print("config1 done; WLSE(noint) =", rec["wlse_noint"])

    # ---- C. p=100, K=4, n_k=2e4 (seed 7) ----------------------------------
    np.random.seed(7)
    pid, lab, feat = simulate_logistic_arrays(80000, 100, "systematic", 4)
    cols = ["x" + str(i) for i in range(100)]
    df = pd.DataFrame(np.concatenate([pid[:, None], lab[:, None], feat], 1),
                      columns=["partition_id", "label"] + cols)
    outs = ref_map(df, "label", False, tol=1e-12)
    outs_def = ref_map(df, "label", False, tol=1e-4)
    wlse, oneshot, S = combine(outs, 4)
    AIC, BIC, beta, _ = ref_lars(S, wlse, 80000, "lasso")
    np.savez_compressed(os.path.join(OUT, "p100_n8e4_K4.npz"), seed=7, n=80000,
                        p=100, K=4, checksum_X=float(feat.sum()),
                        checksum_y=float(lab.sum()), outs=outs,
                        outs_deftol=outs_def, wlse=wlse, oneshot=oneshot,
                        lars_lasso_AIC=AIC, lars_lasso_BIC=BIC,
                        lars_lasso_beta=beta)
    print("p100 done; default-tol rel err",
          np.abs(outs_def[:, :, 1] - outs[:, :, 1]).max() /
          np.abs(outs[:, :, 1]).max())

    # ---- D. games-expand.csv (reference data file, no intercept) ----------
    g = pd.read_csv(os.path.join(REF, "projects/results/data/games-expand.csv"))
    Xg = g.drop(["label"], axis=1).to_numpy().astype(np.uint8)
    yg = g["label"].to_numpy().astype(np.uint8)
    gdf = g.copy().astype(np.float64)
    gdf.insert(0, "partition_id", (np.arange(len(g)) % 2).astype(np.float64))
    outs_g = ref_map(gdf, "label", False, tol=1e-12)
    np.savez_compressed(os.path.join(OUT, "games_expand.npz"), X=Xg, y=yg,
                        K=2, outs=outs_g)
    print("games-expand done", outs_g[:, :, 1])

    # ---- E. LARS cases with LASSO drop events -----------------------------
    rs = np.random.RandomState(11)
    cases = []
    tries = 0
    while len(cases) < 6 and tries < 5000:
        tries += 1
        m = int(rs.choice([6, 9, 14, 25]))
        A = rs.randn(3 * m, m) @ np.diag(rs.uniform(0.3, 2.0, m))
        A[:, 1] += 0.9 * A[:, 0]  # correlation makes drops likely
        S = A.T @ A
        b = rs.randn(m) * rs.uniform(0, 1, m) + (rs.rand(m) < 0.4) * 2
        try:
            lasso = ref_lars(S, b, 500, "lasso")
            lar = ref_lars(S, b, 500, "lar")
        except Exception:
            continue
        beta = lasso[2]
        drop = bool(any(np.any((np.abs(beta[i - 1]) > 0) & (beta[i] == 0))
                        for i in range(1, beta.shape[0])))
        if drop or len(cases) < 2:
            cases.append(dict(S=S, b=b, n=500, lasso=lasso, lar=lar,
                              drop=drop))
    rec = {}
    for i, c in enumerate(cases):
        rec[f"c{i}_S"] = c["S"]
        rec[f"c{i}_b"] = c["b"]
        rec[f"c{i}_drop"] = c["drop"]
        for typ in ("lasso", "lar"):
            AIC, BIC, beta, beta0 = c[typ]
            rec[f"c{i}_{typ}_AIC"] = AIC
            rec[f"c{i}_{typ}_BIC"] = BIC
            rec[f"c{i}_{typ}_beta"] = beta
            sk = sk_lars(c["S"], c["b"], typ)
            mm = min(sk.shape[0], beta.shape[0])
            print(f"lars case {i} {typ} drop={c['drop']}: ref vs sklearn",
                  np.abs(sk[:mm] - beta[:mm]).max())
    rec["ncases"] = len(cases)
    np.savez_compressed(os.path.join(OUT, "lars_cases.npz"), **rec)

    # ---- F. data_info-standardised case with intercept ---------------------
    rs = np.random.RandomState(5)
    n, p = 6000, 5
    X = rs.randn(n, p) * np.array([1, 3, 0.5, 10, 2]) + np.array([0, 5, -1, 100, 3])
    Xs = (X - X.mean(0)) / X.std(0, ddof=1)
    yy = (rs.rand(n) < 1 / (1 + np.exp(-(0.5 + Xs @ np.array([1, -1, 0.5, 0, 0]))))).astype(float)
    cols = ["a", "b", "c", "d", "e"]
    df = pd.DataFrame(np.concatenate([(np.arange(n) % 3)[:, None], yy[:, None], X], 1),
                      columns=["partition_id", "label"] + cols)
    # Spark describe() layout: rows count, mean, stddev, min, max (strings)
    info = pd.DataFrame({"summary": ["count", "mean", "stddev", "min", "max"]})
    for j, c in enumerate(cols):
        info[c] = [str(n), repr(float(X[:, j].mean())),
                   repr(float(X[:, j].std(ddof=1))),
                   repr(float(X[:, j].min())), repr(float(X[:, j].max()))]
    outs = ref_map(df, "label", True, data_info=info, tol=1e-12)
    np.savez_compressed(os.path.join(OUT, "standardized_intercept.npz"), X=X, y=yy,
                        K=3, center=np.array([float(v) for v in info.iloc[1, 1:]]),
                        scale=np.array([float(v) for v in info.iloc[2, 1:]]),
                        outs=outs)
    print("standardized done")


def golden_dummy():
    """G. The dummy branch of logistic_model (models.py:56-91): string and int
    factors, dropped levels -> 000_OTHERS, baseline dummies dropped, data_info
    standardisation of the numeric columns, intercept; partition 4 lacks a
    selected level -> the reference's all-zero frame."""
    import json
    import tempfile

    import dlsa.dummies as RD  # reference

    rs = np.random.RandomState(11)
    n = 8000
    carriers = np.array(["AA", "DL", "UA", "WN", "B6", "NK", "F9"])
    origins = np.array(["ATL", "ORD", "DFW", "DEN", "LAX", "SEA", "SFO", "BOS"])
    month = rs.randint(1, 7, size=n)
    carrier = carriers[np.minimum((7 * rs.rand(n) ** 2).astype(int), 6)]
    origin = origins[np.minimum((8 * rs.rand(n) ** 1.5).astype(int), 7)]
    dist = rs.exponential(800.0, size=n) + 100.0
    dep = rs.uniform(0, 24, size=n)
    pid = np.arange(n) % 4
    # partition 4: 400 rows, never SEA (a selected Origin level); it keeps the
    # baseline (000_OTHERS) levels: the reference raises KeyError on a chunk
    # without a baseline level (models.py:67 drops them unconditionally)
    m4 = 400
    month = np.concatenate([month, rs.randint(1, 7, size=m4)])
    carrier = np.concatenate([carrier, carriers[rs.randint(0, 7, size=m4)]])
    origin = np.concatenate([origin, np.array(["ATL", "ORD", "DFW", "BOS", "SFO"])[
        rs.randint(0, 5, size=m4)]])
    dist = np.concatenate([dist, rs.exponential(800.0, size=m4) + 100.0])
    dep = np.concatenate([dep, rs.uniform(0, 24, size=m4)])
    pid = np.concatenate([pid, np.full(m4, 4)])
    eff_c = dict(zip(carriers, [0.0, 0.3, -0.2, 0.5, -0.4, 0.2, 0.1]))
    eff_o = dict(zip(origins, [0.0, 0.2, -0.3, 0.4, 0.1, -0.2, 0.3, -0.1]))
    eta = (-0.2 + 0.4 * (dist - 900) / 800 - 0.05 * (dep - 12) + 0.1 * (month - 3.5)
           + np.array([eff_c[c] for c in carrier]) + np.array([eff_o[o] for o in origin]))
    label = (rs.rand(n + m4) < 1 / (1 + np.exp(-eta))).astype(float)
    df = pd.DataFrame({"partition_id": pid.astype(float), "label": label, "Month": month,
                       "UniqueCarrier": carrier, "Origin": origin, "Distance": dist,
                       "DepTime": dep})
    factors = ["Month", "UniqueCarrier", "Origin"]
    counts = RD.dummy_factors_counts(df, factors)
    with tempfile.TemporaryDirectory() as tmp:
        info_d = RD.select_dummy_factors(counts, keep_top=[1, 0.8, 0.9],
                                         replace_with="000_OTHERS",
                                         pickle_file=os.path.join(tmp, "dummy_info.pkl"))
    info_d = {k: {f: [x.item() if hasattr(x, "item") else x for x in v] for f, v in d.items()}
              for k, d in info_d.items()}
    baseline = ["Month_1", "UniqueCarrier_000_OTHERS", "Origin_000_OTHERS"]
    numeric = ["DepTime", "Distance"]
    info = pd.DataFrame({"summary": ["count", "mean", "stddev", "min", "max"]})
    for c in numeric:
        v = df[c].to_numpy()
        info[c] = [str(v.size), repr(float(v.mean())), repr(float(v.std(ddof=1))),
                   repr(float(v.min())), repr(float(v.max()))]
    _TOL[0] = 1e-12
    outs, cols = [], None
    for _, g in df.groupby("partition_id", sort=True):
        g = g.reset_index(drop=True)
        o = RM.logistic_model(g, "label", fit_intercept=True, dummy_info=info_d,
                              dummy_factors_baseline=baseline, data_info=info)
        outs.append(o.to_numpy(dtype=np.float64))
        cols = list(o.columns) if cols is None else cols
    np.savez_compressed(
        os.path.join(OUT, "dummy_branch.npz"), pid=pid, label=label, month=month,
        carrier=carrier.astype("U8"), origin=origin.astype("U8"), distance=dist, deptime=dep,
        dummy_info=json.dumps(info_d), baseline=np.array(baseline, dtype="U32"),
        info=info.to_numpy().astype("U40"), info_cols=np.array(list(info.columns), dtype="U32"),
        outs=np.stack(outs), cols=np.array(cols, dtype="U40"))
    print("dummy branch done:", np.stack(outs).shape, "zero frame:",
          not np.abs(outs[4]).any())


def golden_dummy_file():
    """H. Dummy-level selection over a CSV file (dlsa/dummies.py:111-146):
    the reference's select_dummy_factors_from_file on a 1.2 MB file (two
    readlines(1024000) buffers, level frequencies drifting along the file),
    by column names and by column positions.  The file text is rebuilt by
    tests/golden/dummy_csv.py from its seed; only the outputs are stored."""
    import json
    import tempfile

    import dlsa.dummies as RD  # reference

    sys.path.insert(0, OUT)
    import dummy_csv as DC

    cols = DC.rows()
    txt = DC.text(cols)
    res = {}
    with tempfile.TemporaryDirectory() as tmp:
        path = os.path.join(tmp, "air.csv")
        with open(path, "w") as fh:
            fh.write(txt)
        with open(path) as fh:
            nbuf = 0
            while fh.readlines(1024000):
                nbuf += 1
        for tag, dc, keep in (("names", ["Month", "UniqueCarrier", "Origin"], [1, 0.8, 0.9]),
                              ("positions", [2, 1], [0.75, 0.95])):
            info = RD.select_dummy_factors_from_file(path, True, dc, keep, "000_OTHERS",
                                                     os.path.join(tmp, f"{tag}.pkl"))
            res[tag] = info
    np.savez_compressed(os.path.join(OUT, "dummy_file.npz"), n_buffers=nbuf, n_rows=len(txt),
                        info_names=json.dumps(res["names"]),
                        info_positions=json.dumps(res["positions"]))
    print("dummy file done: buffers", nbuf)


def golden_eval():
    """I. The evaluation pass logistic_model_eval (models.py:151-225): per
    partition the log-likelihood of 4 candidate coefficient columns, on
    (a) config-1 data (p = 10) with and without intercept, (b) the same with
    data_info standardisation, (c) the dummy branch (partitions 0-3 of the
    dummy fixture, every level present) with intercept + data_info; and what
    the reference does on the dummy fixture's partition 4 (a selected level
    missing, models.py:188-195), recorded as the exception it raises."""
    import json

    rs = np.random.RandomState(23)
    np.random.seed(2019)
    pid, lab, feat = simulate_logistic_arrays(100000, 10, "systematic", 4)
    cols = ["x" + str(i) for i in range(10)]
    df = pd.DataFrame(np.concatenate([pid[:, None], lab[:, None], feat], 1),
                      columns=["partition_id", "label"] + cols)
    info = pd.DataFrame({"summary": ["count", "mean", "stddev", "min", "max"]})
    for c in cols:
        v = feat[:, cols.index(c)]
        info[c] = [str(v.size), repr(float(v.mean() + 0.01)), repr(float(v.std(ddof=1) * 1.1)),
                   repr(float(v.min())), repr(float(v.max()))]
    rec = {"info": info.to_numpy().astype("U40"), "info_cols": np.array(list(info.columns), "U32")}
    names = ["beta_byAIC", "beta_byBIC", "beta_byOLS", "beta_byONESHOT"]
    for fi in (False, True):
        for std in (False, True):
            P = 10 + int(fi)
            par = pd.DataFrame(0.6 * rs.randn(P, 4), columns=names)
            out = []
            for k in range(4):
                g = df[df["partition_id"] == k].reset_index(drop=True)
                o = RM.logistic_model_eval(g, "label", par, fit_intercept=fi,
                                           data_info=info if std else [])
                out.append(o.to_numpy(np.float64).reshape(-1))
            tag = f"{'int' if fi else 'noint'}_{'std' if std else 'raw'}"
            rec["par_" + tag] = par.to_numpy()
            rec["ll_" + tag] = np.stack(out)
    # dummy branch
    gd = np.load(os.path.join(OUT, "dummy_branch.npz"))
    ddf = pd.DataFrame({"partition_id": gd["pid"].astype(float), "label": gd["label"],
                        "DepTime": gd["deptime"], "Distance": gd["distance"],
                        "Month": gd["month"], "UniqueCarrier": gd["carrier"].astype(object),
                        "Origin": gd["origin"].astype(object)})
    dinfo = json.loads(str(gd["dummy_info"]))
    base = [str(b) for b in gd["baseline"]]
    dinf = pd.DataFrame(gd["info"].astype(object), columns=list(gd["info_cols"]))
    P = len(gd["cols"]) - 3
    par = pd.DataFrame(0.3 * rs.randn(P, 4), columns=names)
    out = []
    for k in range(4):
        g = ddf[ddf["partition_id"] == k].reset_index(drop=True)
        o = RM.logistic_model_eval(g, "label", par, fit_intercept=True, dummy_info=dinfo,
                                   dummy_factors_baseline=base, data_info=dinf)
        out.append(o.to_numpy(np.float64).reshape(-1))
    rec["par_dummy"] = par.to_numpy()
    rec["ll_dummy"] = np.stack(out)
    g = ddf[ddf["partition_id"] == 4].reset_index(drop=True)
    try:
        RM.logistic_model_eval(g, "label", par, fit_intercept=True, dummy_info=dinfo,
                               dummy_factors_baseline=base, data_info=dinf)
        rec["missing_level_outcome"] = "returned"
    except Exception as e:  # noqa: BLE001 - the reference's behaviour is the datum
        rec["missing_level_outcome"] = f"raises {type(e).__name__}: {str(e)[:160]}"
    np.savez_compressed(os.path.join(OUT, "eval.npz"), **rec)
    print("eval done:", rec["missing_level_outcome"])


def golden_p100_k8():
    """p = 100, K = 8, n_k = 2e4 (seed 7): per-partition frames
    at tol 1e-12, WLSE / ONESHOT and the LASSO path of the reference."""
    np.random.seed(7)
    pid, lab, feat = simulate_logistic_arrays(160000, 100, "systematic", 8)
    cols = ["x" + str(i) for i in range(100)]
    df = pd.DataFrame(np.concatenate([pid[:, None], lab[:, None], feat], 1),
                      columns=["partition_id", "label"] + cols)
    outs = ref_map(df, "label", False, tol=1e-12)
    wlse, oneshot, S = combine(outs, 8)
    AIC, BIC, beta, _ = ref_lars(S, wlse, 160000, "lasso")
    np.savez_compressed(os.path.join(OUT, "p100_n16e4_K8.npz"), seed=7, n=160000,
                        p=100, K=8, checksum_X=float(feat.sum()),
                        checksum_y=float(lab.sum()), outs=outs, wlse=wlse, oneshot=oneshot,
                        lars_lasso_AIC=AIC, lars_lasso_BIC=BIC, lars_lasso_beta=beta)
    print("p100 K8 done; support", np.nonzero(beta[int(np.argmin(BIC))])[0].size)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "p100_k8":
        golden_p100_k8()
    elif len(sys.argv) > 1 and sys.argv[1] == "eval":
        golden_eval()
    elif len(sys.argv) > 1 and sys.argv[1] == "dummy":
        golden_dummy()
    elif len(sys.argv) > 1 and sys.argv[1] == "dummy_file":
        golden_dummy_file()
    else:
        main()
        golden_p100_k8()
        golden_dummy()
        golden_dummy_file()
        golden_eval()
