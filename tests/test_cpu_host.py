"""CPU tests of the product's host side: the C-ABI library loads and exports
every declared symbol, the native LARS/DBIC and the combine match the
reference golden vectors and the oracle, the product fails loudly without a
GPU, and the multi-rank combine is correct under gloo (world_size 2)."""

import os
import re

import numpy as np
import pytest

import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    txt = open(os.path.join(ROOT, "include", "dlsa_hip.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(dlsa_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    import ctypes

    from dlsa_amd import _hip

    lib = ctypes.CDLL(_hip.LIB_PATH)
    syms = _header_symbols()
    assert len(syms) >= 10
    for s in syms:
        assert hasattr(lib, s), f"{s} declared in include/dlsa_hip.h but not exported"
    assert set(syms) == set(_hip.SIGNATURES), "ctypes binding out of sync with the header"
    assert b"gfx950" in _hip.load().dlsa_build_info()


def test_fit_fails_loudly_without_gpu():
    import torch

    from dlsa_amd import DlsaHipError
    from dlsa_amd.models import logistic_model_batched

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(DlsaHipError):
        logistic_model_batched(np.zeros((4, 2)), np.zeros(4), [0, 4])


@pytest.mark.parametrize("typ", ["lar", "lasso"])
def test_native_lars_config1_golden(golden_dir, typ):
    from dlsa_amd.lsa import lars_lsa

    g = np.load(os.path.join(golden_dir, "config1_n1e5_p10_K4.npz"))
    S = g["outs_noint"][:, :, 3:].sum(0)
    r = lars_lsa(S, g["wlse_noint"], False, 100000, type=typ)
    assert r["beta"].shape == g[f"lars_{typ}_beta"].shape
    assert np.abs(r["beta"] - g[f"lars_{typ}_beta"]).max() < 1e-12
    assert np.abs(r["BIC"] - g[f"lars_{typ}_BIC"]).max() < 1e-8
    assert np.abs(r["AIC"] - g[f"lars_{typ}_AIC"]).max() < 1e-8


def test_native_lars_drop_cases_golden(golden_dir):
    from dlsa_amd.lsa import lars_lsa

    L = np.load(os.path.join(golden_dir, "lars_cases.npz"))
    for i in range(int(L["ncases"])):
        for typ in ("lar", "lasso"):
            r = lars_lsa(L[f"c{i}_S"], L[f"c{i}_b"], False, 500, type=typ)
            gb = L[f"c{i}_{typ}_beta"]
            assert r["beta"].shape == gb.shape
            assert np.abs(r["beta"] - gb).max() < 1e-10
            assert np.abs(r["BIC"] - L[f"c{i}_{typ}_BIC"]).max() < 1e-8


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("intercept", [False, True])
@pytest.mark.parametrize("typ", ["lar", "lasso"])
def test_native_lars_vs_oracle_random(seed, intercept, typ):
    from dlsa_amd.lsa import lars_lsa

    rs = np.random.RandomState(seed)
    m = [5, 12, 30, 60, 3, 101][seed]
    A = rs.randn(2 * m + 5, m)
    A[:, 1 % m] += 0.8 * A[:, 0]
    S = A.T @ A
    b = rs.randn(m) * (rs.rand(m) < 0.5) + 0.05 * rs.randn(m)
    r = lars_lsa(S, b, intercept, 1000, type=typ)
    o = O.lars_lsa(S, b, intercept, 1000, type=typ)
    assert r["beta"].shape == o["beta"].shape
    assert np.allclose(r["beta"], o["beta"], rtol=0, atol=1e-9 * max(1, np.abs(o["beta"]).max()))
    assert np.allclose(r["BIC"], o["BIC"], rtol=1e-10, atol=1e-8)
    assert np.allclose(r["beta0"], o["beta0"], rtol=1e-10, atol=1e-10)


@pytest.mark.parametrize("seed", [9, 13, 37])
def test_native_lars_drop_heavy_vs_oracle(seed):
    """LASSO paths with 5-7 drops (low-rank correlated designs): after each
    drop the kept columns are renumbered in active order, so the path after a
    drop follows the oracle (lsa.py:90-212) as closely as before one."""
    from dlsa_amd.lsa import lars_lsa

    rs = np.random.RandomState(seed)
    m = 40
    Z = rs.randn(3 * m, 8)
    A = Z @ rs.randn(8, m) + 0.3 * rs.randn(3 * m, m)
    S = A.T @ A
    b = rs.randn(m)
    o = O.lars_lsa(S, b, False, 1000, type="lasso")
    nz = np.abs(o["beta"]) > 0
    assert int((nz[:-1] & ~nz[1:]).sum()) >= 5
    r = lars_lsa(S, b, False, 1000, type="lasso")
    assert r["beta"].shape == o["beta"].shape
    assert np.abs(r["beta"] - o["beta"]).max() < 1e-10 * max(1.0, np.abs(o["beta"]).max())
    assert np.allclose(r["BIC"], o["BIC"], rtol=1e-10, atol=1e-8)


def test_native_lars_vs_oracle_config5_size():
    """LASSO path at the config-5 width class (m = 400, 401 knots): the native
    path (permuted-Sigma equiangular products, transposed-R back solve) against
    the oracle restatement of lsa.py:90-212, knot by knot."""
    from dlsa_amd.lsa import lars_lsa

    rs = np.random.RandomState(3)
    m = 400
    X = rs.rand(3000, m) - 0.5
    S = X.T @ X
    b = np.where(rs.rand(m) < 0.4, 1.0, 0.0) + 0.05 * rs.randn(m)
    r = lars_lsa(S, b, False, 1e5, type="lasso")
    o = O.lars_lsa(S, b, False, 1e5, type="lasso")
    assert r["beta"].shape == o["beta"].shape
    assert np.abs(r["beta"] - o["beta"]).max() < 1e-10 * max(1.0, np.abs(o["beta"]).max())
    assert np.abs(r["BIC"] - o["BIC"]).max() < 1e-10 * np.abs(o["BIC"]).max()
    assert int(np.argmin(r["BIC"])) == int(np.argmin(o["BIC"]))


@pytest.mark.parametrize("fi", [False, True])
def test_dlsa_selection_vs_oracle(golden_dir, fi):
    from dlsa_amd.dlsa import dlsa

    g = np.load(os.path.join(golden_dir, "config1_n1e5_p10_K4.npz"))
    tag = "int" if fi else "noint"
    S = g["outs_" + tag][:, :, 3:].sum(0)
    w = g["wlse_" + tag]
    out = dlsa(S, w, 100000, fit_intercept=fi)
    oa, ob = O.dlsa(S, w, 100000, fit_intercept=fi)
    assert np.allclose(out["beta_byAIC"], oa, atol=1e-12)
    assert np.allclose(out["beta_byBIC"], ob, atol=1e-12)
    # DBIC picks the true support {x0..x3}
    sup = np.nonzero(out["beta_byBIC"].to_numpy()[1 if fi else 0:])[0]
    assert set(sup) == {0, 1, 2, 3}


def test_dlsa_mapred_pandas_vs_golden(golden_dir):
    """Stacked Spark-style map output (par_id, coef, Sig_invMcoef, cols)."""
    import pandas as pd

    from dlsa_amd.dlsa import dlsa_mapred

    g = np.load(os.path.join(golden_dir, "config1_n1e5_p10_K4.npz"))
    outs = g["outs_int"]
    cols = ["par_id", "coef", "Sig_invMcoef", "intercept"] + [f"x{i}" for i in range(10)]
    frames = [pd.DataFrame(o, columns=cols) for o in outs]
    res = dlsa_mapred(frames)
    assert list(res.columns[:2]) == ["beta_byOLS", "beta_byONESHOT"]
    assert np.abs(res["beta_byOLS"].to_numpy() - g["wlse_int"]).max() < 1e-12
    assert np.abs(res["beta_byONESHOT"].to_numpy() - g["oneshot_int"]).max() < 1e-12
    assert np.allclose(res.iloc[:, 2:].to_numpy(), outs[:, :, 3:].sum(0), rtol=1e-13, atol=1e-12)
    with pytest.raises(Exception):
        dlsa_mapred(pd.DataFrame(columns=cols))


@pytest.mark.parametrize("name", ["simulate_s2019_n3000_p10_K4.npz", "simulate_s7_n600_p7_K3.npz"])
def test_simulate_logistic_product_bit_identical(golden_dir, name):
    from dlsa_amd.models import simulate_logistic

    g = np.load(os.path.join(golden_dir, name))
    np.random.seed(int(g["seed"]))
    df = simulate_logistic(int(g["n"]), int(g["p"]), "systematic", int(g["K"]))
    assert np.array_equal(df.to_numpy(np.float64), g["data"])


def test_partition_offsets():
    from dlsa_amd.models import partition_offsets

    pid = np.arange(23) % 5
    order, off = partition_offsets(pid)
    assert off.tolist() == [0, 5, 10, 15, 19, 23]
    assert all((pid[order[off[k]:off[k + 1]]] == k).all() for k in range(5))
    assert all(np.all(np.diff(order[off[k]:off[k + 1]]) > 0) for k in range(5))


# ---- multi-rank combine (gloo, world_size 2) -------------------------------

def _gloo_worker(rank, world, port, golden_dir, q, shards):
    import torch
    import torch.distributed as dist

    from dlsa_amd.distributed import combine_and_finish

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = np.load(os.path.join(golden_dir, "config1_n1e5_p10_K4.npz"))
    outs = g["outs_noint"]
    mine = outs[shards[rank]]  # this rank's partitions (25 000 rows each)
    P = outs.shape[1]
    # the local buffer in the layout of reduce_partitions_device(fit, n_rows=True):
    # [sum Sig_inv | sum Sig_inv theta | sum theta | K | N]
    buf = np.concatenate([mine[:, :, 3:].sum(0).ravel(), mine[:, :, 2].sum(0),
                          mine[:, :, 1].sum(0), [float(len(mine)), 25000.0 * len(mine)]])
    calls = []
    orig = dist.all_reduce

    def counting(*a, **k):
        calls.append(1)
        return orig(*a, **k)

    dist.all_reduce = counting
    res = combine_and_finish(torch.from_numpy(buf), P)
    dist.all_reduce = orig
    q.put((rank, res["wlse"], res["oneshot"], res["dbic_support"].tolist(),
           res["path"]["BIC"], len(calls)))
    dist.destroy_process_group()


@pytest.mark.parametrize("shards", [([0, 2], [1, 3]), ([0, 1, 3], [2])])
def test_distributed_combine_gloo(golden_dir, shards):
    """The sharded path's exchange + host tail (distributed.combine_and_finish)
    on world_size 2 with even and uneven shards: ONE all-reduce carries the
    partition sums, K and N; every rank gets the golden WLSE / ONESHOT and the
    DBIC path of the full data (n = 1e5)."""
    import multiprocessing as mp
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gloo_worker, args=(r, 2, port, golden_dir, q, shards))
          for r in range(2)]
    for p_ in ps:
        p_.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p_ in ps:
        p_.join(timeout=60)
        assert p_.exitcode == 0
    g = np.load(os.path.join(golden_dir, "config1_n1e5_p10_K4.npz"))
    S = g["outs_noint"][:, :, 3:].sum(0)
    ref = O.lars_lsa(S, g["wlse_noint"], False, 100000, type="lasso")
    for rank, wlse, oneshot, support, bic, n_calls in res:
        assert n_calls == 1
        assert np.abs(wlse - g["wlse_noint"]).max() < 1e-10
        assert np.abs(oneshot - g["oneshot_noint"]).max() < 1e-12
        assert support == [0, 1, 2, 3]
        assert np.allclose(bic, ref["BIC"], rtol=1e-9, atol=1e-6)  # N = 1e5 reached the DBIC


def test_dummy_design_generator():
    """Config-3 generator: 181 columns, at most one dummy set per factor per
    row, deterministic in the seed, every level present at moderate n."""
    torch = pytest.importorskip("torch")
    from dlsa_amd.models import AIRLINE_FACTORS, AIRLINE_NUMERIC, simulate_dummy_design

    X, y = simulate_dummy_design(30000, seed=3, device="cpu")
    X2, y2 = simulate_dummy_design(30000, seed=3, device="cpu")
    assert X.shape == (30000, 181) and torch.equal(X, X2) and torch.equal(y, y2)
    num = X[:, :AIRLINE_NUMERIC]
    assert float(num.min()) >= -0.5 and float(num.max()) < 0.5
    col = AIRLINE_NUMERIC
    for L in AIRLINE_FACTORS:
        block = X[:, col:col + L - 1]
        assert set(block.unique().tolist()) <= {0.0, 1.0}
        assert float(block.sum(1).max()) <= 1.0
        assert bool((block.sum(0) > 0).all())
        col += L - 1
    assert set(y.unique().tolist()) == {0.0, 1.0}


def test_wlse_cholesky_matches_lstsq_and_falls_back():
    """dlsa.py:48-49 solves with lstsq; the Cholesky solve agrees on a positive-
    definite sum and a singular sum (an all-zero dummy column) keeps lstsq's
    minimum-norm answer."""
    from dlsa_amd.dlsa import wlse

    rng = np.random.default_rng(5)
    A = rng.standard_normal((400, 60))
    S = A.T @ A
    v = rng.standard_normal(60)
    ref = np.linalg.lstsq(S, v, rcond=None)[0]
    assert np.abs(wlse(S, v) - ref).max() < 1e-12 * np.abs(ref).max()
    S[7, :] = 0.0
    S[:, 7] = 0.0
    v[7] = 0.0
    ref = np.linalg.lstsq(S, v, rcond=None)[0]
    assert np.allclose(wlse(S, v), ref, rtol=1e-10, atol=1e-12)


def test_encode_categorical_matches_reference_design(golden_dir):
    """The product's categorical-code encoding (dlsa_amd.models.encode_categorical)
    expands to exactly the oracle's restatement of the reference dummy design
    (models.py:56-91) and the reference's column names; the missing-level
    partition is detected from the level counts."""
    from test_oracle_golden import _dummy_fixture

    from dlsa_amd.models import encode_categorical

    g, df, dinfo, base, info = _dummy_fixture(golden_dir)
    cols = [str(c) for c in g["cols"]][4:]
    for k in range(5):
        part = df[df["partition_id"] == k].reset_index(drop=True)
        enc = encode_categorical(part, "label", dinfo, base)
        assert enc["cols"] == cols and enc["numeric"] == ["DepTime", "Distance"]
        assert enc["codes"].dtype == np.uint8 and enc["levels"].tolist() == [6, 5, 7]
        num = {c: part[c].to_numpy() for c in ("Distance", "DepTime")}
        fac = {c: part[c].to_numpy() for c in ("Month", "UniqueCarrier", "Origin")}
        X, _, missing = O.dummy_design(num, fac, dinfo, base)
        assert np.array_equal(O.expand_codes(enc["Xn"], enc["codes"], enc["levels"]), X)
        assert missing == (bool((enc["counts"] == 0).any()) or enc["unknown"])
        assert missing == (k == 4)


def test_categorical_generator_expands_to_dummy_design():
    """Config-3 data: the categorical-code generator and the dense design are
    the same draws (expand(codes) == simulate_dummy_design)."""
    torch = pytest.importorskip("torch")
    from dlsa_amd.models import simulate_categorical, simulate_dummy_design

    Xn, codes, y, levels = simulate_categorical(5000, seed=9, device="cpu")
    X, y2 = simulate_dummy_design(5000, seed=9, device="cpu")
    assert codes.dtype == torch.uint8 and codes.shape == (5000, 5)
    assert np.array_equal(O.expand_codes(Xn.numpy(), codes.numpy(), levels), X.numpy())
    assert torch.equal(y, y2)


def test_read_table_select_dropna_binarise(tmp_path):
    """Host half of the ingest (logistic_dlsa.py:226-239) against pandas."""
    import pandas as pd

    from dlsa_amd.ingest import read_table

    rs = np.random.RandomState(1)
    df = pd.DataFrame({"a": rs.randn(500), "b": rs.rand(500), "c": rs.rand(500),
                       "y": rs.randint(-3, 4, 500).astype(float)})
    df.loc[[3, 17, 400], "a"] = np.nan
    df.loc[[5], "c"] = np.nan  # not selected: keeps the row
    df.to_csv(tmp_path / "t.csv", index=False)
    t = read_table(str(tmp_path / "t.csv"), "y", ["b", "a"])
    ref = df[["b", "a", "y"]].dropna().reset_index(drop=True)
    ref["y"] = (ref["y"] > 0).astype(float)
    assert list(t.columns) == ["b", "a", "y"]
    assert np.array_equal(t.to_numpy(), ref.to_numpy())


def test_ingest_fails_loudly_without_gpu():
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from dlsa_amd._hip import DlsaHipError
    from dlsa_amd.ingest import repartition

    with pytest.raises(DlsaHipError):
        repartition(torch.zeros(4, dtype=torch.int32), 2, torch.zeros((4, 2)))


def test_encode_categorical_missing_value_is_all_zero_block():
    """pd.get_dummies (dummy_na=False) gives a missing factor value no column:
    the encoder maps it to code 0 (the all-zero dummy block)."""
    import pandas as pd

    from dlsa_amd.models import encode_categorical

    df = pd.DataFrame({"partition_id": [0.0] * 6, "y": [0, 1, 0, 1, 1, 0.0],
                       "F": ["a", "b", None, "c", "a", "b"], "x": [1, 2, 3, 4, 5, 6.0]})
    di = {"factor_selected": {"F": ["a", "b", "c"]}, "factor_dropped": {"F": []},
          "factor_selected_names": {"F": ["F_a", "F_b", "F_c"]}}
    e = encode_categorical(df, "y", di, ["F_a"])
    ref = pd.get_dummies(df, columns=["F"]).drop(columns=["F_a", "partition_id", "y"])
    assert e["cols"] == list(ref.columns)
    assert np.array_equal(O.expand_codes(e["Xn"], e["codes"], e["levels"]),
                          ref.to_numpy(dtype=np.float64))


def test_encode_categorical_unknown_rows():
    """A value outside the selected names and the baselines is flagged per
    row (the reference's column-set check, models.py:84): its row is coded 0
    and reported in ``unknown_rows``."""
    import pandas as pd

    from dlsa_amd.models import encode_categorical

    df = pd.DataFrame({"partition_id": [0.0] * 5, "y": [0, 1, 0, 1, 1.0],
                       "F": ["a", "b", "zz", "c", "a"], "x": [1, 2, 3, 4, 5.0]})
    di = {"factor_selected": {"F": ["a", "b", "c"]}, "factor_dropped": {"F": []},
          "factor_selected_names": {"F": ["F_a", "F_b", "F_c"]}}
    e = encode_categorical(df, "y", di, ["F_a"])
    assert e["unknown"] and e["unknown_rows"].tolist() == [False, False, True, False, False]
    assert e["codes"][:, 0].tolist() == [0, 1, 0, 2, 0]


def test_bench_rejects_world_size_mismatch():
    """bench.py refuses to run when the process group would not hold --gpus
    ranks (before touching any GPU)."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2"],
                       cwd=root, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "WORLD_SIZE" in r.stderr


def test_bench_host_cores_reports_quota():
    import importlib.util

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(root, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    cores, info = b.host_cores()
    assert 1 <= cores <= info["nproc"]
    assert info["affinity"] <= info["nproc"]


# ---- data_info: moments merge and the sharded combine ------------------------

def test_merge_moments_and_describe_frame_match_pandas():
    """merge_moments (Chan) of the [5, p] moments of uneven row blocks equals
    the moments of the whole; describe_frame is Spark's describe() layout
    whose count / mean / stddev / min / max equal pandas describe()
    (projects/logistic_dlsa.py:287-298; models.py:99-101 reads rows 1, 2)."""
    import pandas as pd

    from dlsa_amd.ingest import describe_frame, merge_moments

    rs = np.random.RandomState(3)
    X = rs.randn(5003, 4) * [1.0, 1e3, 1e-3, 5.0] + [0.0, -7.0, 0.05, 2.0]
    X[17, 2] = np.nan
    cuts = [0, 1, 900, 901, 3000, 5003]
    parts = [O.column_moments(X[a:b]) for a, b in zip(cuts[:-1], cuts[1:])]
    whole = O.column_moments(X)
    got = merge_moments(parts)
    assert np.array_equal(got[0], whole[0]) and np.array_equal(got[3:], whole[3:])
    assert np.abs(got[1] - whole[1]).max() <= 1e-14 * np.abs(X[~np.isnan(X)]).max()
    assert np.allclose(got[2], whole[2], rtol=1e-13, atol=0)
    cols = ["a", "b", "c", "d"]
    info = describe_frame(got, cols)
    assert list(info.columns) == ["summary"] + cols
    assert info["summary"].tolist() == ["count", "mean", "stddev", "min", "max"]
    pdd = pd.DataFrame(X, columns=cols).describe()
    for c in cols:
        assert int(info[c][0]) == int(pdd[c]["count"])
        for row, key in ((1, "mean"), (2, "std"), (3, "min"), (4, "max")):
            assert abs(float(info[c][row]) - pdd[c][key]) <= 1e-12 * max(1.0, abs(pdd[c][key]))


def _moments_worker(rank, world, port, X, q):
    import torch.distributed as dist

    from dlsa_amd.ingest import combine_moments, describe_frame

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    calls = []
    orig = dist.all_reduce

    def counting(*a, **k):
        calls.append(1)
        return orig(*a, **k)

    dist.all_reduce = counting
    try:
        # rank r holds rows i % K in its partitions (K = 5: ranks own 2 / 3 partitions)
        K = 5
        k0, k1 = rank * K // world, (rank + 1) * K // world
        mine = X[(np.arange(len(X)) % K >= k0) & (np.arange(len(X)) % K < k1)]
        tot = combine_moments(O.column_moments(mine), distributed=True)
    finally:
        dist.all_reduce = orig
    q.put((rank, describe_frame(tot, ["u", "v", "w"]).to_numpy().tolist(), len(calls)))
    dist.destroy_process_group()


def test_sharded_describe_gloo_equals_one_rank():
    """data_info of a sharded data set: every rank's local moments go through
    ONE all-reduce and merge in rank order -- the frame is identical on both
    ranks and equal (to the last digits) to the one-rank frame of all rows."""
    import multiprocessing as mp
    import socket

    from dlsa_amd.ingest import describe_frame

    rs = np.random.RandomState(8)
    X = rs.rand(20011, 3) * [1.0, 100.0, 1e-6] - [0.5, 3.0, 0.0]
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_moments_worker, args=(r, 2, port, X, q)) for r in range(2)]
    for p_ in ps:
        p_.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p_ in ps:
        p_.join(timeout=60)
        assert p_.exitcode == 0
    one = describe_frame(O.column_moments(X), ["u", "v", "w"]).to_numpy()
    assert res[0][1] == res[1][1]  # bit-identical on every rank
    assert res[0][2] == 1 and res[1][2] == 1
    got = np.array(res[0][1], dtype=object)
    assert (got[:, 0] == one[:, 0]).all() and (got[0] == one[0]).all()
    for i in range(1, 5):
        for j in range(1, 4):
            assert abs(float(got[i, j]) - float(one[i, j])) <= 1e-13 * max(1.0, abs(float(one[i, j])))


def test_pmc_traffic_records_match_bench_kernel_keys():
    """bench.py fills roofline.traffic only when the PMC record's kernel_key is
    the key it computes for the config's dominant kernel (bench.py pmc_key):
    a record under another key leaves traffic null without an error."""
    import json
    import os
    root = os.path.join(os.path.dirname(__file__), "..")
    rec = json.load(open(os.path.join(root, "profiles", "pmc_traffic.json")))
    src = open(os.path.join(root, "bench.py")).read()
    # (config 3's p counts the numeric and dummy columns, without the intercept)
    want = {"config2": ("irls_coop<bf16>", 100), "config3": ("cat_pass_kernel", 181),
            "config4": ("ols_stream", 64), "config5": ("wide_fused_bf16", 500)}
    for cfg, (key, p) in want.items():
        assert f'pmc_key = "{key}"' in src, key
        assert rec[cfg]["kernel_key"] == key and rec[cfg]["p"] == p, (cfg, rec[cfg])
