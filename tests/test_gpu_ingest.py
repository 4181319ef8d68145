"""GPU tests of the ingest path: the HIP repartition (stable counting sort,
dlsa_partition_rows) against numpy's stable argsort (bit-exact), and CSV ->
HBM partition layout -> fit against the oracle."""

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a visible MI355X"
    return torch


@pytest.mark.parametrize("n,K", [(100003, 37), (20001, 5000), (9000, 1), (4096 * 3 + 17, 1024)])
def test_repartition_bit_exact(torch_cuda, n, K):
    """Rows of X (fp64, 56 B), y (8 B) and uint8 codes (3 B) grouped by
    partition id exactly like numpy's stable sort; offsets and order too."""
    torch = torch_cuda
    from dlsa_amd.ingest import repartition

    rs = np.random.RandomState(n % 1000 + K)
    pid = rs.randint(0, K, size=n).astype(np.int32)
    X = rs.randn(n, 7)
    y = rs.rand(n)
    codes = rs.randint(0, 256, size=(n, 3)).astype(np.uint8)
    dev = torch.device("cuda")
    (Xp, yp, cp), off, order = repartition(torch.from_numpy(pid).to(dev), K,
                                           torch.from_numpy(X).to(dev),
                                           torch.from_numpy(y).to(dev),
                                           torch.from_numpy(codes).to(dev), return_order=True)
    perm = np.argsort(pid, kind="stable")
    assert np.array_equal(order.cpu().numpy(), perm)
    assert np.array_equal(Xp.cpu().numpy(), X[perm])
    assert np.array_equal(yp.cpu().numpy(), y[perm])
    assert np.array_equal(cp.cpu().numpy(), codes[perm])
    assert np.array_equal(off, np.concatenate([[0], np.cumsum(np.bincount(pid, minlength=K))]))


def test_repartition_systematic_matches_reference_layout(torch_cuda):
    """partition_id = row % K (insert_partition_id_pdf / monotonically_increasing_id
    % K): the layout equals oracle.systematic_partition."""
    torch = torch_cuda
    from dlsa_amd.ingest import repartition, systematic_partition_id

    n, K = 50000, 8
    X = np.random.RandomState(0).rand(n, 5)
    pid = systematic_partition_id(n, K)
    (Xp,), off = repartition(pid, K, torch.from_numpy(X).cuda())
    order, off_ref = O.systematic_partition(np.arange(n) % K)
    assert np.array_equal(off, off_ref)
    assert np.array_equal(Xp.cpu().numpy(), X[order])


def test_repartition_rejects_bad_ids(torch_cuda):
    torch = torch_cuda
    from dlsa_amd._hip import DlsaHipError
    from dlsa_amd.ingest import repartition

    pid = torch.tensor([0, 1, 2, 3], dtype=torch.int32, device="cuda")
    with pytest.raises(DlsaHipError, match="outside"):
        repartition(pid, 3, torch.zeros((4, 2), dtype=torch.float64, device="cuda"))


def _write_csv(path, rs, n):
    import pandas as pd

    a = rs.randn(n)
    b = rs.rand(n) * 10
    eta = 0.4 * a - 0.1 * (b - 5)
    delay = np.where(rs.rand(n) < 1 / (1 + np.exp(-eta)), rs.randint(1, 60, n), -rs.randint(0, 5, n))
    df = pd.DataFrame({"a": a, "b": b, "junk": rs.rand(n), "ArrDelay": delay.astype(float)})
    df.loc[rs.choice(n, 25, replace=False), "a"] = np.nan  # dropna() rows
    df.to_csv(path, index=False)
    return df


def test_read_csv_partitioned_fit_vs_oracle(torch_cuda, tmp_path):
    """CSV -> select/dropna/binarise (logistic_dlsa.py:226-239) -> row % K
    partitions -> HBM layout -> batched fit; the same steps in pandas + the
    oracle give the same estimates."""
    from dlsa_amd.ingest import read_csv_partitioned
    from dlsa_amd.models import logistic_model_batched

    rs = np.random.RandomState(3)
    df = _write_csv(tmp_path / "air.csv", rs, 30000)
    lay = read_csv_partitioned(str(tmp_path / "air.csv"), "ArrDelay", ["a", "b"],
                               sample_size_per_partition=10000)
    ref = df[["a", "b", "ArrDelay"]].dropna().reset_index(drop=True)
    yref = (ref["ArrDelay"] > 0).to_numpy(float)
    Xref = ref[["a", "b"]].to_numpy()
    K = lay["K"]
    assert K == int(np.ceil(len(ref) / 10000))
    order, off = O.systematic_partition(np.arange(len(ref)) % K)
    assert np.array_equal(lay["offsets"], off)
    assert np.array_equal(lay["X"].cpu().numpy(), Xref[order])
    assert np.array_equal(lay["y"].cpu().numpy(), yref[order])
    fit = logistic_model_batched(lay["X"], lay["y"], lay["offsets"], fit_intercept=True)
    th, S, St, ll, it = O.logistic_fit_partitions(Xref[order], yref[order], off,
                                                  fit_intercept=True)
    assert np.abs(fit.theta.cpu().numpy() - th).max() / np.abs(th).max() < 1e-8
    assert np.abs(fit.sig_inv.cpu().numpy() - S).max() / np.abs(S).max() < 1e-8


def test_read_csv_partitioned_dummies(torch_cuda, tmp_path, golden_dir):
    """CSV with string/int factors -> categorical-code HBM layout (the
    reference's dummy semantics) -> categorical fit == oracle on the
    reference design of each partition."""
    from test_oracle_golden import _dummy_fixture

    from dlsa_amd.ingest import read_csv_partitioned
    from dlsa_amd.models import logistic_model_batched_categorical

    g, df, dinfo, base, info = _dummy_fixture(golden_dir)
    df = df[df["partition_id"] < 4].drop(columns=["partition_id"])
    df.to_csv(tmp_path / "d.csv", index=False)
    cols = ["Month", "UniqueCarrier", "Origin", "Distance", "DepTime"]
    lay = read_csv_partitioned(str(tmp_path / "d.csv"), "label", cols, K=3, dummy_info=dinfo,
                               dummy_factors_baseline=base)
    fit = logistic_model_batched_categorical(lay["Xn"], lay["codes"], lay["y"], lay["offsets"],
                                             lay["levels"], fit_intercept=True)
    assert (fit.status.cpu().numpy() == 0).all()
    order, off = O.systematic_partition(np.arange(len(df)) % 3)
    d = df.reset_index(drop=True).iloc[order].reset_index(drop=True)
    for k in range(3):
        part = d.iloc[off[k]:off[k + 1]]
        X, names, missing = O.dummy_design({c: part[c].to_numpy() for c in ("Distance", "DepTime")},
                                           {c: part[c].to_numpy() for c in
                                            ("Month", "UniqueCarrier", "Origin")}, dinfo, base)
        assert names == lay["cols"] and not missing
        r = O.logistic_fit(X, part["label"].to_numpy(float), fit_intercept=True)
        assert np.abs(fit.theta[k].cpu().numpy() - r["coef"]).max() / np.abs(r["coef"]).max() < 1e-8
        assert np.abs(fit.sig_inv[k].cpu().numpy() - r["Sig_inv"]).max() / \
            np.abs(r["Sig_inv"]).max() < 1e-8


def test_read_csv_partitioned_unknown_level_zero_frame(torch_cuda, tmp_path, golden_dir):
    """A factor value that is neither selected nor a baseline (an airport
    dummy_info has never seen): the reference's column-set check fails for
    that chunk (models.py:84-91) and it returns the zero frame.  The ingest
    reports the partition in ``zero_partitions`` and the fit returns the zero
    frame with status missing_level there; the other partitions are fitted
    as usual."""
    from test_oracle_golden import _dummy_fixture

    from dlsa_amd.ingest import read_csv_partitioned
    from dlsa_amd.models import logistic_model_batched_categorical

    g, df, dinfo, base, info = _dummy_fixture(golden_dir)
    df = df[df["partition_id"] < 4].drop(columns=["partition_id"]).reset_index(drop=True)
    df["Origin"] = df["Origin"].astype(str)
    bad_row = 301
    df.loc[bad_row, "Origin"] = "ZZZ_unseen"
    df.to_csv(tmp_path / "u.csv", index=False)
    cols = ["Month", "UniqueCarrier", "Origin", "Distance", "DepTime"]
    lay = read_csv_partitioned(str(tmp_path / "u.csv"), "label", cols, K=3, dummy_info=dinfo,
                               dummy_factors_baseline=base)
    assert lay["zero_partitions"].tolist() == [bad_row % 3]
    fit = logistic_model_batched_categorical(lay["Xn"], lay["codes"], lay["y"], lay["offsets"],
                                             lay["levels"], fit_intercept=True,
                                             zero_partitions=lay["zero_partitions"])
    st = fit.status.cpu().numpy()
    k0 = bad_row % 3
    assert st[k0] == 5 and (np.delete(st, k0) == 0).all()
    assert not fit.theta[k0].abs().max().item() and not fit.sig_inv[k0].abs().max().item()
    order, off = O.systematic_partition(np.arange(len(df)) % 3)
    d = df.iloc[order].reset_index(drop=True)
    for k in range(3):
        if k == k0:
            continue
        part = d.iloc[off[k]:off[k + 1]]
        X, names, missing = O.dummy_design({c: part[c].to_numpy() for c in ("Distance", "DepTime")},
                                           {c: part[c].to_numpy() for c in
                                            ("Month", "UniqueCarrier", "Origin")}, dinfo, base)
        assert not missing
        r = O.logistic_fit(X, part["label"].to_numpy(float), fit_intercept=True)
        assert np.abs(fit.theta[k].cpu().numpy() - r["coef"]).max() / np.abs(r["coef"]).max() < 1e-8


def test_csv_to_config3_fit_needs_no_reference_code(torch_cuda, tmp_path):
    """End to end on the product alone: CSV -> dummy-level selection over the
    file (dlsa_amd.dummies, = dummies.py:111-146) -> categorical-code HBM
    layout (read_csv_partitioned) -> categorical fit; every partition against
    the oracle on the reference's dense dummy design."""
    import os
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden"))
    import dummy_csv as DC

    from dlsa_amd.dummies import select_dummy_factors_from_file
    from dlsa_amd.ingest import read_csv_partitioned, read_table
    from dlsa_amd.models import logistic_model_batched_categorical

    path = tmp_path / "air.csv"
    path.write_text(DC.text(DC.rows()))
    factors = ["Month", "UniqueCarrier", "Origin"]
    info = select_dummy_factors_from_file(str(path), True, factors, [1, 0.8, 0.9], "000_OTHERS")
    base = ["Month_1", "UniqueCarrier_000_OTHERS", "Origin_000_OTHERS"]
    cols = factors + ["Distance"]
    lay = read_csv_partitioned(str(path), "ArrDelay", cols, K=4, dummy_info=info,
                               dummy_factors_baseline=base)
    assert lay["zero_partitions"].size == 0
    fit = logistic_model_batched_categorical(lay["Xn"], lay["codes"], lay["y"], lay["offsets"],
                                             lay["levels"], fit_intercept=True,
                                             center=[900.0], scale=[800.0])
    assert (fit.status.cpu().numpy() == 0).all()
    df = read_table(str(path), "ArrDelay", cols)
    order, off = O.systematic_partition(np.arange(len(df)) % 4)
    d = df.iloc[order].reset_index(drop=True)
    for k in range(4):
        part = d.iloc[off[k]:off[k + 1]]
        X, names, missing = O.dummy_design({"Distance": part["Distance"].to_numpy()},
                                           {c: part[c].to_numpy() for c in factors}, info, base)
        assert names == lay["cols"] and not missing
        center = np.array([900.0] + [0.0] * (X.shape[1] - 1))
        scale = np.array([800.0] + [1.0] * (X.shape[1] - 1))
        r = O.logistic_fit(X, part["ArrDelay"].to_numpy(float), fit_intercept=True, center=center,
                           scale=scale)
        assert np.abs(fit.theta[k].cpu().numpy() - r["coef"]).max() / np.abs(r["coef"]).max() < 1e-8
        assert np.abs(fit.sig_inv[k].cpu().numpy() - r["Sig_inv"]).max() / \
            np.abs(r["Sig_inv"]).max() < 1e-8


# ---- data_info on the device (Spark describe(), logistic_dlsa.py:287-298) ------

@pytest.mark.parametrize("n,p", [(10007, 130), (1, 3), (0, 2), (300001, 7)])
def test_column_moments_vs_oracle(torch_cuda, n, p):
    """dlsa_column_moments: count / mean / M2 / min / max per column with NaNs
    skipped, 3 column blocks at p = 130, empty and one-row inputs."""
    from dlsa_amd.ingest import column_moments

    rs = np.random.RandomState(n + p)
    X = rs.randn(n, p) * np.linspace(1e-3, 1e3, p) + np.linspace(-5.0, 5.0, p)
    if n > 10:
        X[rs.choice(n, 9), rs.choice(p, 9)] = np.nan
        X[:, 1] = 4.25  # constant column: M2 exactly 0
    got = column_moments(X)
    ref = O.column_moments(X)
    assert np.array_equal(got[0], ref[0])
    if n == 0:
        assert np.isnan(got[1:]).all()
        return
    assert np.array_equal(got[3:], ref[3:])
    # compensated sums on the device, numpy's pairwise sums in the oracle:
    # agreement to a few ulp of the column's magnitude
    scale = np.nanmax(np.abs(X), axis=0)
    assert (np.abs(got[1] - ref[1]) <= 1e-14 * scale).all()
    assert np.allclose(got[2], ref[2], rtol=1e-12, atol=1e-300)
    if n > 10:
        assert got[2, 1] == 0.0
    assert np.array_equal(column_moments(X), got)  # fixed order: bit-identical


def test_read_csv_data_info_matches_pandas_describe(torch_cuda, tmp_path):
    """read_csv_partitioned returns data_info in Spark's describe().toPandas()
    layout (summary column, string values) over the x columns, the label and
    partition_id; its numbers equal pandas describe() of the same rows."""
    import pandas as pd

    from dlsa_amd.ingest import read_csv_partitioned

    rs = np.random.RandomState(12)
    df = _write_csv(tmp_path / "air.csv", rs, 23456)
    lay = read_csv_partitioned(str(tmp_path / "air.csv"), "ArrDelay", ["a", "b"], K=7)
    info = lay["data_info"]
    assert list(info.columns) == ["summary", "a", "b", "ArrDelay", "partition_id"]
    assert info["summary"].tolist() == ["count", "mean", "stddev", "min", "max"]
    ref = df[["a", "b", "ArrDelay"]].dropna().reset_index(drop=True)
    ref["ArrDelay"] = (ref["ArrDelay"] > 0).astype(float)
    ref["partition_id"] = (np.arange(len(ref)) % 7).astype(float)
    pdd = ref.describe()
    for c in ["a", "b", "ArrDelay", "partition_id"]:
        assert int(info[c][0]) == int(pdd[c]["count"]) == len(ref)
        for row, key in ((1, "mean"), (2, "std"), (3, "min"), (4, "max")):
            assert abs(float(info[c][row]) - pdd[c][key]) <= 1e-13 * max(1.0, abs(pdd[c][key]))


def test_standardized_fit_through_device_data_info(torch_cuda, golden_dir):
    """The golden data_info (numpy mean / stddev(n-1) in the describe layout)
    equals the device describe() of the fixture's X, and the standardised fit
    through the device frame (models.py:99-101) matches the reference's
    standardized_intercept outputs."""
    import os

    from dlsa_amd.ingest import describe
    from dlsa_amd.models import logistic_model_batched

    D = np.load(os.path.join(golden_dir, "standardized_intercept.npz"))
    info = describe(D["X"], ["a", "b", "c", "d", "e"])
    center = np.array([float(v) for v in info.iloc[1, 1:]])
    scale = np.array([float(v) for v in info.iloc[2, 1:]])
    assert np.allclose(center, D["center"], rtol=1e-14, atol=1e-15)
    assert np.allclose(scale, D["scale"], rtol=1e-14, atol=0)
    order, off = O.systematic_partition(np.arange(len(D["y"])) % 3)
    fit = logistic_model_batched(D["X"][order], D["y"][order], off, fit_intercept=True,
                                 center=center, scale=scale)
    ref = D["outs"]
    assert np.abs(fit.theta.cpu().numpy() - ref[:, :, 1]).max() / np.abs(ref[:, :, 1]).max() < 1e-8
    assert np.abs(fit.sig_inv.cpu().numpy() - ref[:, :, 3:]).max() / np.abs(ref[:, :, 3:]).max() < 1e-8


def _ingest_rank(rank, world, port, path, q):
    import os

    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dlsa_amd.ingest import read_csv_partitioned

        lay = read_csv_partitioned(path, "ArrDelay", ["a", "b"], K=6, rank=rank, world=world)
        q.put((rank, lay["data_info"].to_numpy().tolist(), lay["partitions"].tolist(),
               lay["offsets"].tolist(), lay["X"].cpu().numpy()))
    finally:
        dist.destroy_process_group()


def test_sharded_ingest_two_ranks_same_data_info(torch_cuda, tmp_path):
    """Two ranks (gloo, one GPU) each ingest their partitions of the CSV
    (3 of K = 6); the data_info they combine through one all-reduce equals
    the one-rank frame, and each rank's rows are its partitions' rows."""
    import multiprocessing as mp
    import socket

    from dlsa_amd.ingest import read_csv_partitioned

    rs = np.random.RandomState(21)
    _write_csv(tmp_path / "air.csv", rs, 12000)
    path = str(tmp_path / "air.csv")
    one = read_csv_partitioned(path, "ArrDelay", ["a", "b"], K=6)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_ingest_rank, args=(r, 2, port, path, q)) for r in range(2)]
    for p_ in ps:
        p_.start()
    res = sorted((q.get(timeout=180) for _ in range(2)), key=lambda t: t[0])
    for p_ in ps:
        p_.join(timeout=60)
        assert p_.exitcode == 0
    ref = one["data_info"].to_numpy()
    assert res[0][1] == res[1][1]
    got = np.array(res[0][1], dtype=object)
    assert (got[0] == ref[0]).all()  # counts exact
    for i in range(1, 5):
        for j in range(1, ref.shape[1]):
            assert abs(float(got[i, j]) - float(ref[i, j])) <= 1e-13 * max(1.0, abs(float(ref[i, j])))
    Xone, off1 = one["X"].cpu().numpy(), one["offsets"]
    for rank, _, parts, offs, X in res:
        assert parts == [3 * rank, 3 * rank + 1, 3 * rank + 2]
        exp = np.concatenate([Xone[off1[k]:off1[k + 1]] for k in parts])
        assert np.array_equal(X, exp)
        assert offs == (np.concatenate([[0], np.cumsum([off1[k + 1] - off1[k] for k in parts])])).tolist()
