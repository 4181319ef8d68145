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
