"""Dummy-level selection (dlsa_amd.dummies, the drop-in for dlsa/dummies.py)
against dummy_info produced by the reference itself: the in-memory path
(dummy_factors_counts + select_dummy_factors, dummies.py:10-108) on the
dummy-branch fixture, and the file path (select_dummy_factors_from_file,
dummies.py:111-146) on a two-buffer CSV, by column names and positions."""

import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _norm(info):
    """JSON-normal form (numpy scalars -> Python) for comparison."""
    return json.loads(json.dumps(info, default=lambda x: x.item()))


def test_select_dummy_factors_matches_reference_fixture(golden_dir, tmp_path):
    import pickle

    from test_oracle_golden import _dummy_fixture

    from dlsa_amd.dummies import dummy_factors_counts, select_dummy_factors

    g, df, dinfo, base, info = _dummy_fixture(golden_dir)
    counts = dummy_factors_counts(df, ["Month", "UniqueCarrier", "Origin"])
    pk = tmp_path / "dummy_info.pkl"
    got = select_dummy_factors(counts, keep_top=[1, 0.8, 0.9], replace_with="000_OTHERS",
                               pickle_file=str(pk))
    assert _norm(got) == dinfo
    with open(pk, "rb") as fh:  # written by this test (the product's own pickle)
        assert _norm(pickle.load(fh)) == dinfo
    # positions select the same columns
    cols = df.columns.tolist()
    by_pos = dummy_factors_counts(df, [cols.index(c) for c in ("Month", "UniqueCarrier",
                                                               "Origin")])
    assert list(by_pos) == ["Month", "UniqueCarrier", "Origin"]


def _csv(tmp_path):
    sys.path.insert(0, os.path.join(HERE, "golden"))
    import dummy_csv as DC

    path = tmp_path / "air.csv"
    path.write_text(DC.text(DC.rows()))
    return str(path)


@pytest.mark.parametrize("tag,cols,keep", [("names", ["Month", "UniqueCarrier", "Origin"],
                                            [1, 0.8, 0.9]),
                                           ("positions", [2, 1], [0.75, 0.95])])
def test_select_dummy_factors_from_file_matches_reference(golden_dir, tmp_path, tag, cols, keep):
    from dlsa_amd.dummies import readlines_batches, select_dummy_factors_from_file

    g = np.load(os.path.join(golden_dir, "dummy_file.npz"))
    path = _csv(tmp_path)
    data = open(path, "rb").read()
    assert len(readlines_batches(data)) == int(g["n_buffers"]) == 2
    got = select_dummy_factors_from_file(path, True, cols, keep, "000_OTHERS", None)
    assert _norm(got) == json.loads(str(g["info_" + tag]))


def test_file_selection_keeps_first_buffer_order(tmp_path):
    """The merged counts follow the first buffer's value_counts order (the
    reference's cumsum_dicts), which here differs from the global frequency
    order -- the selection must use the former to match the reference."""
    import pandas as pd

    from dlsa_amd.dummies import readlines_batches, select_dummy_factors_from_file

    path = _csv(tmp_path)
    info = select_dummy_factors_from_file(path, True, ["UniqueCarrier"], [0.8], "000_OTHERS")
    df = pd.read_csv(path, dtype=str)
    a, b = readlines_batches(open(path, "rb").read())[0]
    first = pd.read_csv(path, dtype=str, nrows=open(path, "rb").read()[a:b].count(b"\n") - 1)
    assert info["factor_set"]["UniqueCarrier"][: 4] == \
        list(first["UniqueCarrier"].value_counts().index[: 4])
    assert list(df["UniqueCarrier"].value_counts().index) != info["factor_set"]["UniqueCarrier"]


def test_readlines_batches_match_python(tmp_path):
    from dlsa_amd.dummies import readlines_batches

    rs = np.random.RandomState(0)
    for trial in range(4):
        lines = [("x" * rs.randint(0, 4000)) + "\n" for _ in range(rs.randint(1, 2000))]
        if trial % 2:
            lines[-1] = lines[-1].rstrip("\n")
        p = tmp_path / f"t{trial}.txt"
        p.write_text("".join(lines))
        ref, pos = [], 0
        with open(p) as f:
            while True:
                b = f.readlines(1024000)
                if not b:
                    break
                n = sum(len(x) for x in b)
                ref.append((pos, pos + n))
                pos += n
        assert readlines_batches(p.read_bytes()) == ref


@pytest.mark.parametrize("kind", ["blank", "whitespace", "short", "long", "header_mismatch"])
def test_file_selection_blank_and_ragged_lines_follow_reference_loop(tmp_path, kind):
    """Inputs the pyarrow fast path cannot parse like the reference's
    split-per-line loop (dummies.py:111-146): a blank line is a row whose
    first field is "" (value_counts counts it), a short row is padded with
    None (not counted), a long row widens the frame.  The product must give
    the line loop's result (here: the module's own restatement of that loop,
    which is the reference's code path step for step)."""
    from dlsa_amd.dummies import _select_from_file_textmode, select_dummy_factors_from_file

    rng = np.random.default_rng(7)
    rows = [f"{rng.integers(0, 5)},{rng.choice(['a', 'b', 'c'])},{rng.random():.4f}"
            for _ in range(3000)]
    if kind == "blank":
        rows[100] = ""
        rows[2000] = ""
    elif kind == "whitespace":
        rows[50] = "   "
    elif kind == "short":
        rows[10] = "3,b"
        rows[2500] = "1"
    elif kind == "long":
        rows[7] = "2,a,0.5,extra"
    header = kind == "header_mismatch"
    text = ("A,B\n" if header else "") + "\n".join(rows) + "\n"
    path = tmp_path / "f.csv"
    path.write_text(text)
    cols = ["A", "B"] if header else [0, 1]
    args = (str(path), header, cols, [0.9, 1.0], "000_OTHERS")
    try:
        want = _select_from_file_textmode(*args, None)
    except Exception as e:  # the reference loop's own failure must be reproduced
        with pytest.raises(type(e)):
            select_dummy_factors_from_file(*args)
        return
    got = select_dummy_factors_from_file(*args)
    assert _norm(got) == _norm(want)
