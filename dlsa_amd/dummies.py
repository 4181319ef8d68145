"""Dummy-level selection (drop-in for dlsa/dummies.py of the reference).

The categorical layout of BASELINE config 3 needs ``dummy_info``: which levels
of each factor get a dummy column and which are folded into ``000_OTHERS``.
The reference computes it on the host by streaming the CSV
(dlsa/dummies.py:111-146), counting levels (:10-31, :34-49) and keeping the
levels that cover the top ``keep_top`` fraction (:52-108).  This module
restates that with the same signatures and the same result:

* ``dummy_factors_counts``   -- dummies.py:10-31 (pandas ``value_counts``);
* ``cumsum_dicts``           -- dummies.py:34-49 (``Counter`` merge order);
* ``select_dummy_factors``   -- dummies.py:52-108 (cumulative keep-top);
* ``select_dummy_factors_from_file`` -- dummies.py:111-146, with the file
  parsed by pyarrow's C++ CSV reader instead of a Python ``split`` per line.

The reference's selection depends on the ORDER of the merged counts: each
``readlines(1024000)`` buffer's counts come in ``value_counts`` order and
``cumsum_dicts`` appends the keys a later buffer adds, so on a multi-buffer
file the cumulative percentage runs over first-seen order, not global
frequency.  The restatement keeps that: it cuts the file at exactly the
reference's buffer boundaries (CPython ``IOBase.readlines`` hint rule) and
counts each buffer with the same pandas call.  Host-side work: the counts feed
the encoding (``models.encode_categorical``) that produces the uint8 level
codes the HIP categorical pass consumes.
"""

from __future__ import annotations

import os
import pickle
from collections import Counter

import numpy as np

#: the reference's buffer size hint (dummies.py:121-122)
READLINES_HINT = 1024000


def dummy_factors_counts(pdf, dummy_columns):
    """Level counts of the given columns (dlsa/dummies.py:10-31): a dict
    column -> {level: count} in ``value_counts`` order.  Integer entries of
    ``dummy_columns`` are positions in ``pdf.columns``."""
    cols = pdf.columns.tolist()
    if all(isinstance(c, int) for c in dummy_columns):
        names = [cols[i] for i in dummy_columns]
    else:
        names = dummy_columns
    return {c: pdf[c].value_counts().to_dict() for c in names}


def cumsum_dicts(dict1, dict2):
    """Merge two count dicts (dlsa/dummies.py:34-49): per column
    ``Counter(d1) + Counter(d2)`` -- the keys of d1 in their order, then the
    new keys of d2."""
    if len(dict1) == 0:
        return dict2
    if len(dict2) == 0:
        return dict1
    return {c: dict(Counter(dict1[c]) + Counter(dict2[c])) for c in dict1.keys()}


def select_dummy_factors(dummy_dict, keep_top, replace_with, pickle_file=None):
    """Keep, per column i, the levels whose cumulative count share (in the
    dict's order) is <= keep_top[i]; the others are dropped and represented
    by ``replace_with`` (dlsa/dummies.py:52-108).  Returns ``dummy_info``
    {factor_set, factor_selected, factor_dropped, factor_selected_names} and,
    like the reference, pickles it to ``pickle_file`` when one is given."""
    factor_set, factor_selected, factor_dropped, names = {}, {}, {}, {}
    for i, col in enumerate(list(dummy_dict)):
        levels = list(dummy_dict[col].keys())
        cum = np.cumsum(list(dummy_dict[col].values()))
        share = cum / cum[-1]
        keep = share <= keep_top[i]
        factor_set[col] = levels
        factor_selected[col] = list(np.array(levels)[np.nonzero(keep)[0]])
        factor_dropped[col] = list(np.array(levels)[np.nonzero(~keep)[0]])
        new = [replace_with] if (~keep).any() else []
        new.extend(factor_selected[col])
        names[col] = [col + "_" + str(x) for x in new]
    info = {"factor_set": factor_set, "factor_selected": factor_selected,
            "factor_dropped": factor_dropped, "factor_selected_names": names}
    if pickle_file:
        with open(os.path.expanduser(pickle_file), "wb") as fh:
            pickle.dump(info, fh)
        print("dummy_info saved in:\t" + pickle_file)
    return info


def readlines_batches(data, hint=READLINES_HINT):
    """Byte ranges of the line batches ``f.readlines(hint)`` returns on a
    text file holding ``data`` (ASCII, "\\n" line ends): CPython's
    IOBase.readlines appends lines until one takes the running length past
    ``hint`` -- that line is the batch's last."""
    buf = np.frombuffer(data, dtype=np.uint8)
    ends = np.flatnonzero(buf == 10) + 1          # one past each "\n"
    if len(buf) and (ends.size == 0 or ends[-1] != len(buf)):
        ends = np.append(ends, len(buf))          # last line without "\n"
    out = []
    start, n_lines = 0, ends.size
    while start < n_lines:
        s0 = 0 if start == 0 else int(ends[start - 1])
        # first line j >= start whose end lies past s0 + hint closes the batch
        last = min(int(np.searchsorted(ends, s0 + hint, side="right")), n_lines - 1)
        out.append((s0, int(ends[last])))
        start = last + 1
    return out


def _batch_columns(chunk, ncols_hint=None):
    """Fields of each line of a text chunk split on "," (the reference's
    ``x.strip().split(",")``) as a pyarrow table of strings."""
    import io
    import re

    import pyarrow as pa
    import pyarrow.csv as pacsv

    if re.search(rb"[ \t\v\f]\n|\n[ \t\v\f]|^[ \t\v\f]|[ \t\v\f]$", chunk):
        # some line has surrounding whitespace: strip line by line (rare)
        lines = chunk.decode("ascii").split("\n")
        if lines and lines[-1] == "":
            lines.pop()
        stripped = ("\n".join(x.strip() for x in lines) + "\n").encode("ascii")
    else:
        stripped = chunk if chunk.endswith(b"\n") else chunk + b"\n"
    first = stripped[: stripped.find(b"\n")]
    n = first.count(b",") + 1 if ncols_hint is None else ncols_hint
    ro = pacsv.ReadOptions(column_names=[f"c{j}" for j in range(n)], block_size=1 << 26)
    # empty lines are rows (the reference's split gives them one "" field):
    # with more than one column pyarrow then rejects them as ragged, and the
    # caller falls back to the reference's own loop
    po = pacsv.ParseOptions(delimiter=",", quote_char=False, escape_char=False,
                            newlines_in_values=False, ignore_empty_lines=False)
    co = pacsv.ConvertOptions(column_types={f"c{j}": pa.string() for j in range(n)},
                              strings_can_be_null=False)
    return pacsv.read_csv(io.BytesIO(stripped), read_options=ro, parse_options=po,
                          convert_options=co)


def select_dummy_factors_from_file(file, header, dummy_columns, keep_top, replace_with,
                                   pickle_file=None):
    """Count the levels of ``dummy_columns`` over a CSV file in the
    reference's buffers and select them (dlsa/dummies.py:111-146).  Levels
    are the raw text of the fields (strings), as the reference reads them."""
    import mmap

    path = os.path.expanduser(file)
    if os.path.getsize(path) == 0:
        return select_dummy_factors({}, keep_top, replace_with, pickle_file)
    with open(path, "rb") as fh:
        data = mmap.mmap(fh.fileno(), 0, access=mmap.ACCESS_READ)
    u8 = np.frombuffer(data, dtype=np.uint8)
    if (u8 >= 128).any() or data.find(b"\r") >= 0:
        # non-ASCII text or "\r\n" line ends: the reference's own (slow) loop
        return _select_from_file_textmode(file, header, dummy_columns, keep_top, replace_with,
                                          pickle_file)
    try:
        dummy_dict = _counts_fast(data, header, dummy_columns)
    except _Ragged:
        # blank or whitespace-only lines, rows with a different field count:
        # the reference pads short rows with None (pd.DataFrame of ragged
        # lists) and counts a blank line as a row -- its own loop reproduces
        # that exactly
        return _select_from_file_textmode(file, header, dummy_columns, keep_top, replace_with,
                                          pickle_file)
    return select_dummy_factors(dummy_dict, keep_top, replace_with, pickle_file)


class _Ragged(Exception):
    pass


def _counts_fast(data, header, dummy_columns):
    """Level counts of every readlines buffer (pyarrow parse), merged in the
    reference's order.  Raises _Ragged when a line's field count differs from
    the file's first line (blank lines included)."""
    import pandas as pd
    import pyarrow as pa

    dummy_dict = {}
    names = None
    ncols = None
    for bi, (a, b) in enumerate(readlines_batches(data)):
        chunk = data[a:b]
        if bi == 0 and header is True:
            nl = chunk.find(b"\n")
            head = chunk[: nl if nl >= 0 else len(chunk)].decode("ascii").strip().split(",")
            chunk = chunk[nl + 1:] if nl >= 0 else b""
            names = head
        if not chunk:
            pdf = pd.DataFrame(columns=names if names is not None else [])
            counts = dummy_factors_counts(pdf, dummy_columns)
        else:
            try:
                tab = _batch_columns(chunk, ncols)
            except pa.ArrowInvalid as e:  # a row with another field count
                raise _Ragged(str(e)) from e
            ncols = tab.num_columns
            if names is not None and ncols != len(names):
                raise _Ragged("header and rows differ in field count")
            pdf = pd.DataFrame({(names[j] if names is not None else j): tab.column(j).to_numpy(
                zero_copy_only=False).astype(object) for j in range(tab.num_columns)})
            counts = dummy_factors_counts(pdf, dummy_columns)
        dummy_dict = cumsum_dicts(dummy_dict, counts)
    return dummy_dict


def _select_from_file_textmode(file, header, dummy_columns, keep_top, replace_with, pickle_file):
    """Line-by-line restatement for files the fast path does not cover
    (non-ASCII text, "\\r\\n" line ends, blank lines, ragged rows): the
    reference's own loop (dummies.py:111-146)."""
    import pandas as pd

    dummy_dict = {}
    buffer_num = 0
    head = None
    with open(os.path.expanduser(file)) as f:
        while True:
            buf = f.readlines(READLINES_HINT)
            if len(buf) == 0:
                break
            rows = [x.strip().split(",") for x in buf]
            buffer_num += 1
            start = 0
            if buffer_num == 1 and header is True:
                head = rows[0]
                start = 1
            pdf = pd.DataFrame(rows[start:])
            if header is True:
                pdf.columns = head
            dummy_dict = cumsum_dicts(dummy_dict, dummy_factors_counts(pdf, dummy_columns))
    return select_dummy_factors(dummy_dict, keep_top, replace_with, pickle_file)
