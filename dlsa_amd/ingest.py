"""Ingest: CSV -> HBM partition layout.

Replaces the reference's Spark read + partitioning in front of the map stage
(projects/logistic_dlsa.py:226-245 and :303-325):

    spark.read.csv(header=True) -> select(usecols_x + [Y]) -> dropna()
    -> Y = (Y > 0) -> partition_id = monotonically_increasing_id() % K
    -> repartition(K, "partition_id") -> groupby("partition_id")

Here the CSV is parsed by pyarrow's multi-threaded C++ reader on the host,
copied to HBM once, and grouped by partition on the GPU with
``dlsa_partition_rows`` (a stable counting sort in HIP; partition_rows.hip).
Spark's ``monotonically_increasing_id`` is the row index for a single input
split (its upper bits hold the split index otherwise); the restatement uses
the row index, i.e. the reference's ``insert_partition_id_pdf`` systematic
assignment (dlsa/utils.py:93-107).  There is no CPU fallback for the
partitioning step.
"""

from __future__ import annotations

import ctypes
import math

import numpy as np

from . import _hip
from .models import _ptr, _require_gpu, _stream, encode_categorical

try:
    import torch
except ImportError:  # pragma: no cover
    torch = None


def systematic_partition_id(n, K, row0=0, device=None):
    """partition_id = (row0 + i) % K as an int32 device tensor (the reference's
    ``monotonically_increasing_id() % K`` for one split,
    projects/logistic_dlsa.py:243-245)."""
    dev = _require_gpu(device)
    return ((torch.arange(int(n), dtype=torch.int64, device=dev) + int(row0)) % int(K)).to(
        torch.int32)


def repartition(part_id, K, *arrays, return_order=False, device=None):
    """Group the rows of ``arrays`` (device tensors with n rows, any dtype,
    row-major) by ``part_id`` ([n] ids in [0, K)) on the GPU: returns
    (list of partition-contiguous copies, offsets [K+1] numpy int64[, order]).
    Stable: rows keep their input order inside each partition -- what
    ``repartition(K, "partition_id")`` + ``groupby`` hand to the map stage."""
    dev = _require_gpu(device)
    pid = part_id.to(device=dev, dtype=torch.int32).contiguous().reshape(-1)
    n = pid.numel()
    K = int(K)
    if len(arrays) > 4:
        raise ValueError("at most 4 arrays per call")
    srcs, dsts, widths = [], [], []
    for a in arrays:
        if not isinstance(a, torch.Tensor) or a.device != pid.device:
            raise ValueError("arrays must be tensors on the partition ids' device")
        if a.shape[0] != n:
            raise ValueError("every array needs n rows")
        a = a.contiguous()
        srcs.append(a)
        dsts.append(torch.empty_like(a))
        widths.append(a.element_size() * (a.numel() // max(n, 1)) if n else a.element_size())
    order = torch.empty((n,), dtype=torch.int64, device=dev) if return_order else None
    offsets = np.zeros(K + 1, dtype=np.int64)
    na = len(srcs)
    src_arr = (ctypes.c_void_p * max(na, 1))(*[a.data_ptr() for a in srcs])
    dst_arr = (ctypes.c_void_p * max(na, 1))(*[a.data_ptr() for a in dsts])
    rb_arr = (ctypes.c_int64 * max(na, 1))(*widths)
    lib = _hip.load()
    rc = lib.dlsa_partition_rows(_ptr(pid), n, K, na, src_arr, dst_arr, rb_arr,
                                 offsets.ctypes.data_as(ctypes.c_void_p), _ptr(order), _stream(dev))
    _hip.check(rc, "dlsa_partition_rows")
    if return_order:
        return dsts, offsets, order
    return dsts, offsets


def read_table(path, Y_name, usecols_x, read_options=None):
    """Host half of the ingest: pyarrow CSV reader (header row), select
    ``usecols_x + [Y_name]``, drop rows with a null in them, binarise Y
    (Y > 0 -> 1, else 0) -- projects/logistic_dlsa.py:226-239.  Returns a
    pandas DataFrame (numeric columns float64, others as read)."""
    import pyarrow.csv as pacsv

    cols = list(usecols_x) + [Y_name]
    tab = pacsv.read_csv(path, read_options=read_options,
                         convert_options=pacsv.ConvertOptions(include_columns=cols))
    df = tab.to_pandas()
    df = df[cols].dropna().reset_index(drop=True)
    df[Y_name] = (df[Y_name] > 0).astype(np.float64)
    return df


def read_csv_partitioned(path, Y_name, usecols_x, K=None, sample_size_per_partition=None,
                         dummy_info=None, dummy_factors_baseline=(), device=None):
    """CSV -> fit-ready HBM layout.

    ``K`` partitions, or ``ceil(n / sample_size_per_partition)`` like the
    reference (logistic_dlsa.py:236-238).  Without ``dummy_info`` returns a
    dict with ``X`` [n, p] fp64 (columns ``usecols_x`` in order), ``y``,
    ``offsets``, ``columns``; with it, the categorical-code layout of
    ``encode_categorical`` (``Xn``, ``codes``, ``levels``, ``cols``, ...) for
    ``logistic_model_batched_categorical``; ``zero_partitions`` lists the
    partitions holding a factor value that is neither selected nor a baseline
    (their rows are coded as the baseline; pass the list on to the fit, which
    returns the reference's zero frame for them, models.py:84-91)."""
    dev = _require_gpu(device)
    df = read_table(path, Y_name, usecols_x)
    n = len(df)
    if K is None:
        if not sample_size_per_partition:
            raise ValueError("give K or sample_size_per_partition")
        K = max(1, math.ceil(n / sample_size_per_partition))
    pid = systematic_partition_id(n, K, device=dev)
    y = torch.from_numpy(df[Y_name].to_numpy(dtype=np.float64)).pin_memory().to(dev,
                                                                               non_blocking=True)
    if dummy_info:
        df.insert(0, "partition_id", 0.0)
        enc = encode_categorical(df, Y_name, dummy_info, dummy_factors_baseline)
        Xn = torch.from_numpy(enc["Xn"]).pin_memory().to(dev, non_blocking=True)
        codes = torch.from_numpy(enc["codes"]).pin_memory().to(dev, non_blocking=True)
        (Xp, cp, yp), offsets = repartition(pid, K, Xn, codes, y, device=dev)
        zero = np.unique(np.nonzero(enc["unknown_rows"])[0] % K).astype(np.int64)
        return {"Xn": Xp, "codes": cp, "y": yp, "offsets": offsets, "levels": enc["levels"],
                "numeric": enc["numeric"], "cols": enc["cols"], "K": K, "zero_partitions": zero}
    X = torch.from_numpy(np.ascontiguousarray(df[list(usecols_x)].to_numpy(dtype=np.float64)))
    X = X.pin_memory().to(dev, non_blocking=True)
    (Xp, yp), offsets = repartition(pid, K, X, y, device=dev)
    return {"X": Xp, "y": yp, "offsets": offsets, "columns": list(usecols_x), "K": K}
