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


DESCRIBE_ROWS = ("count", "mean", "stddev", "min", "max")


def column_moments(X, device=None):
    """Column moments of a 2-D fp64 array on the GPU (``dlsa_column_moments``,
    moments.hip): a host ndarray [5, p] = count, mean, M2 (sum of squared
    deviations), min, max per column; NaNs are skipped."""
    dev = _require_gpu(device)
    if isinstance(X, torch.Tensor):
        Xd = X.to(device=dev, dtype=torch.float64)
    else:
        Xd = torch.from_numpy(np.ascontiguousarray(np.asarray(X, dtype=np.float64))).to(dev)
    if Xd.dim() == 1:
        Xd = Xd.reshape(-1, 1)
    Xd = Xd.contiguous()
    n, p = Xd.shape
    out = torch.empty((5, p), dtype=torch.float64, device=dev)
    rc = _hip.load().dlsa_column_moments(_ptr(Xd) if n else None, n, p, _ptr(out), _stream(dev))
    _hip.check(rc, "dlsa_column_moments")
    return out.cpu().numpy()


def merge_moments(parts):
    """Combine the [5, p] moments of disjoint row sets, in the given order
    (Chan et al.'s pairwise update of mean and M2; min / max of the parts)."""
    acc = None
    for m in parts:
        m = np.asarray(m, dtype=np.float64)
        if acc is None:
            acc = m.copy()
            continue
        na, nb = acc[0], m[0]
        n = na + nb
        with np.errstate(invalid="ignore", divide="ignore"):
            d = m[1] - acc[1]
            mean = np.where(nb == 0, acc[1], np.where(na == 0, m[1], acc[1] + d * (nb / n)))
            m2 = np.where(nb == 0, acc[2], np.where(na == 0, m[2],
                                                    acc[2] + m[2] + d * d * (na * nb / n)))
        acc = np.stack([n, mean, m2, np.fmin(acc[3], m[3]), np.fmax(acc[4], m[4])])
    return acc


def combine_moments(local, group=None, distributed=False):
    """The moments of the whole sharded data set on every rank: each rank's
    [5, p] local moments go through ONE all-reduce (a zero [world, 5, p]
    buffer with this rank's row filled -- an all-gather), then merge in rank
    order, so every rank gets the bit-identical result.  Only with a
    ``group`` or ``distributed=True`` (the default process group); otherwise
    the local moments are returned."""
    local = np.asarray(local, dtype=np.float64)
    import torch.distributed as dist

    if group is None and not distributed:
        return local
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = "cpu"
    if dist.get_backend(group) == "nccl":
        dev = torch.device("cuda", torch.cuda.current_device())
    buf = torch.zeros((world,) + local.shape, dtype=torch.float64, device=dev)
    buf[rank] = torch.from_numpy(local).to(dev)
    dist.all_reduce(buf, group=group)
    return merge_moments(list(buf.cpu().numpy()))


def describe_frame(moments, columns):
    """Spark's ``describe().toPandas()`` layout from [5, p] moments: a
    ``summary`` column with rows count / mean / stddev (n - 1) / min / max and
    one column per input column, every value a string (``repr`` of the
    double, so ``float()`` recovers it exactly; count as an integer) -- the
    ``data_info`` frame logistic_model reads (dlsa/models.py:99-101 takes
    rows 1 and 2)."""
    import pandas as pd

    m = np.asarray(moments, dtype=np.float64)
    info = pd.DataFrame({"summary": list(DESCRIBE_ROWS)})
    for j, c in enumerate(columns):
        n = m[0, j]
        std = float(np.sqrt(m[2, j] / (n - 1))) if n > 1 else float("nan")
        info[c] = [str(int(n)), repr(float(m[1, j])), repr(std), repr(float(m[3, j])),
                   repr(float(m[4, j]))]
    return info


def describe(X, columns, group=None, distributed=False, device=None):
    """data_info on the GPU: describe() of the columns of X (device moments,
    combined across the ranks of ``group`` / the default process group when
    ``distributed``) in the reference's layout (projects/logistic_dlsa.py:
    287-298)."""
    return describe_frame(
        combine_moments(column_moments(X, device=device), group, distributed), columns)


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
                         dummy_info=None, dummy_factors_baseline=(), device=None,
                         rank=0, world=1, group=None, with_data_info=True):
    """CSV -> fit-ready HBM layout.

    ``K`` partitions, or ``ceil(n / sample_size_per_partition)`` like the
    reference (logistic_dlsa.py:236-238).  Without ``dummy_info`` returns a
    dict with ``X`` [n, p] fp64 (columns ``usecols_x`` in order), ``y``,
    ``offsets``, ``columns``; with it, the categorical-code layout of
    ``encode_categorical`` (``Xn``, ``codes``, ``levels``, ``cols``, ...) for
    ``logistic_model_batched_categorical``; ``zero_partitions`` lists the
    partitions holding a factor value that is neither selected nor a baseline
    (their rows are coded as the baseline; pass the list on to the fit, which
    returns the reference's zero frame for them, models.py:84-91).

    Sharded (``world`` > 1, one call per rank): every rank parses the file
    and keeps the rows of its partitions [rank K / world, (rank + 1) K /
    world) -- the partitions dlsa_fit_sharded / bench.py give it -- so X
    lands on the GPU that fits it; ``partitions`` = the global ids of the
    local offsets.

    ``data_info`` (``with_data_info``): the reference's describe() of the
    data set (logistic_dlsa.py:287-298, Spark layout, strings) over the
    numeric columns, the label and partition_id, computed from the device
    copy (``dlsa_column_moments``) and, sharded, combined across the ranks by
    one all-reduce (``group``, or the default process group) -- the global
    mean / stddev logistic_model standardises with (models.py:99-101)."""
    dev = _require_gpu(device)
    df = read_table(path, Y_name, usecols_x)
    n = len(df)
    if K is None:
        if not sample_size_per_partition:
            raise ValueError("give K or sample_size_per_partition")
        K = max(1, math.ceil(n / sample_size_per_partition))
    K, world, rank = int(K), int(world), int(rank)
    if not (0 <= rank < world) or K < world:
        raise ValueError("need 0 <= rank < world <= K")
    k0, k1 = rank * K // world, (rank + 1) * K // world
    gid = np.arange(n, dtype=np.int64) % K  # monotonically_increasing_id() % K
    keep = (gid >= k0) & (gid < k1)
    if world > 1:
        df = df[keep].reset_index(drop=True)
        gid = gid[keep]
    nl = len(df)
    pid = torch.from_numpy((gid - k0).astype(np.int32)).to(dev)
    y = torch.from_numpy(df[Y_name].to_numpy(dtype=np.float64)).pin_memory().to(dev,
                                                                               non_blocking=True)
    out = {"K": K, "partitions": np.arange(k0, k1)}
    if dummy_info:
        df.insert(0, "partition_id", 0.0)
        enc = encode_categorical(df, Y_name, dummy_info, dummy_factors_baseline)
        Xn = torch.from_numpy(enc["Xn"]).pin_memory().to(dev, non_blocking=True)
        codes = torch.from_numpy(enc["codes"]).pin_memory().to(dev, non_blocking=True)
        (Xp, cp, yp), offsets = repartition(pid, k1 - k0, Xn, codes, y, device=dev)
        unknown = np.nonzero(enc["unknown_rows"])[0]
        zero = np.unique(gid[unknown] - k0).astype(np.int64)
        out.update({"Xn": Xp, "codes": cp, "y": yp, "offsets": offsets, "levels": enc["levels"],
                    "numeric": enc["numeric"], "cols": enc["cols"], "zero_partitions": zero})
        Xd, xcols = Xn, list(enc["numeric"])
    else:
        X = torch.from_numpy(np.ascontiguousarray(df[list(usecols_x)].to_numpy(dtype=np.float64)))
        X = X.pin_memory().to(dev, non_blocking=True)
        (Xp, yp), offsets = repartition(pid, k1 - k0, X, y, device=dev)
        out.update({"X": Xp, "y": yp, "offsets": offsets, "columns": list(usecols_x)})
        Xd, xcols = X, list(usecols_x)
    if with_data_info:
        mom = [column_moments(Xd, device=dev) if Xd.shape[1] else np.zeros((5, 0)),
               column_moments(y, device=dev),
               column_moments(torch.from_numpy(gid.astype(np.float64)).to(dev), device=dev)]
        local = np.concatenate(mom, axis=1)
        tot = combine_moments(local, group, distributed=world > 1)
        out["data_info"] = describe_frame(tot, xcols + [Y_name, "partition_id"])
    assert nl == int(offsets[-1])
    return out
