#!/usr/bin/env python3
"""Throughput of the HBM repartition (dlsa_partition_rows): X [n, p] fp64 +
y grouped into K partitions by partition_id = row % K (config-2 shape by
default, n reduced so input + output fit comfortably).  Prints one JSON line:
GB/s = (read + write of every row + 2 reads of the 4-byte id) / kernel time."""

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20_000_000)
    ap.add_argument("--p", type=int, default=100)
    ap.add_argument("--K", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch

    from dlsa_amd.ingest import repartition, systematic_partition_id
    from dlsa_amd.models import simulate_logistic_device

    X, y = simulate_logistic_device(args.n, args.p, seed=1)
    pid = systematic_partition_id(args.n, args.K)
    repartition(pid, args.K, X, y)  # warm-up
    torch.cuda.synchronize()
    ts = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        out, off = repartition(pid, args.K, X, y)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
        del out
    t = min(ts)
    bytes_ = args.n * (2 * (8 * args.p + 8) + 8)
    print(json.dumps({"kernel": "dlsa_partition_rows (count + scan + scatter)", "n": args.n,
                      "p": args.p, "K": args.K, "ms": t * 1e3, "GBps": bytes_ / t / 1e9,
                      "frac_of_8TBps": bytes_ / t / 8e12, "ms_all": [x * 1e3 for x in ts]}))


if __name__ == "__main__":
    main()
