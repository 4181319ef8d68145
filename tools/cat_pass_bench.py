#!/usr/bin/env python3
"""Per-pass timing of the categorical pass (cat_pass_kernel) at config 3's
shape, for A/B runs across library builds (DLSA_LIB) in separate processes.

    DLSA_LIB=var/libdlsa_hip_<v>.so python tools/cat_pass_bench.py [--n 120000000] [--K 120]

Each fit runs max_iter = 1: one full-data Newton pass from theta = 0 plus the
polish pass at the returned theta, i.e. exactly two full
passes whatever the kernel's numerics, so ablation builds time the same work.
Prints one JSON line: the median per-pass time over --rounds fits and the
algorithmic GB/s (8 q + F + 8 bytes per row).
"""

import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=120_000_000)
    ap.add_argument("--K", type=int, default=120)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--tag", default=os.environ.get("DLSA_LIB", "in-tree"))
    args = ap.parse_args()

    import numpy as np
    import torch

    from dlsa_amd import models as M

    Xn, codes, y, levels = M.simulate_categorical(args.n, seed=2019, device="cuda")
    off = (np.arange(args.K + 1, dtype=np.int64) * args.n) // args.K
    row_bytes = 8 * Xn.shape[1] + codes.shape[1] + 8
    per = []
    for r in range(args.rounds + 1):
        fit = M.logistic_model_batched_categorical(Xn, codes, y, off, levels, fit_intercept=True,
                                                   max_iter=1, record_timing=True)
        st = fit.stats
        if r:  # the first fit warms up
            per.append(st["ms_pass_fp64"] / st["passes_fp64"])
        del fit
    torch.cuda.synchronize()
    ms = statistics.median(per)
    print(json.dumps({"lib": args.tag, "n": args.n, "K": args.K, "passes_per_fit": st["passes_fp64"],
                      "ms_per_pass": ms, "ms_all": per,
                      "GBps": args.n * row_bytes / (ms * 1e-3) / 1e9}), flush=True)


if __name__ == "__main__":
    main()
