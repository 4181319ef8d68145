#!/usr/bin/env python3
"""Newton-solve cost breakdown: K partitions of P = 101 with few rows, so the
pass is negligible; 1 vs 8 chunks per partition separates the partial-tile
assembly from the factorisation."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from dlsa_amd.models import logistic_model_batched, simulate_logistic_device

K, nk, p = 1024, 4096, 100
X, y = simulate_logistic_device(K * nk, p, seed=3)
off = np.arange(K + 1, dtype=np.int64) * nk
for rpc in (nk, nk // 8):
    for rep in range(2):
        f = logistic_model_batched(X, y, off, record_timing=True, rows_per_chunk=rpc)
    st = f.stats
    print(f"chunks/partition={nk // rpc}: iterations {st['iterations']}, solve ms/iter "
          f"{st['ms_solve'] / st['iterations']:.3f}, pass ms {st['ms_pass_fp32'] + st['ms_pass_fp64']:.2f}")
