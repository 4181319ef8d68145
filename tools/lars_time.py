#!/usr/bin/env python3
"""Host LARS/DBIC path time at the BASELINE sizes (P = 100, 182, 500), best of 5."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from dlsa_amd import _hip  # noqa: E402
from dlsa_amd.lsa import lars_lsa  # noqa: E402

_hip.load()
for P in (100, 182, 500):
    rs = np.random.RandomState(0)
    A = rs.randn(3 * P, P)
    S = A.T @ A * 1000
    b = rs.randn(P) * (rs.rand(P) < 0.4) + rs.randn(P) * 0.01
    ts = []
    for _ in range(5):
        t = time.perf_counter()
        lars_lsa(S, b, False, 10 ** 8, type="lasso")
        ts.append(time.perf_counter() - t)
    print(P, "lasso ms best/median", round(min(ts) * 1e3, 2), round(sorted(ts)[2] * 1e3, 2))
