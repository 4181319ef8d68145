"""Host WLSE + LARS timing at config-5 size (P = 500).  (A spinning worker
pool splitting the equiangular product over 4 / 8 threads measured 23 / 31 ms
against 15.4 ms serial on the GPU box's host: removed.)"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    rs = np.random.RandomState(0)
    P, n = 500, 5_000_000
    X = rs.rand(20000, P) - 0.5
    S = X.T @ X * (n / 20000) * 0.2
    beta = np.zeros(P)
    beta[:200] = 1
    est = np.linalg.solve(S, S @ (beta + 0.05 * rs.randn(P)))
    from dlsa_amd.dlsa import wlse
    v = S @ est
    for _ in range(3):
        t = time.perf_counter()
        wlse(S, v)
        print(f"wlse (Cholesky) {(time.perf_counter() - t) * 1e3:.1f} ms", flush=True)
    import scipy.linalg as sla
    for _ in range(2):
        t = time.perf_counter()
        sla.cho_factor(S, lower=True, check_finite=True)
        print(f"  cho_factor alone {(time.perf_counter() - t) * 1e3:.1f} ms", flush=True)
    ref = None
    for thr in ("1",):
        from dlsa_amd.lsa import lars_lsa
        ts = []
        for _ in range(5):
            t = time.perf_counter()
            r = lars_lsa(S, est, False, n, type="lasso")
            ts.append(time.perf_counter() - t)
        same = ref is None or np.array_equal(ref, r["beta"])
        ref = r["beta"] if ref is None else ref
        print(f"lars: min {min(ts) * 1e3:.1f} ms median {sorted(ts)[2] * 1e3:.1f} ms "
              f"steps {len(r['BIC'])} identical {same}", flush=True)


if __name__ == "__main__":
    main()
