"""Stage cycles of wide_newton_kernel (profiling build DLSA_WN_PROF, run with
DLSA_LIB=var/libdlsa_hip_wnprof.so): config-5 fits (n = 5e6, p = 500, K = 32),
counters summed over the measured fits and reported per workgroup run."""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from dlsa_amd import _hip  # noqa: E402
from dlsa_amd.models import logistic_model_batched, simulate_logistic_device  # noqa: E402

n, p, K = 5_000_000, 500, 32
dev = torch.device("cuda:0")
X, y = simulate_logistic_device(n, p, seed=2019, row0=0, device=dev)
off = (np.arange(K + 1, dtype=np.int64) * n) // K
lib = _hip.load()
rd = lib.dlsa_wn_prof_read
buf = (ctypes.c_ulonglong * 16)()
logistic_model_batched(X, y, off, device=dev)  # warm-up
rd(buf)
fits = 3
for _ in range(fits):
    logistic_model_batched(X, y, off, device=dev)
rd(buf)
v = list(buf)
runs = max(v[8], 1)
names = ["prologue factor", "panel solve (trsm)", "update: next panel cols (U1)",
         "wave 0: next diagonal factor (D)", "wave 0: wait after D", "wave 1: rest of update (U2)",
         "forward solve", "backward solve"]
print(f"workgroup runs reaching the factorization: {runs} ({runs / fits:.0f} per fit)")
print(f"{'steps 1-3 (gradient, publication)':40s} {v[9] / runs:12.0f}")
for i, nm in enumerate(names):
    print(f"{nm:40s} {v[i] / runs:12.0f}")
tot = v[9] + v[0] + v[1] + v[2] + v[3] + v[4] + v[6] + v[7]
print(f"{'total (wave 0 path)':40s} {tot / runs:12.0f}")
