"""Cross-build check of the categorical pass: one config-3-shaped fit (9 numeric
+ 5 factors, P = 182, 16 partitions of 62,500 rows, skewed codes) with the
library DLSA_LIB names, outputs saved to <out>.npz; with --compare A B, the two
saves must be bit-identical (the one-hot histograms are order-free int64 sums,
so a change in the kernel's schedule cannot move a bit)."""
import sys

import numpy as np

if sys.argv[1] == "--compare":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    same = all(np.array_equal(a[k], b[k]) for k in a.files)
    print({"bit_identical": same, "keys": a.files})
    sys.exit(0 if same else 1)

import torch  # noqa: E402

from dlsa_amd import models as M  # noqa: E402

Xn, codes, y, levels = M.simulate_categorical(16 * 62500, seed=5, device="cuda")
off = np.arange(17, dtype=np.int64) * 62500
fit = M.logistic_model_batched_categorical(Xn, codes, y, off, levels, fit_intercept=True)
torch.cuda.synchronize()
np.savez(sys.argv[1], theta=fit.theta.cpu().numpy(), sig_inv=fit.sig_inv.cpu().numpy(),
         loglik=fit.loglik.cpu().numpy(), status=fit.status.cpu().numpy())
print({"saved": sys.argv[1], "status0": int((fit.status.cpu().numpy() == 0).sum())})
