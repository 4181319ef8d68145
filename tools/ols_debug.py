"""Debug: OLS fit at p=64 (FULL path) with/without standardisation, dumped to
npz for a cross-library comparison (DLSA_LIB selects the build)."""
import sys
import numpy as np
sys.path.insert(0, ".")
from dlsa_amd import models as M  # noqa: E402

out = sys.argv[1]
rs = np.random.RandomState(164)
sizes = [3001, 2045, 4093]
n = sum(sizes)
X = rs.rand(n, 64) * 4.0 - 1.0
y = X @ rs.randn(64) + 0.7 + 0.1 * rs.randn(n)
off = np.concatenate([[0], np.cumsum(sizes)])
res = {}
for std in (False, True):
    c = X.mean(0) if std else None
    s = X.std(0) if std else None
    for rpc in (1003, 0):
        f = M.ols_model_batched(X, y, off, fit_intercept=False, center=c, scale=s, rows_per_chunk=rpc)
        key = f"std{int(std)}_rpc{rpc}"
        res[key + "_theta"] = f.theta.cpu().numpy()
        res[key + "_S"] = f.sig_inv.cpu().numpy()
        res[key + "_St"] = f.sig_inv_theta.cpu().numpy()
np.savez(out, **res)
print("saved", out)
