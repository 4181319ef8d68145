#!/usr/bin/env python3
"""The first full-data pass of a fit that starts after the GPU sat idle
(VERDICT r5 item 6).  Config-2 data (n = 1e8, p = 100, K = 1024): one warm-up
fit, then fits after a host sleep of 0, 20, 100, 300 ms, each with and without
a ~30 ms busy kernel stream just before the fit (--prewarm), so the kernel
trace (rocprofv3 --kernel-trace, tools/gpu.sh `profpy:` step) shows whether
the slow first pass follows the idle time, not the fit's own work.

    rocprofv3 --kernel-trace ... -- python3 tools/idle_ramp.py

Prints one line per fit (the order matches the trace's fits).
"""

import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch

    from dlsa_amd import models as M

    n, p, K = 100_000_000, 100, 1024
    X, y = M.simulate_logistic_device(n, p, seed=2019)
    off = (np.arange(K + 1, dtype=np.int64) * n) // K
    ws = torch.empty((1,), dtype=torch.uint8, device="cuda")
    a = torch.randn((4096, 4096), device="cuda", dtype=torch.float32)

    def fit():
        nonlocal ws
        f = M.logistic_model_batched(X, y, off, workspace=ws)
        if ws.numel() < f.stats["workspace_bytes"]:
            ws = torch.empty((f.stats["workspace_bytes"],), dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        return f

    fit()
    fit()
    for gap_ms in (0, 20, 100, 300):
        for prewarm in (False, True):
            time.sleep(gap_ms / 1e3)
            if prewarm:  # ~30 ms of back-to-back GEMMs right before the fit
                t = time.perf_counter()
                while time.perf_counter() - t < 0.03:
                    a = (a @ a).clamp_(-1, 1)
            t0 = time.perf_counter()
            fit()
            print(f"gap {gap_ms:4d} ms prewarm {int(prewarm)}: fit {1e3 * (time.perf_counter() - t0):.2f} ms",
                  flush=True)


if __name__ == "__main__":
    main()
