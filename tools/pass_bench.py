#!/usr/bin/env python3
"""A/B timing of the fused IRLS pass across library variants and host knobs,
all in one process on one GPU (rule: interleaved rounds, same device).

    python tools/pass_bench.py [--n 25000000] [--p 100] [--K 256] [--rounds 3]
        [--libs base,ablate1,...] [--knobs "DLSA_WAVES_F32=8;DLSA_WAVES_F32=4"]

Variants are the .so files tools/build_variants.sh produces
(dlsa_amd/libdlsa_hip.so = base, var/libdlsa_hip_<name>.so; host knobs need a
`knobs` build, -DDLSA_ENV_KNOBS=1).
Prints one JSON line per (variant, knob) with the median fp32-/fp64-pass time
and the algorithmic GB/s (n (8p+8) bytes per pass).
"""

import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def load_variant(path):
    from dlsa_amd import _hip

    lib = ctypes.CDLL(path)
    for name, (res, args) in _hip.SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=25_000_000)
    ap.add_argument("--p", type=int, default=100)
    ap.add_argument("--K", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--libs", default="base")
    ap.add_argument("--knobs", default="default",
                    help='";"-separated configs of ","-separated ENV=VAL; "default" = none')
    ap.add_argument("--hessian", default="mixed")
    ap.add_argument("--rows-per-chunk", type=int, default=0)
    ap.add_argument("--warm", type=int, default=0, help="warm-start levels (0: full-row passes only)")
    ap.add_argument("--max-iter", type=int, default=100)
    args = ap.parse_args()

    import numpy as np
    import torch

    from dlsa_amd import _hip
    from dlsa_amd.models import simulate_logistic_device

    dev = torch.device("cuda", 0)
    n, p, K = args.n, args.p, args.K
    X, y = simulate_logistic_device(n, p, seed=2019, device=dev)
    offs = (np.arange(K + 1, dtype=np.int64) * n) // K
    P = p
    theta = torch.empty((K, P), dtype=torch.float64, device=dev)
    sig = torch.empty((K, P, P), dtype=torch.float64, device=dev)
    sigt = torch.empty((K, P), dtype=torch.float64, device=dev)
    ll = torch.empty((K,), dtype=torch.float64, device=dev)
    it = torch.empty((K,), dtype=torch.int32, device=dev)
    st = torch.empty((K,), dtype=torch.int32, device=dev)
    ws = torch.empty((1 << 31,), dtype=torch.uint8, device=dev)
    vp = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)

    libs = {}
    for name in args.libs.split(","):
        path = _hip.LIB_PATH if name == "base" else os.path.join(
            ROOT, "var", f"libdlsa_hip_{name}.so")
        libs[name] = load_variant(path)
    knobs = [("" if k.strip() == "default" else k) for k in args.knobs.split(";") if k.strip()] or [""]
    bytes_per_pass = n * (8 * p + 8)
    res = {}
    for r in range(args.rounds):
        for name, lib in libs.items():
            for kn in knobs:
                for other in knobs:  # knobs of the other settings do not leak
                    for kv in [x for x in other.split(",") if x]:
                        os.environ.pop(kv.split("=")[0], None)
                for kv in [x for x in kn.split(",") if x]:
                    k, v = kv.split("=")
                    os.environ[k] = v
                opt = _hip.FitOptions()
                lib.dlsa_fit_options_default(ctypes.byref(opt))
                opt.hessian_mode = {"fp64": 1, "mixed_f32": 2}.get(args.hessian, 0)
                opt.record_timing = 1
                opt.rows_per_chunk = args.rows_per_chunk
                opt.warm_start = args.warm
                opt.workspace = ws.data_ptr()
                opt.workspace_bytes = ws.numel()
                rc = lib.dlsa_logistic_fit_batched_ex(
                    vp(X), vp(y), offs.ctypes.data_as(ctypes.c_void_p), K, p, 0, None, None,
                    args.max_iter, 1e-10, vp(theta), vp(sig), vp(sigt), vp(ll), vp(it), vp(st),
                    ctypes.byref(opt), stream)
                if rc != 0:
                    raise RuntimeError(lib.dlsa_last_error().decode())
                s = _hip.FitStats()
                lib.dlsa_last_fit_stats(ctypes.byref(s))
                d = res.setdefault((name, kn), {"f32": [], "f64": [], "solve": [], "it": []})
                if s.passes_fp32:
                    d["f32"].append(s.ms_pass_fp32 / s.passes_fp32)
                if s.passes_fp64:
                    d["f64"].append(s.ms_pass_fp64 / s.passes_fp64)
                d["solve"].append(s.ms_solve / max(1, s.iterations))
                d.setdefault("total", []).append(s.ms_total)
                d["it"].append((s.passes_fp32, s.passes_fp64))
                for kv in [x for x in kn.split(",") if x]:
                    os.environ.pop(kv.split("=")[0], None)
                # profiling builds (DLSA_OZ_PROF): exact-pass stamp sums per 32-row block
                prof = [0] * 32
                for fn in ("dlsa_oz_prof_read", "dlsa_oz_prof_read_g2"):
                    if hasattr(lib, fn):
                        buf = (ctypes.c_ulonglong * 32)()
                        getattr(lib, fn)(buf)
                        prof = [a + b for a, b in zip(prof, buf)]
                if any(prof):
                    # per-wave sums over all workgroups -> cycles per 64-row iteration
                    nit = max(1, n // 64 * max(1, s.passes_fp64))
                    d.setdefault("prof", []).append(
                        {**{f"producer{w}": {k: round(prof[4 * w + i] / nit, 1)
                                             for i, k in enumerate(["barrier", "row", "digits"])}
                            for w in range(4)},
                         **{f"consumer{w}": {k: round(prof[16 + 4 * w + i] / nit, 1)
                                             for i, k in enumerate(["barrier", "issue", "mfma",
                                                                    "vmwait"])}
                            for w in range(4)}})
    for (name, kn), d in res.items():
        out = {"lib": name, "knobs": kn, "n": n, "p": p, "K": K, "passes": d["it"][-1]}
        for key in ("f32", "f64"):
            if d[key]:
                m = statistics.median(d[key])
                out[f"{key}_ms"] = round(m, 3)
                out[f"{key}_GBps"] = round(bytes_per_pass / (m * 1e-3) / 1e9, 1)
        out["solve_ms_per_iter"] = round(statistics.median(d["solve"]), 3)
        out["fit_ms"] = round(statistics.median(d["total"]), 2)
        if d.get("prof"):
            out["cycles_per_block"] = d["prof"][-1]
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
