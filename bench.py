#!/usr/bin/env python3
"""DLSA logistic fit benchmark (BASELINE.json metric, config 2 by default).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4|5]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One step = one complete DLSA fit of the GPU's shard: batched Newton/IRLS over
all partitions (approximate-Hessian passes + the final fp64 pass whose Hessian
is Sig_inv), local partition reduction in HBM, one RCCL all-reduce of the
P^2+2P+1 sums across ranks, WLSE solve, LARS path and DBIC selection on the
host.  Data are synthetic, generated in HBM by the counter-based generator
before the timed region.

Configs (BASELINE.json "configs"); per GPU (weak scaling):
  2  logistic n = 1e8, p = 100, K = 1024            (default; the headline metric)
  3  logistic n = 1.5e7, p = 181 + intercept, K = 128 (airline-like dummy-coded design;
                                                     1.2e8 rows on 8 GPUs)
  5  logistic n = 5e6, p = 500, K = 32              (wide path: row + Gram pass)
  4  OLS      n = 1.25e8, p = 64, K = 128           (1e9 rows / 1024 partitions on 8 GPUs)

Rank 0 prints one JSON line (metric/value/... plus "roofline" for the dominant
kernel and, at N = 1, "cpu_baseline": the numpy oracle on a bounded sample of
the same workload on host cores).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "DLSA logistic fit rows/sec (node), n=1e8 p=100, 1/2/4/8 GPUs; HBM GB/s"
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md chip table (spec)
FP64_MFMA_PEAK_TF = 78.6   # MI355X fp64 matrix (spec; = fp64 vector on CDNA4)

CONFIGS = {
    2: dict(n=100_000_000, p=100, K=1024, family="logistic",
            name="config2: synthetic logistic n=1e8 rows/GPU, p=100, K=1024 partitions/GPU"),
    3: dict(n=15_000_000, p=181, K=128, family="logistic", data="dummy", intercept=True,
            name="config3: airline-like logistic n=1.5e7 rows/GPU (1.2e8 on 8 GPUs), 9 numeric + "
                 "172 dummy columns + intercept, K=128 partitions/GPU"),
    5: dict(n=5_000_000, p=500, K=32, family="logistic",
            name="config5: synthetic logistic n=5e6 rows/GPU, p=500, K=32 partitions/GPU (wide path)"),
    4: dict(n=125_000_000, p=64, K=128, family="ols",
            name="config4: synthetic OLS n=1.25e8 rows/GPU (1e9 on 8 GPUs), p=64, K=128 partitions/GPU"),
}


def _cpu_worker(args):
    """One partition of the CPU baseline: regenerate its rows from the counter
    stream, fit with the numpy oracle (1 BLAS thread)."""
    n, p, seed, row0, family, data = args
    import numpy as np
    from threadpoolctl import threadpool_limits

    import oracle as O

    with threadpool_limits(1):
        if data == "dummy":
            import torch

            from dlsa_amd.models import simulate_dummy_design
            torch.set_num_threads(1)
            Xt, yt = simulate_dummy_design(n, seed=seed + row0, device="cpu")
            X, y = Xt.numpy(), yt.numpy()
            X = np.hstack([np.ones((n, 1)), X])  # intercept column
        else:
            X, y = O.simulate_counter(n, p, seed=seed, row0=row0)
        t0 = time.perf_counter()
        if family == "ols":
            O.ols_fit(X, y)
            it = 1
        else:
            it = int(O.logistic_fit(X, y)["iters"])
        return time.perf_counter() - t0, it


def cpu_baseline(nk, p, n_parts, workers, family, seed=2019, data="counter"):
    """Oracle (port) timed on host cores: n_parts partitions of nk rows, one
    process per core, fit time only (data regeneration excluded)."""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    jobs = [(nk, p, seed, k * nk, family, data) for k in range(n_parts)]
    t0 = time.perf_counter()
    with ctx.Pool(workers) as pool:
        res = pool.map(_cpu_worker, jobs, chunksize=1)
    wall = time.perf_counter() - t0
    fit_s = sum(r[0] for r in res)
    rows_per_s = n_parts * nk / (fit_s / workers)  # all `workers` cores fitting concurrently
    return {"value": rows_per_s, "unit": "rows/s", "cores": workers, "kind": "port",
            "sample": f"{n_parts} partitions x {nk} rows x p={p}{' (dummy design + intercept)' if data == 'dummy' else ''}, numpy fp64 "
                      f"{'OLS' if family == 'ols' else 'IRLS'} oracle, 1 BLAS thread per process, "
                      f"{workers} processes; fit CPU time {fit_s:.1f} s, wall {wall:.1f} s incl. "
                      f"data regeneration",
            "iters_mean": sum(r[1] for r in res) / len(res)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS))
    ap.add_argument("--n", type=int, default=0, help="rows per GPU (0: the config's)")
    ap.add_argument("--p", type=int, default=0)
    ap.add_argument("--partitions", type=int, default=0, help="partitions per GPU")
    ap.add_argument("--hessian", default="mixed", choices=["mixed", "fp64", "mixed_f32"])
    ap.add_argument("--tol", type=float, default=1e-10)
    ap.add_argument("--cpu-parts", type=int, default=32)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--seed", type=int, default=2019)
    ap.add_argument("--layout", default="codes", choices=["codes", "dense"],
                    help="config 3: categorical-code layout (LDS-histogram pass) or the dense "
                         "dummy-coded design")
    args = ap.parse_args()
    cfg = dict(CONFIGS[args.config])
    for key, v in (("n", args.n), ("p", args.p), ("K", args.partitions)):
        if v:
            cfg[key] = v

    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from dlsa_amd import _hip
    from dlsa_amd.dlsa import reduce_partitions_device, split_reduced, wlse
    from dlsa_amd.lsa import lars_lsa
    from dlsa_amd.models import (logistic_model_batched, logistic_model_batched_categorical,
                                 ols_model_batched, simulate_categorical, simulate_dummy_design,
                                 simulate_logistic_device)

    n, p, K, family = cfg["n"], cfg["p"], cfg["K"], cfg["family"]
    data = cfg.get("data", "counter")
    fit_intercept = bool(cfg.get("intercept", False))
    P = p + int(fit_intercept)
    wide = P > _hip.MAX_P_FUSED
    offsets = (np.arange(K + 1, dtype=np.int64) * n) // K
    codes_layout = data == "dummy" and args.layout == "codes"
    if codes_layout:
        X, codes, y, levels = simulate_categorical(n, seed=args.seed + rank, device=dev)
        assert X.shape[1] + int((levels - 1).sum()) == p
    elif data == "dummy":
        X, y = simulate_dummy_design(n, seed=args.seed + rank, device=dev)
        assert X.shape[1] == p
    else:
        X, y = simulate_logistic_device(n, p, seed=args.seed, row0=rank * n, device=dev)
    if family == "ols":  # linear response on the same design
        y = X[:, : max(1, int(0.4 * p))].sum(1) + 0.5 * (y - 0.5)
    ws = torch.empty((1,), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()

    n_global = n * world
    stats_acc = []

    def step(record):
        nonlocal ws
        if family == "ols":
            fit = ols_model_batched(X, y, offsets, record_timing=record, device=dev)
        elif codes_layout:
            fit = logistic_model_batched_categorical(X, codes, y, offsets, levels,
                                                     fit_intercept=fit_intercept, tol=args.tol,
                                                     record_timing=record, device=dev)
        else:
            fit = logistic_model_batched(X, y, offsets, fit_intercept=fit_intercept,
                                         hessian=args.hessian, tol=args.tol,
                                         record_timing=record, workspace=ws, device=dev)
            if ws.numel() < fit.stats["workspace_bytes"]:
                ws = torch.empty((fit.stats["workspace_bytes"],), dtype=torch.uint8, device=dev)
        buf = reduce_partitions_device(fit)
        if world > 1:
            dist.all_reduce(buf, op=dist.ReduceOp.SUM)  # RCCL over xGMI
        S, v, st, Ksum = split_reduced(buf.cpu().numpy(), fit.P)
        est = wlse(S, v)
        lars = lars_lsa(S, est, fit_intercept, n_global, type="lasso")
        ib = int(np.argmin(lars["BIC"]))
        support = np.nonzero(lars["beta"][ib])[0]
        return fit, est, support

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        fit, est, support = step(True)
        stats_acc.append(fit.stats)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    ms_per_step = elapsed / args.steps * 1e3
    value = n_global * args.steps / elapsed

    # ---- per-kernel throughput and the roofline of the dominant kernel -----
    # (HIP events recorded on the fit's stream around every launch)
    tot = lambda key: sum(s[key] for s in stats_acc)  # noqa: E731
    row_bytes = 8 * p + 8                        # X row + y, read once per pass
    if codes_layout:                             # numeric columns + uint8 codes + y
        row_bytes = 8 * X.shape[1] + codes.shape[1] + 8
    alg_flops_row = P * (P + 1) + 4 * P + 20     # symmetric X^T W X + X.b, X^T r
    kern = {}
    if codes_layout:
        ms64, n64, rows64 = tot("ms_pass_fp64"), tot("passes_fp64"), tot("rows_fp64")
        kern["cat_pass_kernel"] = {
            "launches_per_step": n64 / args.steps, "ms_per_step": ms64 / args.steps,
            "avg_launch_ms": ms64 / n64, "rows_per_launch": rows64 / n64,
            "GBps": rows64 * row_bytes / (ms64 * 1e-3) / 1e9,
            "Grows_per_s": rows64 / (ms64 * 1e-3) / 1e9}
        kern["newton_solve"] = {"ms_per_step": tot("ms_solve") / args.steps}
        achieved = rows64 * row_bytes / (ms64 * 1e-3) / 1e9
        roof = {"kernel": "cat_pass_kernel (categorical codes, one-hot blocks as fp64 LDS "
                          "histograms)", "bound": "hbm", "achieved": achieved,
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                "traffic": None, "algorithmic_bytes_per_launch": rows64 * row_bytes / n64,
                "avg_launch_ms": ms64 / n64,
                "note": "bytes/row = 8 q + F + 8 (codes layout); the kernel issues ~47 fp64 "
                        "LDS atomics per row, which bound it before HBM"}
    elif wide:
        NB = (P + 127) // 128
        gram_flops_row = NB * (NB + 1) // 2 * 128 * 128 * 2  # issued MFMA work per row
        n32, n64 = tot("passes_fp32"), tot("passes_fp64")
        rows32, rows64 = tot("rows_fp32"), tot("rows_fp64")
        ms32, ms64, ms_row = tot("ms_pass_fp32"), tot("ms_pass_fp64"), tot("ms_wide_row")
        kern["wide_row_kernel"] = {"ms_per_step": ms_row / args.steps,
                                   "GBps": (rows32 + rows64) * row_bytes / (ms_row * 1e-3) / 1e9}
        if n32:
            kern["wide_gram_bf16_kernel"] = {
                "launches_per_step": n32 / args.steps, "avg_launch_ms": ms32 / n32,
                "alg_TFps": rows32 * p * (p + 1) / (ms32 * 1e-3) / 1e12,
                "mfma_TFps": rows32 * gram_flops_row / (ms32 * 1e-3) / 1e12}
        if n64:
            kern["wide_gram_kernel<fp64>"] = {
                "launches_per_step": n64 / args.steps, "avg_launch_ms": ms64 / n64,
                "alg_TFps": rows64 * p * (p + 1) / (ms64 * 1e-3) / 1e12,
                "mfma_TFps": rows64 * gram_flops_row / (ms64 * 1e-3) / 1e12}
        kern["wide_assemble_kernel"] = {"ms_per_step": tot("ms_wide_assemble") / args.steps}
        kern["wide_newton_kernel"] = {"ms_per_step": tot("ms_solve") / args.steps}
        if ms64 >= ms32:
            achieved = rows64 * p * (p + 1) / (ms64 * 1e-3) / 1e12
            roof = {"kernel": "wide_gram_kernel<fp64> (X^T W X, 128x128 tiles)", "bound": "mfma",
                    "achieved": achieved, "peak": FP64_MFMA_PEAK_TF, "unit": "TFLOP/s",
                    "frac": achieved / FP64_MFMA_PEAK_TF, "traffic": None,
                    "algorithmic_flops_per_launch": rows64 * p * (p + 1) / n64,
                    "avg_launch_ms": ms64 / n64,
                    "mfma_issued_TFps": rows64 * gram_flops_row / (ms64 * 1e-3) / 1e12}
        else:
            achieved = rows32 * row_bytes / (ms32 * 1e-3) / 1e9
            roof = {"kernel": "wide_gram_bf16_kernel (approximate X^T W X)", "bound": "hbm",
                    "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                    "algorithmic_bytes_per_launch": rows32 * row_bytes / n32,
                    "avg_launch_ms": ms32 / n32}
    else:
        NT = (P + 15) // 16
        mfma_flops_per_row = NT * (NT + 1) // 2 * 16 * 16 * 2  # lower-triangle 16x16 tiles
        ms32, ms64 = tot("ms_pass_fp32"), tot("ms_pass_fp64")
        n32, n64 = tot("passes_fp32"), tot("passes_fp64")
        rows32, rows64 = tot("rows_fp32"), tot("rows_fp64")
        if n32:
            kern["irls_coop<bf16 Hessian>"] = {
                "launches_per_step": n32 / args.steps, "ms_per_step": ms32 / args.steps,
                "avg_launch_ms": ms32 / n32, "rows_per_launch": rows32 / n32,
                "GBps": rows32 * row_bytes / (ms32 * 1e-3) / 1e9,
                "mfma_TFps": rows32 * mfma_flops_per_row / (ms32 * 1e-3) / 1e12}
        if n64:
            kern["irls_coop<fp64 Hessian>"] = {
                "launches_per_step": n64 / args.steps, "ms_per_step": ms64 / args.steps,
                "avg_launch_ms": ms64 / n64, "rows_per_launch": rows64 / n64,
                "GBps": rows64 * row_bytes / (ms64 * 1e-3) / 1e9,
                "mfma_TFps": rows64 * mfma_flops_per_row / (ms64 * 1e-3) / 1e12}
        kern["newton_solve"] = {"ms_per_step": tot("ms_solve") / args.steps}
        if ms32 >= ms64:
            achieved = rows32 * row_bytes / (ms32 * 1e-3) / 1e9
            roof = {"kernel": f"irls_coop_kernel<NT={NT},bf16 Hessian> (approximate-Hessian passes)",
                    "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                    "algorithmic_bytes_per_launch": rows32 * row_bytes / n32,
                    "avg_launch_ms": ms32 / n32}
        else:
            achieved = rows64 * mfma_flops_per_row / (ms64 * 1e-3) / 1e12
            kname = (f"irls_wave_kernel<NT={NT},fp64> (per-wave exact pass)" if NT <= 8
                     else f"irls_coop_kernel<NT={NT},fp64 Hessian>")
            roof = {"kernel": kname, "bound": "mfma",
                    "achieved": achieved, "peak": FP64_MFMA_PEAK_TF, "unit": "TFLOP/s",
                    "frac": achieved / FP64_MFMA_PEAK_TF, "traffic": None,
                    "mfma_flops_per_launch": rows64 * mfma_flops_per_row / n64,
                    "avg_launch_ms": ms64 / n64,
                    "GBps": rows64 * row_bytes / (ms64 * 1e-3) / 1e9}
    pmc_file = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc_file):
        try:
            pmc = json.load(open(pmc_file)).get(f"config{args.config}", {})
            if pmc.get("p") == p and pmc.get("n") == n and pmc.get("kernel") == roof["kernel"]:
                roof["traffic"] = pmc["hbm_bytes_per_launch"]
                roof["traffic_source"] = pmc.get("source")
        except Exception:
            pass

    last = stats_acc[-1]
    out = {
        "metric": METRIC, "value": value, "unit": "rows/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": ("synthetic airline-like: 9 U(-1/2,1/2) numeric + dummies of 5 skewed factors "
                 "(12/7/20/69/69 levels, baseline dropped), y~Bernoulli(sigmoid(-0.3+X beta*)); "
                 "torch generator in HBM (not timed); layout: " +
                 ("uint8 level codes + numeric columns" if codes_layout else
                  "dense dummy design")) if data == "dummy" else
                "synthetic: X~U(-1/2,1/2), beta*=1 on first floor(0.4p) cols, y~Bernoulli"
                "(sigmoid(X beta*)); counter-based generator in HBM (not timed)",
        "config": {"workload": cfg["name"] + " + DLSA combine + LARS/DBIC",
                   "n_rows_per_gpu": n, "p": p, "P": P, "fit_intercept": fit_intercept,
                   "partitions_per_gpu": K,
                   **({"layout": args.layout} if data == "dummy" else {}),
                   "family": family, "hessian": args.hessian if family == "logistic" and not codes_layout else "fp64",
                   "tol": args.tol,
                   "parallelism": f"dp{world} (partitions sharded; 1 RCCL all-reduce of P^2+2P+1 fp64)"},
        "roofline": roof,
        "kernels": kern,
        "newton": {"iterations": last["iterations"], "passes_fp32": last["passes_fp32"],
                   "passes_fp64": last["passes_fp64"], "n_chunks": last["n_chunks"],
                   "status": fit.status_counts()},
        "dbic_support_size": int(len(support)),
        "algorithmic": {"bytes_per_pass": n * row_bytes, "flops_per_pass": n * alg_flops_row},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        workers = min(16, os.cpu_count() or 1)
        if args.config == 5:
            nk_cpu, parts = 20000, 16      # ~8 s of single-thread work per partition
        else:
            nk_cpu, parts = n // K, args.cpu_parts
        out["cpu_baseline"] = cpu_baseline(nk_cpu, p, parts, workers, family, data=data)
        out["vs_cpu_baseline"] = value / out["cpu_baseline"]["value"]
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
