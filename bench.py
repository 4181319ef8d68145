#!/usr/bin/env python3
"""DLSA logistic fit benchmark (BASELINE.json metric, config 2 by default).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4|5]
                    [--scaling strong|weak] [--backend nccl|gloo]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

``--gpus N`` with N > 1 and no torchrun environment starts the N ranks itself:
the launcher process (which never touches the GPU) starts N child processes
of this script with the torch.distributed environment variables and exits
with their status.  Every rank checks that the process group holds exactly N
ranks.

One step = one complete DLSA fit of the GPU's shard: batched Newton/IRLS over
all partitions (approximate-Hessian passes + the final fp64 pass whose Hessian
is Sig_inv), local partition reduction in HBM, ONE RCCL all-reduce of the
P^2+2P+2 sums (Sig_inv, Sig_inv theta, theta, K, N) across ranks, WLSE solve,
LARS path and DBIC selection on the host.  Data are synthetic, generated in
HBM by the counter-based generator before the timed region.

Configs (BASELINE.json "configs").  Under --scaling strong (the
default) n and K are those of the whole job and rank r owns partitions
[rK/N, (r+1)K/N) of the same global data set (config 2 is then
north_star's "n=1e8, p=100, 1024 partitions on 8 GPUs"); under --scaling weak
they are per GPU.  Config 4's job (1e9 rows x 64 = 520 GB) does not fit one
GPU, so it defaults to weak scaling with the 8-GPU job's per-GPU share:
  2  logistic n = 1e8, p = 100, K = 1024            (default; the headline metric)
  3  logistic n = 1.2e8, p = 181 + intercept, K = 120 (airline-like dummy-coded design at
                                                     the reference's 1e6 rows per partition)
  5  logistic n = 5e6, p = 500, K = 32              (wide path: row + Gram pass)
  4  OLS      n = 1.25e8, p = 64, K = 128 per GPU   (1e9 rows / 1024 partitions on 8 GPUs)

Rank 0 prints one JSON line (metric/value/... plus "roofline" for the dominant
kernel, "parity_rel" of two sampled partitions against the CPU oracle after
the timed region, and, at N = 1, "cpu_baseline": the numpy oracle on a
bounded sample of the same workload on host cores, timed by wall clock).
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
I8_MFMA_PEAK_TOPS = 5000.0  # int8 dense: 2x the ~2.5 PF bf16 dense rate (MI355X_MICROARCH.md
#                             "Matrix cores": i8 16x16x64 = the bf16 cycles at 2x the K)

CONFIGS = {
    2: dict(n=100_000_000, p=100, K=1024, family="logistic",
            name="config2: synthetic logistic n=1e8, p=100, K=1024 partitions"),
    3: dict(n=120_000_000, p=181, K=120, family="logistic", data="dummy", intercept=True,
            name="config3: airline-like logistic n=1.2e8, 9 numeric + 172 dummy columns + "
                 "intercept, K=120 partitions (1e6 rows each, logistic_dlsa.py:239-240)"),
    5: dict(n=5_000_000, p=500, K=32, family="logistic",
            name="config5: synthetic logistic n=5e6, p=500, K=32 partitions (wide path)"),
    4: dict(n=125_000_000, p=64, K=128, family="ols", scaling="weak",
            name="config4: synthetic OLS n=1.25e8 (1e9 on 8 GPUs), p=64, K=128 partitions"),
}


# ---------------------------------------------------------------------------
# CPU baseline: the numpy oracle (port) on host cores, wall clock
# ---------------------------------------------------------------------------


def _cpu_worker(jobs, family, data, barrier, t_done, idx):
    """Generate this worker's partitions (not timed), wait for every worker,
    then fit them with the numpy oracle (1 BLAS thread) and record the
    wall-clock finish time."""
    import numpy as np
    from threadpoolctl import threadpool_limits

    import oracle as O

    with threadpool_limits(1):
        parts = []
        for (n, p, seed, row0) in jobs:
            if data == "dummy":
                import torch

                from dlsa_amd.models import simulate_dummy_design
                torch.set_num_threads(1)
                Xt, yt = simulate_dummy_design(n, seed=seed + row0, device="cpu")
                X, y = Xt.numpy(), yt.numpy()
                X = np.hstack([np.ones((n, 1)), X])  # intercept column
            else:
                X, y = O.simulate_counter(n, p, seed=seed, row0=row0)
                if family == "ols":
                    y = X[:, : max(1, int(0.4 * p))].sum(1) + 0.5 * (y - 0.5)
            parts.append((X, y))
        barrier.wait()
        for X, y in parts:
            if family == "ols":
                O.ols_fit(X, y)
            else:
                O.logistic_fit(X, y)
        t_done[idx] = time.time()


def host_cores():
    """CPUs this process may use: the affinity mask, capped by a cgroup CPU
    quota (cpu.max / cfs_quota_us) when one is set.  Returns (cores, info)."""
    import math

    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = nproc
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    cores = aff if quota is None else max(1, min(aff, int(math.ceil(quota))))
    return cores, {"nproc": nproc, "affinity": aff, "cgroup_cpu_quota": quota}


def cpu_baseline(nk, p, n_parts, workers, family, seed=2019, data="counter"):
    """Oracle (port) timed on host cores: n_parts partitions of nk rows dealt
    to `workers` processes (1 BLAS thread each).  Every worker generates its
    data first (untimed); the clock runs from the barrier that releases all
    workers to the last worker's finish: rows / wall time."""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    barrier = ctx.Barrier(workers + 1)
    t_done = ctx.Array("d", workers)
    jobs = [[] for _ in range(workers)]
    for k in range(n_parts):
        jobs[k % workers].append((nk, p, seed, k * nk))
    procs = [ctx.Process(target=_cpu_worker, args=(jobs[w], family, data, barrier, t_done, w))
             for w in range(workers)]
    for pr in procs:
        pr.start()
    barrier.wait()
    t0 = time.time()
    for pr in procs:
        pr.join()
    wall = max(t_done[:]) - t0
    return {"value": n_parts * nk / wall, "unit": "rows/s", "cores": workers, "kind": "port",
            "sample": f"{n_parts} partitions x {nk} rows x p={p}"
                      f"{' (dummy design + intercept)' if data == 'dummy' else ''}, numpy fp64 "
                      f"{'OLS' if family == 'ols' else 'IRLS (tol 1e-12)'} oracle, 1 BLAS thread "
                      f"per process, {workers} processes; wall clock {wall:.1f} s from the start "
                      f"barrier to the last finish (data generation excluded)"}


# ---------------------------------------------------------------------------
# parity of sampled partitions (the oracle as the checker, after timing)
# ---------------------------------------------------------------------------


def sampled_parity(fit, X, y, offsets, family, codes=None, levels=None, fit_intercept=False,
                   sample=None):
    """max relative error (theta, Sig_inv) of the sampled partitions against
    the CPU oracle; relative to the largest entry, as the GPU tests."""
    import numpy as np

    import oracle as O

    K = len(offsets) - 1
    sample = sample if sample is not None else sorted({0, K - 1})
    worst = 0.0
    for k in sample:
        a, b = int(offsets[k]), int(offsets[k + 1])
        Xk = X[a:b].cpu().numpy()
        yk = y[a:b].cpu().numpy()
        if codes is not None:
            Xk = O.expand_codes(Xk, codes[a:b].cpu().numpy(), levels)
        if family == "ols":
            o = O.ols_fit(Xk, yk, fit_intercept=fit_intercept)
        else:
            o = O.logistic_fit(Xk, yk, fit_intercept=fit_intercept)
        for got, ref in ((fit.theta[k], o["coef"]), (fit.sig_inv[k], o["Sig_inv"])):
            g = got.cpu().numpy()
            worst = max(worst, float(np.abs(g - ref).max() / np.abs(ref).max()))
    return worst, sample


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS))
    ap.add_argument("--scaling", default=None, choices=["weak", "strong"],
                    help="strong (default; config 4: weak): n and K of the whole job, "
                         "partitions sharded over the ranks; weak: the config's n and K per GPU")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="process-group transport for N > 1 (nccl = RCCL over xGMI; gloo: "
                         "host transport, lets several ranks share one GPU in tests)")
    ap.add_argument("--force-pg", action="store_true",
                    help="create the process group (--backend) even at --gpus 1, so the "
                         "combine runs its all-reduce (RCCL at one rank)")
    ap.add_argument("--n", type=int, default=0, help="rows (per GPU, or total when strong)")
    ap.add_argument("--p", type=int, default=0)
    ap.add_argument("--partitions", type=int, default=0)
    ap.add_argument("--hessian", default="mixed", choices=["mixed", "fp64", "mixed_f32"])
    ap.add_argument("--tol", type=float, default=1e-10)
    ap.add_argument("--cpu-parts", type=int, default=0,
                    help="partitions of the CPU baseline sample (0: ~10-30 s of CPU work per config)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-fp64-step", action="store_true",
                    help="skip the two untimed fp64-Sig_inv steps reported beside the line")
    ap.add_argument("--seed", type=int, default=2019)
    ap.add_argument("--layout", default="codes", choices=["codes", "dense"],
                    help="config 3: categorical-code layout (LDS-histogram pass) or the dense "
                         "dummy-coded design")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    cfg = dict(CONFIGS[args.config])
    if args.scaling is None:
        args.scaling = cfg.get("scaling", "strong")
    for key, v in (("n", args.n), ("p", args.p), ("K", args.partitions)):
        if v:
            cfg[key] = v

    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE = {world}")
    ndev = torch.cuda.device_count()
    if ndev < 1:
        raise SystemExit("bench.py: no GPU visible")
    if args.backend == "nccl" and world > ndev:
        raise SystemExit(f"bench.py: {world} RCCL ranks need {world} GPUs ({ndev} visible); "
                         "--backend gloo lets ranks share a GPU")
    torch.cuda.set_device(local % ndev)
    dev = torch.device("cuda", local % ndev)
    use_pg = world > 1 or args.force_pg
    if use_pg:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if "MASTER_PORT" not in os.environ:
            import socket
            with socket.socket() as s_:
                s_.bind(("127.0.0.1", 0))
                os.environ["MASTER_PORT"] = str(s_.getsockname()[1])
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", str(world))
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"bench.py: process group has {dist.get_world_size()} ranks, "
                             f"--gpus {args.gpus}")

    from dlsa_amd import _hip
    from dlsa_amd.distributed import combine
    from dlsa_amd.dlsa import reduce_partitions_device, split_reduced, wlse
    from dlsa_amd.lsa import lars_lsa
    from dlsa_amd.models import (logistic_model_batched, logistic_model_batched_categorical,
                                 ols_model_batched, simulate_categorical, simulate_dummy_design,
                                 simulate_logistic_device)

    p, family = cfg["p"], cfg["family"]
    data = cfg.get("data", "counter")
    fit_intercept = bool(cfg.get("intercept", False))
    P = p + int(fit_intercept)
    wide = P > _hip.MAX_P_FUSED
    if args.scaling == "strong":
        n_job, K_job = cfg["n"], cfg["K"]
        if K_job < world:
            raise SystemExit("strong scaling needs at least one partition per rank")
        goff = (np.arange(K_job + 1, dtype=np.int64) * n_job) // K_job
        k0, k1 = rank * K_job // world, (rank + 1) * K_job // world
        row0, n = int(goff[k0]), int(goff[k1] - goff[k0])
        offsets = goff[k0:k1 + 1] - goff[k0]
        K = k1 - k0
    else:
        n, K = cfg["n"], cfg["K"]
        n_job, K_job = n * world, K * world
        row0 = rank * n
        offsets = (np.arange(K + 1, dtype=np.int64) * n) // K
    codes_layout = data == "dummy" and args.layout == "codes"
    codes = levels = None
    if codes_layout:
        X, codes, y, levels = simulate_categorical(n, seed=args.seed + rank, device=dev)
        assert X.shape[1] + int((levels - 1).sum()) == p
    elif data == "dummy":
        X, y = simulate_dummy_design(n, seed=args.seed + rank, device=dev)
        assert X.shape[1] == p
    else:
        X, y = simulate_logistic_device(n, p, seed=args.seed, row0=row0, device=dev)
    if family == "ols":  # linear response on the same design
        y = X[:, : max(1, int(0.4 * p))].sum(1) + 0.5 * (y - 0.5)
    ws = torch.empty((1,), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()

    stats_acc = []
    stage_ms = {"fit": 0.0, "reduce_allreduce": 0.0, "wlse_lars_dbic": 0.0}

    def step(record, hessian=None, exact="auto"):
        nonlocal ws
        t_a = time.perf_counter()
        if family == "ols":
            fit = ols_model_batched(X, y, offsets, record_timing=record, device=dev)
        elif codes_layout:
            fit = logistic_model_batched_categorical(X, codes, y, offsets, levels,
                                                     fit_intercept=fit_intercept, tol=args.tol,
                                                     record_timing=record, device=dev)
        else:
            fit = logistic_model_batched(X, y, offsets, fit_intercept=fit_intercept,
                                         hessian=hessian or args.hessian, tol=args.tol,
                                         record_timing=record, workspace=ws, device=dev,
                                         exact=exact)
            if ws.numel() < fit.stats["workspace_bytes"]:
                ws = torch.empty((fit.stats["workspace_bytes"],), dtype=torch.uint8, device=dev)
        t_b = time.perf_counter()  # the fit returns after its stream synchronisation
        buf = reduce_partitions_device(fit, n_rows=True)
        combine(buf)  # the one collective: RCCL all-reduce over xGMI (none at N = 1
        #                without --force-pg)
        b = buf.cpu().numpy()
        t_c = time.perf_counter()
        S, v, st, Ksum = split_reduced(b[:-1], fit.P)
        est = wlse(S, v)
        lars = lars_lsa(S, est, fit_intercept, int(round(b[-1])), type="lasso")
        ib = int(np.argmin(lars["BIC"]))
        support = np.nonzero(lars["beta"][ib])[0]
        if record:  # per-rank wall-clock budget of a step
            t_d = time.perf_counter()
            stage_ms["fit"] += (t_b - t_a) * 1e3
            stage_ms["reduce_allreduce"] += (t_c - t_b) * 1e3
            stage_ms["wlse_lars_dbic"] += (t_d - t_c) * 1e3
        return fit, est, support, int(round(Ksum)), int(round(b[-1]))

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    if use_pg:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        # release the previous step's outputs before the next fit allocates
        # its own, so the caching allocator reuses their blocks: a fresh
        # device allocation held the next launches back by ~5 ms
        # (profiles/r05y_c5_host_gaps.txt)
        fit = None
        fit, est, support, K_red, n_red = step(True)
        stats_acc.append(fit.stats)
    torch.cuda.synchronize()
    if use_pg:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if use_pg:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device=dev if args.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    assert K_red == K_job and n_red == n_job, (K_red, n_red, K_job, n_job)
    ms_per_step = elapsed / args.steps * 1e3
    value = n_job * args.steps / elapsed

    # the same step with an fp64-MFMA Sig_inv, beside the headline line (one
    # step each, after the timed region; N = 1 without a process group only,
    # since a rank-0-only step would wait in the all-reduce)
    fp64_steps = {}
    if family == "logistic" and not codes_layout and not use_pg and not args.no_fp64_step:
        for key, hs, ex in (("sig_inv_fp64_ms_per_step", "fp64", "fp64"),
                            ("exact_fp64_ms_per_step", None, "fp64")):
            torch.cuda.synchronize()
            t_f = time.perf_counter()
            step(False, hessian=hs, exact=ex)
            torch.cuda.synchronize()
            fp64_steps[key] = (time.perf_counter() - t_f) * 1e3

    # ---- per-kernel throughput and the roofline of the dominant kernel -----
    # (HIP events recorded on the fit's stream around every launch)
    tot = lambda key: sum(s[key] for s in stats_acc)  # noqa: E731
    row_bytes = 8 * p + 8                        # X row + y, read once per pass
    if codes_layout:                             # numeric columns + uint8 codes + y
        row_bytes = 8 * X.shape[1] + codes.shape[1] + 8
    alg_flops_row = P * (P + 1) + 4 * P + 20     # symmetric X^T W X + X.b, X^T r
    kern = {}

    def hbm_roof(kname, ms, launches, rows):
        achieved = rows * row_bytes / (ms * 1e-3) / 1e9
        return {"kernel": kname, "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                "algorithmic_bytes_per_launch": rows * row_bytes / launches,
                "rows_per_launch": rows / launches, "avg_launch_ms": ms / launches}

    if codes_layout:
        ms64, n64, rows64 = tot("ms_pass_fp64"), tot("passes_fp64"), tot("rows_fp64")
        kern["cat_pass_kernel"] = {
            "launches_per_step": n64 / args.steps, "ms_per_step": ms64 / args.steps,
            "avg_launch_ms": ms64 / n64, "rows_per_launch": rows64 / n64,
            "GBps": rows64 * row_bytes / (ms64 * 1e-3) / 1e9,
            "Grows_per_s": rows64 / (ms64 * 1e-3) / 1e9}
        kern["newton_solve"] = {"ms_per_step": tot("ms_solve") / args.steps}
        roof = hbm_roof("cat_pass_kernel (categorical codes, one-hot blocks as fp64 LDS "
                        "histograms)", ms64, n64, rows64)
        roof["note"] = "bytes/row = 8 q + F + 8 (codes layout)"
        pmc_key = "cat_pass_kernel"
    elif wide:
        NB = (P + 127) // 128
        gram_flops_row = NB * (NB + 1) // 2 * 128 * 128 * 2  # issued MFMA work per row
        n32, n64 = tot("passes_fp32"), tot("passes_fp64")
        rows32, rows64 = tot("rows_fp32"), tot("rows_fp64")
        ms32, ms64, ms_row = tot("ms_pass_fp32"), tot("ms_pass_fp64"), tot("ms_wide_row")
        if n64:  # the exact passes' row pass (eta, w, gradient; the fused pass does its own)
            kern["wide_row_kernel"] = {"ms_per_step": ms_row / args.steps,
                                       "GBps": rows64 * row_bytes / (ms_row * 1e-3) / 1e9}
        if n32:
            kern["wide_fused_bf16_kernel"] = {
                "launches_per_step": n32 / args.steps, "avg_launch_ms": ms32 / n32,
                "GBps": rows32 * row_bytes / (ms32 * 1e-3) / 1e9,
                "alg_TFps": rows32 * p * (p + 1) / (ms32 * 1e-3) / 1e12,
                "mfma_TFps": rows32 * gram_flops_row / (ms32 * 1e-3) / 1e12}
        n_oz = tot("passes_oz")
        gram_name = ("wide_oz_gram (int8 digit slices: scale + digits + 128x128 tiles)" if n_oz
                     else "wide_gram_kernel<fp64>")
        if n64:
            kern[gram_name] = {
                "launches_per_step": n64 / args.steps, "avg_launch_ms": ms64 / n64,
                "alg_TFps": rows64 * p * (p + 1) / (ms64 * 1e-3) / 1e12,
                "mfma_TFps": rows64 * gram_flops_row / (ms64 * 1e-3) / 1e12}
            if n_oz:
                # 72 v_mfma_i32_16x16x64_i8 per wave (8 waves) per 32 rows per 128x128
                # tile: 9 per 16x16 sub-tile, diagonal tiles' upper quadrants idle
                tiles = NB * (NB + 1) // 2
                i8_ops_row = tiles * 8 * 72 * 16 * 16 * 64 * 2 / 32
                tops = rows64 * i8_ops_row / (ms64 * 1e-3) / 1e12
                del kern[gram_name]["mfma_TFps"]
                kern[gram_name].update({
                    "int8_mfma_TOPS_issued_upper_bound": tops,
                    "int8_mfma_frac_upper_bound": tops / I8_MFMA_PEAK_TOPS,
                    "note": "DESIGN.md 4.4b: scale + digits + 128x128 int8 tiles; alg_TFps "
                            "counts the fp64-equivalent Gram work; the int8 rate counts every "
                            "tile's MFMAs as issued (the idle diagonal quadrants included)"})
        kern["wide_assemble_kernel"] = {"ms_per_step": tot("ms_wide_assemble") / args.steps}
        kern["wide_newton_kernel"] = {"ms_per_step": tot("ms_solve") / args.steps}
        if ms64 >= ms32 and not n_oz:
            achieved = rows64 * p * (p + 1) / (ms64 * 1e-3) / 1e12
            roof = {"kernel": "wide_gram_kernel<fp64> (X^T W X, 128x128 tiles)", "bound": "mfma",
                    "achieved": achieved, "peak": FP64_MFMA_PEAK_TF, "unit": "TFLOP/s",
                    "frac": achieved / FP64_MFMA_PEAK_TF, "traffic": None,
                    "algorithmic_flops_per_launch": rows64 * p * (p + 1) / n64,
                    "rows_per_launch": rows64 / n64, "avg_launch_ms": ms64 / n64,
                    "mfma_issued_TFps": rows64 * gram_flops_row / (ms64 * 1e-3) / 1e12}
            pmc_key = "wide_gram_kernel<fp64>"
        else:
            roof = hbm_roof("wide_fused_bf16_kernel (one X stream per iteration: gradient + "
                            "approximate X^T W X)", ms32, n32, rows32)
            pmc_key = "wide_fused_bf16"
    else:
        NT = (P + 15) // 16
        mfma_flops_per_row = NT * (NT + 1) // 2 * 16 * 16 * 2  # lower-triangle 16x16 tiles
        ms32, ms64 = tot("ms_pass_fp32"), tot("ms_pass_fp64")
        n32, n64 = tot("passes_fp32"), tot("passes_fp64")
        rows32, rows64 = tot("rows_fp32"), tot("rows_fp64")
        n_oz = tot("passes_oz")
        ols_stream = family == "ols" and NT <= 4  # capi.hip: ols_stream_applies
        exact = (f"irls_oz_kernel<NT={NT}> (exact pass, int8-MFMA digit slices)" if n_oz
                 else f"ols_stream_kernel<NT={NT}> (X streamed into the fp64 MFMA operands)"
                 if ols_stream
                 else f"irls_wave_kernel<NT={NT},fp64> (per-wave exact pass)" if NT <= 8
                 else f"irls_coop_kernel<NT={NT},fp64 Hessian>")
        if n32:
            kern["irls_coop<bf16 Hessian>"] = {
                "launches_per_step": n32 / args.steps, "ms_per_step": ms32 / args.steps,
                "avg_launch_ms": ms32 / n32, "rows_per_launch": rows32 / n32,
                "GBps": rows32 * row_bytes / (ms32 * 1e-3) / 1e9,
                "mfma_TFps": rows32 * mfma_flops_per_row / (ms32 * 1e-3) / 1e12}
        if n64:
            gbps = rows64 * row_bytes / (ms64 * 1e-3) / 1e9
            kern[exact] = {
                "launches_per_step": n64 / args.steps, "ms_per_step": ms64 / args.steps,
                "avg_launch_ms": ms64 / n64, "rows_per_launch": rows64 / n64,
                "GBps": gbps, "hbm_frac": gbps / HBM_PEAK_GBS,
                "alg_TFps": rows64 * alg_flops_row / (ms64 * 1e-3) / 1e12}
            if n_oz:
                # the Hessian runs on the int8 matrix cores: 9 v_mfma_i32_16x16x64_i8 per
                # lower-triangle 16x16 tile per 32 rows, 32768 ops each
                i8_ops_row = NT * (NT + 1) // 2 * 9 * 16 * 16 * 64 * 2 / 32
                tops = rows64 * i8_ops_row / (ms64 * 1e-3) / 1e12
                kern[exact].update({"int8_mfma_TOPS": tops,
                                    "int8_mfma_frac": tops / I8_MFMA_PEAK_TOPS,
                                    "note": "X^T W X as int8 digit-slice products (5 levels of "
                                            "a 38-bit grid, DESIGN.md 4.1c); bound: HBM"})
            else:
                tf = rows64 * mfma_flops_per_row / (ms64 * 1e-3) / 1e12
                kern[exact].update({"mfma_TFps": tf, "mfma_frac": tf / FP64_MFMA_PEAK_TF})
        kern["newton_solve"] = {"ms_per_step": tot("ms_solve") / args.steps}
        if ms32 >= ms64:
            roof = hbm_roof(f"irls_coop_kernel<NT={NT},bf16 Hessian> (approximate-Hessian "
                            "passes)", ms32, n32, rows32)
            pmc_key = "irls_coop<bf16>"
        elif family == "ols":
            # config 4 is HBM-bound (65 GB vs 0.54 TF per GPU)
            roof = hbm_roof(exact + " (OLS: X^T X, X^T y in one pass)", ms64, n64, rows64)
            roof["mfma_issued_frac"] = kern[exact].get("mfma_frac")
            pmc_key = "ols_stream" if ols_stream else "irls_wave<ols>"
        elif n_oz:  # the int8 exact pass streams X once: HBM-bound
            roof = hbm_roof(exact, ms64, n64, rows64)
            roof["int8_mfma_frac"] = kern[exact]["int8_mfma_frac"]
            pmc_key = "irls_oz"
        else:
            achieved = rows64 * mfma_flops_per_row / (ms64 * 1e-3) / 1e12
            roof = {"kernel": exact, "bound": "mfma", "achieved": achieved,
                    "peak": FP64_MFMA_PEAK_TF, "unit": "TFLOP/s",
                    "frac": achieved / FP64_MFMA_PEAK_TF, "traffic": None,
                    "mfma_flops_per_launch": rows64 * mfma_flops_per_row / n64,
                    "rows_per_launch": rows64 / n64, "avg_launch_ms": ms64 / n64}
            pmc_key = "irls_wave<fp64>"
    # HBM traffic from the PMC passes (tools/pmc.sh + tools/pmc_summary.py):
    # bytes per row of a full-pass launch of this kernel at this p, scaled to
    # this run's rows per launch, so traffic and the algorithmic bytes
    # describe the same launch
    pmc_file = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc_file):
        try:  # the int8 exact pass's own record (config 2), beside its kernel entry
            ex = json.load(open(pmc_file)).get(f"config{args.config}_exact", {})
            if not wide and not codes_layout and n_oz and ex.get("p") == p:
                kern[exact]["traffic_bytes_per_row"] = ex["hbm_bytes_per_row"]
                kern[exact]["traffic_source"] = ex.get("source")
        except Exception:
            pass
        try:
            rec = json.load(open(pmc_file)).get(f"config{args.config}", {})
            if rec.get("p") == p and rec.get("kernel_key") == pmc_key and \
                    rec.get("calibrated", True) is False:
                roof["traffic_note"] = rec.get("note")
            elif rec.get("p") == p and rec.get("kernel_key") == pmc_key:
                roof["traffic"] = rec["hbm_bytes_per_row"] * roof["rows_per_launch"]
                roof["traffic_bytes_per_row"] = rec["hbm_bytes_per_row"]
                roof["algorithmic_bytes_per_row"] = row_bytes
                roof["traffic_source"] = rec.get("source")
        except Exception:
            pass

    last = stats_acc[-1]
    # the arithmetic of the published Sig_inv (dtype "f64" is the data and the
    # gradient; the exact Hessian may be int8-Ozaki emulated)
    if last.get("passes_oz", 0):
        sig_inv_arith = "int8-ozaki-5L (38-bit digit grid, 5 levels; ~1e-12 relative)"
    elif codes_layout:
        sig_inv_arith = "fp64 + int64 fixed-point LDS histograms"
    else:
        sig_inv_arith = "fp64-mfma"
    out = {
        "metric": METRIC, "value": value, "unit": "rows/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step,
        "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None, "dtype": "f64",
        "data": ("synthetic airline-like: 9 U(-1/2,1/2) numeric + dummies of 5 skewed factors "
                 "(12/7/20/69/69 levels, baseline dropped), y~Bernoulli(sigmoid(-0.3+X beta*)); "
                 "torch generator in HBM (not timed); layout: " +
                 ("uint8 level codes + numeric columns" if codes_layout else
                  "dense dummy design")) if data == "dummy" else
                "synthetic: X~U(-1/2,1/2), beta*=1 on first floor(0.4p) cols, y~Bernoulli"
                "(sigmoid(X beta*)); counter-based generator in HBM (not timed)",
        "config": {"workload": cfg["name"] + (" per GPU" if args.scaling == "weak" else
                                              " in total") + " + DLSA combine + LARS/DBIC",
                   "n_rows_job": n_job, "n_rows_per_gpu": n, "p": p, "P": P,
                   "fit_intercept": fit_intercept, "partitions_job": K_job,
                   "partitions_per_gpu": K,
                   **({"layout": args.layout} if data == "dummy" else {}),
                   "family": family,
                   "hessian": args.hessian if family == "logistic" and not codes_layout else "fp64",
                   "sig_inv": sig_inv_arith,
                   "tol": args.tol,
                   "parallelism": f"dp{world} (partitions sharded; 1 "
                                  f"{'RCCL' if args.backend == 'nccl' else 'gloo'} all-reduce of "
                                  "P^2+2P+2 fp64)",
                   "backend": args.backend if use_pg else None},
        "roofline": roof,
        "kernels": kern,
        "stages_ms_per_step": dict({k: v / args.steps for k, v in stage_ms.items()},
                                   fit_native=tot("ms_total") / args.steps),
        "newton": {"iterations": last["iterations"], "passes_fp32": last["passes_fp32"],
                   "passes_fp64": last["passes_fp64"], "passes_oz": last.get("passes_oz", 0),
                   "n_chunks": last["n_chunks"],
                   "status": fit.status_counts()},
        "dbic_support_size": int(len(support)),
        **fp64_steps,
        **({"fp64_steps_note": (
            "one untimed step each after the timed region: sig_inv_fp64 = --hessian fp64 (every "
            "pass on the fp64 MFMA); exact_fp64 = the mixed schedule with the exact pass on the "
            "fp64 MFMA (DLSA_EXACT_FP64) instead of the int8 digit slices")} if fp64_steps else {}),
        "algorithmic": {"bytes_per_pass": n * row_bytes, "flops_per_pass": n * alg_flops_row},
    }
    if rank == 0 and not args.no_parity:
        # checker, after the timed region: the last step's fit of this rank
        sample = [0] if (wide or data == "dummy") else None  # 1e6-row / P = 500 oracles
        rel, smp = sampled_parity(fit, X, y, offsets, family, codes=codes, levels=levels,
                                  fit_intercept=fit_intercept, sample=sample)
        out["parity_rel"] = rel
        out["parity_sample"] = (f"partitions {smp} of rank 0 vs the numpy oracle (tol 1e-12): "
                                "max |diff| / max |ref| over theta and Sig_inv")
    if rank == 0 and not args.no_parity:
        # every partition of rank 0 (not a sample): Sig_inv per entry against an
        # independent fp64 library-GEMM evaluation of models.py:114,130 at the
        # returned theta_k, and the WLSE of those independent sums
        # (oracle/device_check.py; after the timed region)
        from oracle.device_check import check_all_partitions
        torch.cuda.synchronize()
        t_ck = time.perf_counter()
        design = None
        if codes_layout:
            from dlsa_amd.models import expand_categorical
            design = lambda a, b: expand_categorical(X[a:b], codes[a:b], levels)  # noqa: E731
        r = check_all_partitions(fit, X, y, family=family, design=design)
        out["sig_inv_all_partitions"] = {
            k: r[k] for k in ("partitions", "max_elem_err", "worst_partition",
                              "sig_inv_theta_rel", "wlse_rel")}
        out["sig_inv_all_partitions"]["note"] = (
            "every partition of rank 0: max_ij |Sig_inv_ij - H_ij| / sqrt(H_ii H_jj) with "
            "H = X_k^T diag(w) X_k at the returned theta_k by torch fp64 GEMMs (an independent "
            "library path); wlse_rel = WLSE of the independent sums vs the product's sums; "
            f"{time.perf_counter() - t_ck:.1f} s, after the timed region")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        workers, cinfo = host_cores()      # every core this process may use
        if args.config == 5:
            nk_cpu, parts = 20000, 16      # ~8 s of single-thread work per partition
        else:                              # ~10-30 s of single-thread work in all
            nk_cpu, parts = min(n // K, 125_000), {2: 32, 3: 32, 4: 128}[args.config]
        parts = args.cpu_parts or max(parts, 2 * workers)  # >= 2 partitions per core
        out["cpu_baseline"] = cpu_baseline(nk_cpu, p, parts, workers, family, data=data)
        out["cpu_baseline"].update(cinfo)
        out["vs_cpu_baseline"] = value / out["cpu_baseline"]["value"]
    if rank == 0:
        print(json.dumps(out), flush=True)
    if use_pg:
        dist.destroy_process_group()


def launch_ranks(n):
    """N ranks on this node without an external launcher: N child processes of
    this script with the torch.distributed environment (RANK, LOCAL_RANK,
    WORLD_SIZE, MASTER_ADDR = 127.0.0.1, a free MASTER_PORT) and the same
    arguments.  This process never initialises the GPU (children, no exec).
    If a rank fails the others are stopped (they would wait in a collective).
    Returns the first non-zero exit code, else 0."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:],
                                      env=env))
    rc = 0
    while procs:
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in procs:
                    q.terminate()
        time.sleep(0.05)
    return rc


if __name__ == "__main__":
    main()
