"""The product's sharded path end to end with world_size 2 on the GPU box:
two processes (ranks) on the one visible MI355X, each fitting its own
partitions in HBM (dlsa_fit_sharded: batched fit -> HBM pre-reduction ->
ONE all-reduce carrying the sums, K and N -> WLSE / ONESHOT / LARS / DBIC),
gloo as the transport (RCCL needs one GPU per rank; the driver's 8-GPU bench
runs the same code over nccl = RCCL).  Every rank must get the reference's
config-1 golden WLSE, ONESHOT and DBIC support."""

import os

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, golden_dir, shards, q, backend="gloo"):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world,
                                device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from dlsa_amd.distributed import dlsa_fit_sharded

        g = np.load(os.path.join(golden_dir, "config1_n1e5_p10_K4.npz"))
        np.random.seed(int(g["seed"]))
        pid, lab, feat = O.simulate_logistic_arrays(100000, 10, "systematic", 4)
        order, off = O.systematic_partition(pid)
        X, y = feat[order], lab[order]
        mine = shards[rank]
        Xl = np.concatenate([X[off[k]:off[k + 1]] for k in mine])
        yl = np.concatenate([y[off[k]:off[k + 1]] for k in mine])
        offl = np.concatenate([[0], np.cumsum([off[k + 1] - off[k] for k in mine])])
        calls = []
        orig = dist.all_reduce

        def spy(t, *a, **kw):  # the combine's collective: on which tensor, which backend
            calls.append((t.is_cuda, dist.get_backend()))
            return orig(t, *a, **kw)

        dist.all_reduce = spy
        try:
            res = dlsa_fit_sharded(torch.from_numpy(Xl).cuda(), torch.from_numpy(yl).cuda(), offl)
        finally:
            dist.all_reduce = orig
        if backend == "nccl":
            assert calls == [(True, "nccl")], calls
        else:  # gloo reduces a host copy of the device buffer
            assert calls == [(False, "gloo")], calls
        q.put((rank, res["wlse"], res["oneshot"], res["dbic_support"].tolist(),
               res["fit"].theta.cpu().numpy()))
    finally:
        dist.destroy_process_group()


def _run_ranks(golden_dir, shards, backend):
    import multiprocessing as mp
    import socket

    world = len(shards)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")  # children touch the GPU only after they start
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, golden_dir, shards, q, backend))
          for r in range(world)]
    for p_ in ps:
        p_.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p_ in ps:
        p_.join(timeout=60)
        assert p_.exitcode == 0
    return res


def _check_golden(golden_dir, shards, res):
    g = np.load(os.path.join(golden_dir, "config1_n1e5_p10_K4.npz"))
    gb = g["lars_lasso_beta"][int(np.argmin(g["lars_lasso_BIC"]))]
    for rank, wlse, oneshot, support, theta in res:
        assert np.abs(wlse - g["wlse_noint"]).max() / np.abs(g["wlse_noint"]).max() < 1e-8
        assert np.abs(oneshot - g["oneshot_noint"]).max() / np.abs(g["oneshot_noint"]).max() < 1e-8
        assert support == np.nonzero(gb)[0].tolist()
        ref = g["outs_noint"][shards[rank]][:, :, 1]
        assert np.abs(theta - ref).max() / np.abs(ref).max() < 1e-8


@pytest.mark.parametrize("shards", [([0, 2], [1, 3]), ([3], [0, 1, 2])])
def test_sharded_fit_two_ranks_one_gpu(golden_dir, shards):
    _check_golden(golden_dir, shards, _run_ranks(golden_dir, shards, "gloo"))


def test_sharded_fit_rccl_one_rank(golden_dir):
    """The RCCL branch of the combine on the box's one GPU: a child process
    (spawned before it touches the GPU) creates a "nccl" process group of one
    rank with device_id = cuda:0, and dlsa_fit_sharded's combine runs its
    all_reduce on the device buffer over RCCL (checked by a spy on
    torch.distributed.all_reduce); WLSE, ONESHOT and the DBIC support equal the
    reference's config-1 golden values (dlsa/dlsa.py:30-34, 70-100)."""
    shards = ([0, 1, 2, 3],)
    _check_golden(golden_dir, shards, _run_ranks(golden_dir, shards, "nccl"))


def test_bench_gpus2_launches_two_ranks(tmp_path):
    """`bench.py --gpus 2` started directly (no torchrun environment) must
    spawn 2 ranks itself and report n_gpus = 2 with the sampled partitions at
    parity; gloo lets both ranks share the one GPU of the test box (the
    driver's multi-GPU run uses nccl = RCCL, one GPU per rank)."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--backend", "gloo",
           "--n", "1600000", "--partitions", "16", "--steps", "2", "--warmup", "1",
           "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    assert out["scaling"] == "strong"
    assert out["config"]["n_rows_job"] == 1600000 and out["config"]["partitions_job"] == 16
    assert out["config"]["partitions_per_gpu"] == 8
    assert out["parity_rel"] < 1e-8


def test_bench_force_pg_rccl_one_gpu():
    """`bench.py --gpus 1 --backend nccl --force-pg`: the bench creates an RCCL
    process group of one rank, the combine all-reduces over it, and the line
    reports the backend with the sampled partitions at parity."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", "1", "--backend", "nccl",
           "--force-pg", "--n", "1600000", "--partitions", "16", "--steps", "2", "--warmup",
           "1", "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 1 and out["config"]["backend"] == "nccl"
    assert out["parity_rel"] < 1e-8
