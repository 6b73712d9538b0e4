"""Multi-rank (gloo, CPU) tests of the frame-sharded atlas path: each rank owns the frames
k = rank mod W, Reg_opt is rank-local, GMM_opt exchanges the per-component sufficient
statistics.  Kernels are replaced by the oracle-backed executable spec (tests/fake_hip.py),
so this checks the sharding / exchange logic; results must equal the single-process run on
all frames.  Cases: world 2 / 4 frames, and world 3 / 2 frames with outliers and a
reinitialize_GMM (rank 2 owns no frame and must still join every collective)."""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _frames(K=4):
    g = torch.Generator().manual_seed(5)
    out = []
    for k in range(K):
        base = torch.rand(50, 2, generator=g)
        out.append(base + 0.03 * torch.sin(6.28 * base[:, [1, 0]]) * (1 + 0.5 * k))
    return out


def _run(world, rank, comm, K=4, outliers=False):
    sys.path.insert(0, HERE)
    sys.path.insert(0, ROOT)
    import fake_hip
    fake_hip.install_plain()
    from difficp_amd.core.GMM import GaussianMixtureUnif
    from difficp_amd.core.LDDMM import LDDMMModel
    from difficp_amd.core.PSR import DiffPSR
    spec = {"device": "cpu", "dtype": torch.float32}
    frames = _frames(K)
    g = torch.Generator().manual_seed(9)
    mu0 = torch.rand(6, 2, generator=g)
    GM = GaussianMixtureUnif(mu0, sigma=0.1, use_outliers=outliers, spec=spec)
    LM = LDDMMModel(sigma=0.25, D=2, lambd=100.0, version="hybrid", scheme="Euler", nt=5, spec=spec)
    P = DiffPSR(frames, GM, LM, dataspec=spec, compspec=spec, comm=comm)
    P.printstuff = False
    if outliers:
        torch.manual_seed(11)          # reinitialize_GMM draws on rank 0 and broadcasts
        P.reinitialize_GMM()
    res = {"FE0": P.FE}
    P.GMM_opt(max_iterations=5, tol=1e-6)
    res["FE_gmm"] = P.FE
    res["mu"] = P.GMMi[0].mu.clone()
    res["w"] = P.GMMi[0].w.clone()
    res["sigma"] = P.GMMi[0].sigma
    P.Reg_opt(tol=1e-3, nmax=1)
    res["FE_reg"] = P.FE
    res["x1"] = {k: P.x1[k, 0].clone() for k in P.frames}
    res["frames"] = list(P.frames)
    return res


def _worker(rank, world, port, q, K, outliers):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    import torch.distributed as dist
    torch.set_num_threads(1)  # no OpenMP oversubscription across the worker processes
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = _run(world, rank, True, K, outliers)
        q.put((rank, {k: (v if not isinstance(v, torch.Tensor) else v.numpy()) for k, v in res.items()
                      if k != "x1"}, {k: v.numpy() for k, v in res["x1"].items()}))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,K,outliers", [(2, 4, False), (3, 2, True), (8, 8, True)])
def test_sharded_atlas_matches_single_process(world, K, outliers):
    import numpy as np
    single = _run(1, 0, None, K, outliers)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, K, outliers)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out.sort(key=lambda t: t[0])
    for rank, res, x1 in out:
        assert res["frames"] == [k for k in range(K) if k % world == rank]
        for key in ("FE0", "FE_gmm", "FE_reg"):
            assert abs(res[key] - single[key]) < 1e-4 * abs(single[key]), (rank, key, res[key], single[key])
        assert abs(res["sigma"] - single["sigma"]) < 1e-5 * single["sigma"]
        assert np.abs(res["mu"] - single["mu"].numpy()).max() < 1e-5
        assert np.abs(res["w"] - single["w"].numpy()).max() < 1e-4
        for k, v in x1.items():
            assert np.abs(v - single["x1"][k].numpy()).max() < 1e-4, (rank, k)
    # all ranks hold bit-identical GMM parameters
    for r in range(1, world):
        assert np.array_equal(out[0][1]["mu"], out[r][1]["mu"])
        assert out[0][1]["sigma"] == out[r][1]["sigma"]


def _count_worker(rank, world, port, q, outliers):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    import torch.distributed as dist
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sys.path.insert(0, HERE)
        sys.path.insert(0, ROOT)
        import fake_hip
        fake_hip.install_plain()
        from difficp_amd.core.GMM import GaussianMixtureUnif
        calls = []
        names = ("all_gather", "all_gather_into_tensor", "all_reduce", "broadcast", "reduce_scatter",
                 "all_to_all", "gather", "scatter", "barrier")
        orig = {n: getattr(dist, n) for n in names}

        def wrap(n):
            def f(*a, **k):
                calls.append(n)
                return orig[n](*a, **k)
            return f
        spec = {"device": "cpu", "dtype": torch.float32}
        g = torch.Generator().manual_seed(3 + rank)
        X = torch.rand(40 + 7 * rank, 2, generator=g)
        mu0 = torch.rand(5, 2, generator=torch.Generator().manual_seed(1))
        G = GaussianMixtureUnif(mu0, sigma=0.1, use_outliers=outliers, spec=spec)
        G.to_optimize = {"mu": True, "sigma": True, "w": True, "eta0": True}
        G.comm = True
        if outliers:
            G.set_vol0(X)           # (one-off, outside the counted EM steps)
        for n in names:
            setattr(dist, n, wrap(n))
        per_step = []
        try:
            for _ in range(3):
                del calls[:]
                G.EM_step(X)
                per_step.append(list(calls))
        finally:
            for n in names:
                setattr(dist, n, orig[n])
        q.put((rank, per_step, G.mu.numpy().copy(), G.sigma))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("outliers", [False, True])
def test_em_step_one_stats_exchange(outliers):
    """SURVEY 8(e) / VERDICT r03: an EM step of the sharded GMM exchanges its statistics in
    ONE packed collective (column statistics, sigma numerator, outlier LSE terms, point
    count) plus ONE scalar exchange for the free energy -- at most 2 collectives."""
    import numpy as np
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_count_worker, args=(r, world, port, q, outliers)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=300) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, per_step, mu, sigma in out:
        for calls in per_step:
            assert len(calls) <= 2, (rank, calls)
    assert np.array_equal(out[0][2], out[1][2]) and out[0][3] == out[1][3]
