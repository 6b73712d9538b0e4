"""HIP-graph replay of the fused Euler shooting and its adjoint (core/shooting.py,
_graph_forward / _graph_backward): for small supports the whole forward (nt fused passes and
the cost scan) and the whole adjoint are captured once and replayed.  The kernels and their
order are the direct path's, so everything must be BITWISE the direct path: the trajectory,
the loss, the gradient (first call direct, second captures, third replays), an L-BFGS
optimisation (LDDMMModel.Optimize) and a need_p1=False closure shooting completed after
the fact."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _loss_grad(LM, q0, p0, tgt, need_p1=True):
    p = p0.clone().requires_grad_(True)
    sh = LM.Shoot(q0, p, None, need_p1=need_p1)
    L = LM.trajloss(sh) + ((sh[-1][0] - tgt) ** 2).sum()
    L.backward()
    return [sh.Q.detach().clone(), sh.C.detach().clone(), L.detach().clone(), p.grad.clone()] + (
        [sh.P.detach().clone()] if need_p1 else [])


@pytest.mark.parametrize("version", ["classic", "hybrid", "logdet"])
@pytest.mark.parametrize("M,D", [(2000, 3), (700, 2)])
@pytest.mark.parametrize("need_p1", [True, False])
def test_graph_replay_bitwise(dev, version, M, D, need_p1):
    from difficp_amd.core import shooting
    from difficp_amd.core.LDDMM import LDDMMModel
    g = torch.Generator().manual_seed(M + D)
    # clouds 3 (2D) / 1.5 (3D) wide, momenta 0.01, lambda 100: all three models stay tame (the
    # float64 oracle: logdet loss 365 / 842, largest displacement 5-6 sigma).  Random momenta at
    # lambda 10 on a unit square blow the logdet flow up (loss ~1e16 in float64 too, NaN
    # gradients in float32 on every VJP variant -- tools/probes/logdet2d_nan.py)
    q0 = ((3.0 if D == 2 else 1.5) * torch.rand(M, D, generator=g)).to(dev)
    p0 = (0.01 * torch.randn(M, D, generator=g)).to(dev)
    tgt = (q0.cpu() + 0.05 * torch.randn(M, D, generator=g)).to(dev)
    LM = LDDMMModel(sigma=0.1, D=D, lambd=100.0, version=version, nt=10, scheme="Euler",
                    spec={"device": dev, "dtype": torch.float32})
    LM.shoot_cache = None          # every call computes (no trajectory reuse)
    old = shooting._GRAPH_ON
    try:
        shooting._GRAPH_ON = False
        ref = _loss_grad(LM, q0, p0, tgt, need_p1)
        assert all(bool(torch.isfinite(t).all()) for t in ref)
        shooting._GRAPH_ON = True
        n0 = dict(shooting.graph_stats)
        runs = [_loss_grad(LM, q0, p0, tgt, need_p1) for _ in range(3)]
        assert shooting.graph_stats["captures"] >= n0["captures"] + 2, "no graph was captured"
        assert shooting.graph_stats["replays"] >= n0["replays"] + 4
        runs.append(_loss_grad(LM, q0, 1.01 * p0, tgt, need_p1))     # new inputs, same graph
        shooting._GRAPH_ON = False
        other = _loss_grad(LM, q0, 1.01 * p0, tgt, need_p1)
    finally:
        shooting._GRAPH_ON = old
    for r in runs[:3]:
        for a, b in zip(r, ref):
            assert torch.equal(a, b)
    for a, b in zip(runs[3], other):
        assert torch.equal(a, b)


def test_graph_optimize_bitwise(dev):
    """A whole LDDMMModel.Optimize (L-BFGS, strong-Wolfe) with and without the graphs, and with
    the closures' loss and gradient through autograd or formed directly (shoot_loss_grad,
    LDDMM._DIRECT_LOSSGRAD): all four bitwise equal."""
    from difficp_amd.core import LDDMM as LDm
    from difficp_amd.core import shooting
    from difficp_amd.core.LDDMM import LDDMMModel
    g = torch.Generator().manual_seed(3)
    M = 1500
    q0 = torch.rand(M, 3, generator=g).to(dev)
    tgt = (q0.cpu() + 0.05 * torch.randn(M, 3, generator=g)).to(dev)
    res = []
    old = shooting._GRAPH_ON, LDm._DIRECT_LOSSGRAD
    try:
        for on in (False, True):
            for direct in (False, True):
                shooting._GRAPH_ON, LDm._DIRECT_LOSSGRAD = on, direct
                LM = LDDMMModel(sigma=0.1, D=3, lambd=10.0, version="hybrid", nt=10, scheme="Euler",
                                spec={"device": dev, "dtype": torch.float32})
                dataloss = LM.BasicQuadLossFunctor(tgt)
                p0, shoot, trajl, datal, nsteps, change = LM.Optimize(dataloss, q0, torch.zeros_like(q0), nmax=3)
                res.append((p0, shoot.Q, shoot.P, trajl, datal, nsteps))
    finally:
        shooting._GRAPH_ON, LDm._DIRECT_LOSSGRAD = old
    a = res[0]
    for b in res[1:]:
        assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]) and torch.equal(a[2], b[2])
        assert a[3:] == b[3:]
