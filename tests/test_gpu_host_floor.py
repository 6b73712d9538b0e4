"""The host-floor shortcuts of the L-BFGS closure (round 6) are bitwise the paths they replace:

* PSR's quadratic data loss forms its own gradient (`QuadLossFunctor(k).value_and_grad`,
  core/PSR.py): shoot_loss_grad then builds the adjoint's cotangents without autograd's engine
  -- loss and grad_p0 must be the bits of the autograd path (the same functor without the
  attribute), for graph-replayed (2k) and direct (20k) shootings, hybrid and classic;
* the multi-tensor copies of the graph replays (core/shooting.py _copy_many) -- covered by
  test_gpu_shoot_graph.py's bitwise replay tests -- and a whole Optimize on the 2k two-set
  workload gives the same a0 / loss with and without the data loss's own gradient."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _plain(f):
    """The same data loss without value_and_grad (the autograd path)."""
    return lambda x: f(x)


@pytest.mark.parametrize("N,version", [(2000, "hybrid"), (2000, "classic"), (20000, "hybrid")])
def test_quadloss_direct_grad_bitwise(dev, N, version):
    from difficp_amd import workloads
    from difficp_amd.core.shooting import shoot_loss_grad
    psr = workloads.build_two_set(N, dev, seed=1, version=version)
    psr.GMM_opt(max_iterations=3)
    f = psr.QuadLossFunctor(0)
    assert hasattr(f, "value_and_grad")
    LM = psr.LMi
    q0 = psr.q0[0].detach()
    g = torch.Generator().manual_seed(N)
    for p0 in (psr.a0[0].detach().clone(),
               (1e-3 * torch.randn(q0.shape, generator=g)).to(dev)):
        for _ in range(2):          # capture, then replay (2k: graph path)
            La, ga, _ = shoot_loss_grad(LM, f, q0, p0)
            Lb, gb, _ = shoot_loss_grad(LM, _plain(f), q0, p0)
            assert torch.isfinite(ga).all()
            assert torch.equal(La.reshape(-1), Lb.reshape(-1)), (La, Lb)
            assert torch.equal(ga, gb), (ga - gb).abs().max()


def test_quadloss_grad_matches_autograd_of_functor(dev):
    """value_and_grad's gradient is the autograd gradient of the functor itself."""
    from difficp_amd import workloads
    psr = workloads.build_two_set(3000, dev, seed=2)
    psr.GMM_opt(max_iterations=2)
    f = psr.QuadLossFunctor(0)
    x = (psr.q0[0] + 0.01).detach().requires_grad_(True)
    L = f(x)
    L.backward()
    v, gx = f.value_and_grad(x.detach())
    assert torch.equal(v, L.detach())
    assert torch.equal(gx, x.grad)


def test_optimize_same_with_direct_dataloss(dev):
    from difficp_amd import workloads
    psr = workloads.build_two_set(2000, dev, seed=3)
    psr.GMM_opt(max_iterations=5)
    f = psr.QuadLossFunctor(0)
    LM = psr.LMi
    outs = []
    for loss in (f, _plain(f)):
        p0, shoot, trajl, datal, nsteps, change = LM.Optimize(loss, psr.q0[0], psr.a0[0].clone(), nmax=2)
        outs.append((p0.clone(), trajl, datal, nsteps))
    assert torch.equal(outs[0][0], outs[1][0])
    assert outs[0][1:] == outs[1][1:]
