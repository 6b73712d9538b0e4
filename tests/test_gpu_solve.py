"""GPU parity of the kernel ridge solve (v2p, LDDMM.py:235-253) -- dicp_kernel_ridge_cg_f32.

Oracle: the dense ridge solve KridgeSolve_torch (kernel.py:234-237) in float64 and the
restated KeOps CG (KridgeSolve_keops, kernel.py:239-241; pykeops itself is absent, so the
iteration count is "parity unpinned" -- the solution is pinned by the dense solve).
Tolerances: the fp32 CG stops at |r|^2 < M D eps^2; the solution error is then bounded by
cond(K + alpha I) x residual, so well-conditioned cases (alpha >= 0.1) are compared at 1e-4
relative and ill-conditioned ones through the residual of the float64 system.
"""
import pytest
import torch

from conftest import rel_err
from oracle import torch_ref as R

pytestmark = pytest.mark.gpu


def _lib():
    from difficp_amd import _lib
    return _lib


def _case(M, D, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(M, D, generator=g, dtype=torch.float64)
    v = torch.randn(M, D, generator=g, dtype=torch.float64)
    return x, v


@pytest.mark.parametrize("M,D,sigma,alpha", [(300, 3, 0.1, 1.0), (1000, 2, 0.05, 0.5),
                                             (2000, 3, 0.1, 0.1)])
def test_ridge_cg_vs_dense(dev, M, D, sigma, alpha):
    x, v = _case(M, D)
    b, info = _lib().kernel_ridge_cg(x.float().to(dev), v.float().to(dev), sigma, alpha)
    assert info["status"] == "converged", info
    ref = R.KridgeSolve_torch(x, v, sigma, alpha)
    assert rel_err(b, ref) < 1e-4, rel_err(b, ref)
    bo, ko = R.KridgeSolve_cg(x, v, sigma, alpha)
    assert rel_err(bo, ref) < 1e-5
    # same algorithm: iteration counts agree up to fp32 round-off in the last few steps
    assert abs(info["iterations"] - ko) <= max(3, ko // 5), (info["iterations"], ko)


def test_ridge_cg_ill_conditioned_residual(dev):
    """alpha = 1e-3 (the reference's commented PSR choice, PSR.py:402): the float64 residual
    of the float32 solution meets the KeOps stopping rule up to fp32 round-off."""
    M, D, sigma, alpha = 2000, 3, 0.1, 1e-3
    x, v = _case(M, D, seed=3)
    v = R.KRed(x, x, v, sigma) * 0.01            # speeds in the range of K (a realistic v2p rhs)
    b, info = _lib().kernel_ridge_cg(x.float().to(dev), v.float().to(dev), sigma, alpha,
                                     eps=1e-6, maxiter=5000)
    bb = b.double().cpu()
    res = R.KRed(x, x, bb, sigma) + alpha * bb - v
    assert float((res ** 2).sum()) < 100 * v.numel() * 1e-12, (float((res ** 2).sum()), info)


def test_ridge_cg_zero_rhs_and_determinism(dev):
    x, v = _case(500, 3, seed=1)
    xg = x.float().to(dev)
    b0, info0 = _lib().kernel_ridge_cg(xg, torch.zeros_like(xg), 0.1, 1e-2)
    assert info0["iterations"] == 0 and info0["status"] == "converged"
    assert torch.count_nonzero(b0) == 0
    vg = v.float().to(dev)
    b1, i1 = _lib().kernel_ridge_cg(xg, vg, 0.1, 1e-2, chunk=32)
    b2, i2 = _lib().kernel_ridge_cg(xg, vg, 0.1, 1e-2, chunk=7)   # chunking is invisible
    assert i1["iterations"] == i2["iterations"]
    assert torch.equal(b1, b2)


def test_ridge_cg_maxiter_reports(dev):
    x, v = _case(800, 3, seed=2)
    b, info = _lib().kernel_ridge_cg(x.float().to(dev), v.float().to(dev), 0.1, 1e-6,
                                     eps=1e-9, maxiter=10, chunk=4)
    assert info["status"] == "maxiter" and info["iterations"] == 10
    assert torch.isfinite(b).all()


def test_v2p_ridge_keops_gradcomponent(dev):
    """v2p(version='ridge_keops') for a gradcomponent model (initialize_a0, PSR.py:404-413:
    zero speeds -> K a0 = eta GradKRed(q,q)): v(q, q, a0) ~ 0 up to the ridge term."""
    from difficp_amd.core.LDDMM import LDDMMModel
    M, D = 1500, 3
    x, _ = _case(M, D, seed=4)
    spec = {"device": dev, "dtype": torch.float32}
    LM = LDDMMModel(sigma=0.1, D=D, lambd=1e2, version="logdet", spec=spec)
    q = x.float().to(dev)
    a0 = LM.v2p(q, torch.zeros_like(q), alpha=1e-3, version="ridge_keops")
    assert LM.Kernel.last_solve_info["status"] == "converged"
    rhs = (1.0 / 1e2) * R.GradKRed(x, x, 0.1)
    ref = R.KridgeSolve_torch(x, rhs, 0.1, 1e-3)
    assert rel_err(a0, ref) < 2e-3, rel_err(a0, ref)   # cond(K + 1e-3 I) ~ 1e5: fp32 limit
    # the speed left at q is the ridge term -alpha a0, as for the float64 dense solution
    vq = LM.v(q, q, a0).double().cpu()
    vref = R.KRed(x, x, ref, 0.1) - rhs
    assert float(vq.norm()) <= 1.5 * float(vref.norm()) + 1e-5, (float(vq.norm()), float(vref.norm()))


def test_ridge_cg_large(dev):
    """50k support points (C2 size): converges, residual checked on the device with KRed."""
    M, D, sigma, alpha = 50000, 3, 0.1, 1e-1
    g = torch.Generator().manual_seed(5)
    x = torch.rand(M, D, generator=g).to(dev)
    v = 0.01 * torch.randn(M, D, generator=g).to(dev)
    b, info = _lib().kernel_ridge_cg(x, v, sigma, alpha, eps=1e-6, maxiter=3000)
    assert info["status"] == "converged", info
    res = _lib().gauss_red(_lib().KRED, x, x, sigma, b=b) + alpha * b - v
    assert float((res.double() ** 2).sum()) < 10 * v.numel() * 1e-12
