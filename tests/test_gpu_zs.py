"""Divergence-row reuse (dicp_lddmm_*_zs_f32, include/difficp_hip.h): the forward's per-row
sums zs_i = sum_j K (q_i - q_j) feed the VJP's divergence-cotangent term, whose pair loop
then drops it (SymBwdPk<., ., ., false>).  Parity: zs against the fp64 oracle (-sigma^2
GradKRed), the adjoint steps and pair-subset parts against the fp64 autograd VJP of the
oracle's ODE (tolerance 2e-5 norm-wise relative, as tests/test_gpu_kernels.py) and against the
plain entries (1e-5: fp32 summation order only); q_next / p_next / g of the zs forward are
bitwise those of the plain forward (same pair loop and column splits).
"""
import pytest
import torch

from conftest import rel_err
from oracle import torch_ref as R

pytestmark = pytest.mark.gpu

SIG = 0.15


def _lib():
    from difficp_amd import _lib
    return _lib


def _case(M, D, seed):
    g = torch.Generator().manual_seed(seed)
    q = torch.rand(M, D, generator=g, dtype=torch.float64)
    p = 0.1 * torch.randn(M, D, generator=g, dtype=torch.float64)
    a = torch.randn(M, D, generator=g, dtype=torch.float64)
    bm = torch.randn(M, D, generator=g, dtype=torch.float64)
    gam = torch.randn(1, generator=g, dtype=torch.float64)
    return q, p, a, bm, gam


def _vjp64(q, p, a, bm, gam, D):
    q = q.clone().requires_grad_(True)
    p = p.clone().requires_grad_(True)
    m = R.LDDMM(SIG, D, 50.0, False, True)   # hybrid: eta = 0 with the divergence term
    v, mG, c = m.ODE(q, p, torch.zeros(1, dtype=torch.float64))
    Lf = (a * v).sum() + (gam * c).sum() + ((bm * mG).sum() if bm is not None else 0)
    return torch.autograd.grad(Lf, (q, p))


@pytest.mark.parametrize("M,D", [(1, 3), (129, 2), (700, 3), (5000, 3), (20000, 3)])
@pytest.mark.parametrize("want_p", [True, False])
def test_euler_step_zs_rows(dev, M, D, want_p):
    L = _lib()
    q, p, *_ = _case(M, D, M + D)
    f = lambda t: t.float().to(dev)
    zs = torch.empty(M, D, device=dev)
    qn, pn, g = L.euler_step(f(q), f(p), SIG, 0.0, 0.1, True, want_p=want_p, zs_out=zs)
    qn0, pn0, g0 = L.euler_step(f(q), f(p), SIG, 0.0, 0.1, True, want_p=want_p)
    assert torch.equal(qn, qn0) and torch.equal(g, g0)
    if want_p:
        assert torch.equal(pn, pn0)
    zs64 = -SIG ** 2 * R.GradKRed(q, q, SIG)
    zs32 = -SIG ** 2 * R.GradKRed(q.float(), q.float(), SIG)
    tol = max(1e-5, 4 * rel_err(zs32.double(), zs64))
    assert rel_err(zs.cpu(), zs64) <= tol, rel_err(zs.cpu(), zs64)
    # a row slice (row split): the slice's rows of the full pass's zs
    r0, n = M // 3, M - M // 3
    zl = torch.empty(n, D, device=dev)
    L.euler_step_rows(f(q), f(p), r0, n, SIG, 0.0, 0.1, True, want_p=want_p, zs_out=zl)
    assert rel_err(zl, zs[r0:]) < 1e-6


@pytest.mark.parametrize("M,D", [(1, 3), (129, 2), (700, 3), (5000, 3), (50000, 3)])
@pytest.mark.parametrize("want_lq", [True, False])
@pytest.mark.parametrize("zero_b", [False, True])
def test_adjoint_step_zs(dev, M, D, want_lq, zero_b):
    L = _lib()
    q, p, a, bm, gam = _case(M, D, 3 * M + D)
    if zero_b:
        bm = None
    f = lambda t: None if t is None else t.float().to(dev)
    zs = torch.empty(M, D, device=dev)
    L.euler_step(f(q), f(p), SIG, 0.0, 0.1, True, zs_out=zs)
    dt = 0.1
    lqn, lpn = L.euler_adjoint_step(f(q), f(p), f(a), f(bm), f(gam), SIG, 0.0, dt, None, None,
                                    want_lq=want_lq, zs=zs)
    lqn0, lpn0 = L.euler_adjoint_step(f(q), f(p), f(a), f(bm), f(gam), SIG, 0.0, dt, None, None,
                                      want_lq=want_lq)
    assert rel_err(lpn, lpn0) < 1e-5, rel_err(lpn, lpn0)
    if M <= 5000:   # the fp64 autograd oracle (O(M^2) memory)
        gq64, gp64 = _vjp64(q, p, a, bm, gam, D)
        lp0 = bm if bm is not None else torch.zeros_like(q)
        assert rel_err(lpn.cpu(), lp0 + dt * gp64) < 2e-5
        if want_lq:
            assert rel_err(lqn.cpu(), a + dt * gq64) < 2e-5
    if want_lq:
        assert rel_err(lqn, lqn0) < 1e-5
        # the gq half does not see the divergence rows: bitwise the plain step's
        assert torch.equal(lqn, lqn0) or rel_err(lqn, lqn0) < 1e-6
    else:
        assert lqn is None
    # deterministic
    _, lpn2 = L.euler_adjoint_step(f(q), f(p), f(a), f(bm), f(gam), SIG, 0.0, dt, None, None,
                                   want_lq=want_lq, zs=zs)
    assert torch.equal(lpn, lpn2)


@pytest.mark.parametrize("M", [130, 5000, 50000])
@pytest.mark.parametrize("W", [2, 3, 8])
@pytest.mark.parametrize("zero_b", [False, True])
def test_bwd_parts_zs(dev, M, W, zero_b):
    """Parts with each rank's own zs slice (rows [r * ceil(M/W), ...)) sum to the full VJP."""
    L = _lib()
    q, p, a, bm, gam = _case(M, 3, M + W)
    if zero_b:
        bm = None
    f = lambda t: None if t is None else t.float().to(dev)
    zs = torch.empty(M, 3, device=dev)
    L.euler_step(f(q), f(p), SIG, 0.0, 0.1, True, zs_out=zs)
    per = -(-M // W)
    sq, sp = torch.zeros(M, 3, device=dev), torch.zeros(M, 3, device=dev)
    for r in range(W):
        r0 = min(r * per, M)
        n = min(per, M - r0)
        pq, pp = L.ode_self_bwd_part(f(q), f(p), f(a), f(bm), f(gam), SIG, 0.0, r, W,
                                     zs=zs[r0:r0 + n], zrow0=r0)
        sq += pq
        sp += pp
    gq, gp = L.ode_self_bwd(f(q), f(p), f(a), f(bm) if bm is not None else torch.zeros_like(f(a)),
                            f(gam), SIG, 0.0)
    assert rel_err(sp, gp) < 1e-5, rel_err(sp, gp)
    assert rel_err(sq, gq) < 2e-6, rel_err(sq, gq)


def test_zs_rejected_where_unsupported(dev):
    """eta != 0 has no divergence-row form: the C-ABI refuses it loudly."""
    L = _lib()
    q = torch.rand(300, 3, device=dev)
    p = 0.1 * torch.randn(300, 3, device=dev)
    zs = torch.empty(300, 3, device=dev)
    with pytest.raises(RuntimeError):
        L.euler_step(q, p, SIG, 0.02, 0.1, True, zs_out=zs)
    with pytest.raises(RuntimeError):
        L.euler_adjoint_step(q, p, p, p, torch.ones(1, device=dev), SIG, 0.02, 0.1, zs=zs)


@pytest.mark.parametrize("M,D", [(1, 3), (300, 2), (20000, 3)])
def test_first_step_zs(dev, M, D):
    """dicp_lddmm_ode_self_fwd_zs_f32: v, mG, g bitwise those of the plain pass, zs those of the
    Euler form, and p.v / 2 the plain pass's h rows (to fp32 rounding)."""
    L = _lib()
    q, p, *_ = _case(M, D, 5 * M + D)
    f = lambda t: t.float().to(dev)
    zs = torch.empty(M, D, device=dev)
    v, mG, g, none = L.ode_self_fwd(f(q), f(p), SIG, 0.0, True, zs_out=zs)
    assert none is None
    v0, mG0, g0, h0 = L.ode_self_fwd(f(q), f(p), SIG, 0.0, True, want_h=True)
    assert torch.equal(v, v0) and torch.equal(mG, mG0) and torch.equal(g, g0)
    zs2 = torch.empty(M, D, device=dev)
    L.euler_step(f(q), f(p), SIG, 0.0, 0.1, True, zs_out=zs2)
    assert torch.equal(zs, zs2)
    assert rel_err(0.5 * (f(p) * v).sum(1), h0) < 1e-6
