"""GPU parity of every HIP kernel against the CPU oracle (oracle/torch_ref.py, float64).

Tolerance: norm-wise relative error <= max(1e-5, 4 x the oracle's own fp32-vs-fp64 error)
(SURVEY.md 8c parity criterion), per output.
"""
import math

import pytest
import torch

from conftest import rel_err
from oracle import torch_ref as R

BWD_ALG_DEFAULT = 3  # lddmm.hip g_bwd_alg: symmetric pair-once VJP, packed-FP32 rows
FWD_ALG_DEFAULT = 2  # lddmm.hip g_fwd_alg: eta = 0 packed-FP32 rows
BWD_ETA_ALG_DEFAULT = 2  # lddmm.hip g_bwd_eta_alg (DICP_BWD_ETA_ALG)

pytestmark = pytest.mark.gpu


def _lib():
    from difficp_amd import _lib
    return _lib


def _data(M, N, D, seed=0, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(M, D, generator=g, dtype=torch.float64) * scale
    y = torch.rand(N, D, generator=g, dtype=torch.float64) * scale
    b = torch.randn(N, D, generator=g, dtype=torch.float64)
    c = torch.randn(M, D, generator=g, dtype=torch.float64)
    d = torch.randn(N, generator=g, dtype=torch.float64)
    return x, y, b, c, d


def _tol(ref64, ref32):
    return max(1e-5, 4 * rel_err(ref32, ref64))


def _check(out, fn64, fn32, name):
    r64 = fn64()
    r32 = fn32()
    e = rel_err(out, r64)
    assert e <= _tol(r64, r32), f"{name}: rel err {e:.3e} (oracle32 {rel_err(r32, r64):.3e})"


SIZES = [(1, 1), (7, 300), (300, 7), (257, 513), (1000, 1000), (64, 20000), (3000, 2000)]


@pytest.mark.parametrize("D", [2, 3])
@pytest.mark.parametrize("M,N", SIZES)
def test_reductions(dev, D, M, N):
    L = _lib()
    sigma = 0.2
    x, y, b, c, d = _data(M, N, D, seed=M * 31 + N)
    f = lambda t: t.float().to(dev)
    xs, ys, bs, cs, ds = map(f, (x, y, b, c, d))
    x3, y3, b3, c3, d3 = (t.float() for t in (x, y, b, c, d))
    cases = [
        (L.KBASE, dict(), lambda a: R.KBase(*a[:2], sigma)),
        (L.KREDSCAL, dict(b=ds), lambda a: R.KRedScal(a[0], a[1], a[4], sigma)),
        (L.KRED, dict(b=bs), lambda a: R.KRed(a[0], a[1], a[2], sigma)),
        (L.GRADK, dict(), lambda a: R.GradKRed(a[0], a[1], sigma)),
        (L.DDK, dict(b=bs), lambda a: R.DDKRed(a[0], a[1], a[2], sigma)),
        (L.GENDK, dict(b=bs, c=cs), lambda a: R.GenDKRed(a[0], a[1], a[2], a[3], sigma)),
        (L.HESSK, dict(b=bs, c=cs), lambda a: R.HessKRed(a[0], a[1], a[2], a[3], sigma)),
        (L.LAPK, dict(), lambda a: R.LapKRed(a[0], a[1], sigma)),
        (L.GRADLAPK, dict(), lambda a: R.GradLapKRed(a[0], a[1], sigma)),
    ]
    for op, kw, ref in cases:
        out = L.gauss_red(op, xs, ys, sigma, **kw)
        _check(out.cpu(), lambda: ref((x, y, b, c, d)), lambda: ref((x3, y3, b3, c3, d3)), f"op{op}")
    # GradKRed_rev: column reduction, rows = y
    out = L.gauss_red(L.GRADK_REV, ys, xs, sigma, b=cs)
    _check(out.cpu(), lambda: R.GradKRed_rev(x, y, c, sigma), lambda: R.GradKRed_rev(x3, y3, c3, sigma), "rev")
    # MinSqDist
    out = L.gauss_red(L.MIN_SQDIST, xs, ys, sigma)
    assert rel_err(out.cpu(), R.MinSqDist(x3, y3)) < 1e-6


def test_empty_columns(dev):
    L = _lib()
    x = torch.rand(10, 3, device=dev)
    y = torch.rand(0, 3, device=dev)
    b = torch.rand(0, 3, device=dev)
    assert torch.all(L.gauss_red(L.KRED, x, y, 0.3, b=b) == 0)
    assert torch.all(torch.isinf(L.gauss_red(L.MIN_SQDIST, x, y, 0.3)))


@pytest.mark.parametrize("version", ["classic", "hybrid", "logdet"])
@pytest.mark.parametrize("M,D", [(5, 2), (300, 2), (700, 3), (2500, 3)])
def test_ode_self_fwd(dev, version, M, D):
    L = _lib()
    g = torch.Generator().manual_seed(M + D)
    q = torch.rand(M, D, generator=g, dtype=torch.float64)
    p = torch.randn(M, D, generator=g, dtype=torch.float64) * 0.1
    gc = version == "logdet"
    wl = version != "classic"
    m = R.LDDMM(0.15, D, 50.0, gc, wl)
    m32 = R.LDDMM(0.15, D, 50.0, gc, wl)
    v64, mG64, c64 = m.ODE(q, p, torch.zeros(1, dtype=torch.float64))
    v32, mG32, c32 = m32.ODE(q.float(), p.float(), torch.zeros(1))
    H64, H32 = m.Hamiltonian(q, p), m32.Hamiltonian(q.float(), p.float())
    for alg in (0, 1, 2, 3, 4):  # eta = 0: ordered rows, symmetric, packed rows, MFMA, symmetric packed
        L.set_option("fwd_alg", alg)
        try:
            v, mG, gdiv, h = L.ode_self_fwd(q.float().to(dev), p.float().to(dev), 0.15, m.eta, wl,
                                            want_h=True)
        finally:
            L.set_option("fwd_alg", FWD_ALG_DEFAULT)
        assert rel_err(v.cpu(), v64) <= _tol(v64, v32), alg
        assert rel_err(mG.cpu(), mG64) <= _tol(mG64, mG32), alg
        assert rel_err(h.sum().cpu(), H64) <= _tol(H64, H32), alg
        if wl:
            assert rel_err(gdiv.sum().cpu(), c64) <= _tol(c64, c32), alg


@pytest.mark.parametrize("M,D", [(3, 2), (300, 2), (700, 3), (2100, 3), (4700, 3)])
@pytest.mark.parametrize("withlogdet,gradcomp", [(False, False), (True, False), (True, True), (False, True)])
def test_ode_self_bwd(dev, M, D, withlogdet, gradcomp):
    L = _lib()
    g = torch.Generator().manual_seed(7 * M + D)
    q = torch.rand(M, D, generator=g, dtype=torch.float64).requires_grad_(True)
    p = (0.1 * torch.randn(M, D, generator=g, dtype=torch.float64)).requires_grad_(True)
    a = torch.randn(M, D, generator=g, dtype=torch.float64)
    bm = torch.randn(M, D, generator=g, dtype=torch.float64)
    gam = torch.randn(1, generator=g, dtype=torch.float64)
    m = R.LDDMM(0.15, D, 50.0, gradcomp, withlogdet)
    v, mG, c = m.ODE(q, p, torch.zeros(1, dtype=torch.float64))
    Lf = (a * v).sum() + (bm * mG).sum() + (gam * c).sum()
    gq64, gp64 = torch.autograd.grad(Lf, (q, p))
    f = lambda t: t.detach().float().to(dev)
    for alg in (0, 1, 2, 3):  # eta = 0: pair algebras (lddmm_ops.hpp), symmetric kernel (+ packed)
        L.set_option("bwd_alg", alg)
        try:
            gq, gp = L.ode_self_bwd(f(q), f(p), f(a), f(bm), f(gam) if withlogdet else None, 0.15, m.eta)
        finally:
            L.set_option("bwd_alg", BWD_ALG_DEFAULT)
        assert rel_err(gq.cpu(), gq64) < 2e-5, (alg, rel_err(gq.cpu(), gq64))
        assert rel_err(gp.cpu(), gp64) < 2e-5, (alg, rel_err(gp.cpu(), gp64))


@pytest.mark.parametrize("M,N,D", [(40, 300, 2), (500, 1300, 3), (2000, 100, 3)])
@pytest.mark.parametrize("withlogdet,gradcomp", [(False, False), (True, False), (True, True)])
def test_ode_ext(dev, M, N, D, withlogdet, gradcomp):
    L = _lib()
    g = torch.Generator().manual_seed(M + N + D)
    q = torch.rand(M, D, generator=g, dtype=torch.float64).requires_grad_(True)
    p = (0.1 * torch.randn(M, D, generator=g, dtype=torch.float64)).requires_grad_(True)
    x = torch.rand(N, D, generator=g, dtype=torch.float64).requires_grad_(True)
    m = R.LDDMM(0.2, D, 50.0, gradcomp, withlogdet)
    vq, mG, c, vx = m.ODE(q, p, torch.zeros(1, dtype=torch.float64), x)
    f = lambda t: t.detach().float().to(dev)
    vx_h, gx_h = L.ode_ext_fwd(f(x), f(q), f(p), 0.2, m.eta, withlogdet)
    assert rel_err(vx_h.cpu(), vx) < 1e-5
    if withlogdet:
        assert rel_err(gx_h.sum().cpu(), c) < 1e-5
    a = torch.randn(N, D, generator=g, dtype=torch.float64)
    gam = torch.randn(1, generator=g, dtype=torch.float64)
    Lf = (a * vx).sum() + (gam * c).sum()
    gq64, gp64, gx64 = torch.autograd.grad(Lf, (q, p, x))
    gq = torch.zeros(M, D, device=dev)
    gp = torch.zeros(M, D, device=dev)
    gx = L.ode_ext_bwd(f(x), f(q), f(p), f(a), f(gam) if withlogdet else None, 0.2, m.eta, gq, gp)
    assert rel_err(gx.cpu(), gx64) < 2e-5
    assert rel_err(gq.cpu(), gq64) < 2e-5
    assert rel_err(gp.cpu(), gp64) < 2e-5


@pytest.mark.parametrize("M", [200, 20000])
@pytest.mark.parametrize("eta", [0.0, 0.02])
def test_fused_euler_steps(dev, M, eta):
    """dicp_lddmm_euler_step_f32 / _adjoint_step_f32 (epilogue-fused integrator updates) equal
    the unfused ODE pass + update, in the split (M=20000) and unsplit (M=200 <= one tile) paths."""
    L = _lib()
    g = torch.Generator().manual_seed(M)
    q = torch.rand(M, 3, generator=g).to(dev)
    p = (0.05 * torch.randn(M, 3, generator=g)).to(dev)
    lq = torch.randn(M, 3, generator=g).to(dev)
    lp = torch.randn(M, 3, generator=g).to(dev)
    aq = torch.randn(M, 3, generator=g).to(dev)
    gd = torch.full((1,), 0.3, device=dev)
    dt = 0.1
    v, mG, gr, _ = L.ode_self_fwd(q, p, 0.1, eta, True)
    qn, pn, g2 = L.euler_step(q, p, 0.1, eta, dt, True)
    assert rel_err(qn, q + dt * v) < 1e-6 and rel_err(pn, p + dt * mG) < 1e-6
    assert torch.equal(g2, gr)
    Qo, Po = torch.empty_like(q), torch.empty_like(q)
    L.euler_step(q, p, 0.1, eta, dt, False, q_out=Qo, p_out=Po)
    assert rel_err(Qo, qn) < 1e-6 and rel_err(Po, pn) < 1e-6   # other variant: other split order
    gq, gp = L.ode_self_bwd(q, p, lq, lp, gd, 0.1, eta)
    for addq in (None, aq):
        lqn, lpn = L.euler_adjoint_step(q, p, lq, lp, gd, 0.1, eta, dt, addq, None)
        ref_q = lq + dt * gq + (0 if addq is None else addq)
        assert rel_err(lqn, ref_q) < 1e-6 and rel_err(lpn, lp + dt * gp) < 1e-6


@pytest.mark.parametrize("M", [1, 129, 5000, 50000])
@pytest.mark.parametrize("eta", [0.0, 0.02])
def test_adjoint_step_gp_only(dev, M, eta):
    """euler_adjoint_step(want_lq=False) (lq_next = NULL at the C-ABI: the gq half of the
    symmetric eta = 0 VJP is skipped) gives the lp_next of the full step."""
    L = _lib()
    g = torch.Generator().manual_seed(M + 9)
    q = torch.rand(M, 3, generator=g).to(dev)
    p = (0.05 * torch.randn(M, 3, generator=g)).to(dev)
    lq = torch.randn(M, 3, generator=g).to(dev)
    lp = torch.randn(M, 3, generator=g).to(dev)
    ap = torch.randn(M, 3, generator=g).to(dev)
    gd = torch.full((1,), 0.3, device=dev)
    lqn, lpn = L.euler_adjoint_step(q, p, lq, lp, gd, 0.1, eta, 0.1, None, ap)
    none, lpn1 = L.euler_adjoint_step(q, p, lq, lp, gd, 0.1, eta, 0.1, None, ap, want_lq=False)
    assert none is None
    assert rel_err(lpn1, lpn) < 1e-6, rel_err(lpn1, lpn)
    none, lpn2 = L.euler_adjoint_step(q, p, lq, lp, gd, 0.1, eta, 0.1, None, ap, want_lq=False)
    assert torch.equal(lpn1, lpn2)      # deterministic


@pytest.mark.parametrize("M", [1, 129, 5000, 50000])
@pytest.mark.parametrize("want_lq", [True, False])
@pytest.mark.parametrize("eta", [0.0, 0.02])
def test_adjoint_step_zero_momentum_cotangent(dev, M, want_lq, eta):
    """euler_adjoint_step(lp=None) (lp = NULL at the C-ABI: zero cotangent on mG, the b
    terms of the symmetric VJP skipped; also with the gq half skipped) == the step with
    explicit zeros; both models (eta = 0: SymBwdPk<., ., true>, eta != 0: SymBwdEtaPk)."""
    L = _lib()
    g = torch.Generator().manual_seed(M + 13)
    q = torch.rand(M, 3, generator=g).to(dev)
    p = (0.05 * torch.randn(M, 3, generator=g)).to(dev)
    lq = torch.randn(M, 3, generator=g).to(dev)
    aq = torch.randn(M, 3, generator=g).to(dev)
    gd = torch.full((1,), 0.3, device=dev)
    z = torch.zeros_like(lq)
    lqn, lpn = L.euler_adjoint_step(q, p, lq, z, gd, 0.1, eta, 0.1, aq, None, want_lq=want_lq)
    lqn0, lpn0 = L.euler_adjoint_step(q, p, lq, None, gd, 0.1, eta, 0.1, aq, None, want_lq=want_lq)
    assert rel_err(lpn0, lpn) < 1e-6, rel_err(lpn0, lpn)
    if want_lq:
        assert rel_err(lqn0, lqn) < 1e-6, rel_err(lqn0, lqn)
    else:
        assert lqn0 is None
    for W in (2, 3):   # pair-subset parts with a zero cotangent (row split)
        sq, sp = torch.zeros_like(lq), torch.zeros_like(lq)
        for r in range(W):
            pq, pp = L.ode_self_bwd_part(q, p, lq, None, gd, 0.1, eta, r, W, want_gq=want_lq)
            if want_lq:
                sq += pq
            else:
                assert pq is None
            sp += pp
        gq, gp = L.ode_self_bwd(q, p, lq, z, gd, 0.1, eta)
        assert rel_err(sp, gp) < 2e-6, rel_err(sp, gp)
        if want_lq:
            assert rel_err(sq, gq) < 2e-6, rel_err(sq, gq)


@pytest.mark.parametrize("M", [129, 5000])
def test_eta_zero_cotangent_on_other_algs(dev, M):
    """With a non-packed eta VJP selected (bwd_eta_alg 0 / 1, no zero-cotangent shortcut) the
    host materialises the zeros: lp=None still gives the step with explicit zeros."""
    L = _lib()
    g = torch.Generator().manual_seed(M + 17)
    q = torch.rand(M, 3, generator=g).to(dev)
    p = (0.05 * torch.randn(M, 3, generator=g)).to(dev)
    lq = torch.randn(M, 3, generator=g).to(dev)
    gd = torch.full((1,), 0.3, device=dev)
    ref = L.euler_adjoint_step(q, p, lq, None, gd, 0.1, 0.02, 0.1)
    try:
        for alg in (0, 1):
            L.set_option("bwd_eta_alg", alg)
            got = L.euler_adjoint_step(q, p, lq, None, gd, 0.1, 0.02, 0.1)
            assert rel_err(got[0], ref[0]) < 2e-6 and rel_err(got[1], ref[1]) < 2e-6
    finally:
        L.set_option("bwd_eta_alg", 2)


def test_dpp_wave_rol_semantics(dev):
    """The symmetric VJP rotates column sums with DPP wave_rol:1 assuming lane l reads lane
    l + 1 (lddmm_sym.hpp rol1); pin that on the hardware."""
    import ctypes
    import os
    mb = ctypes.CDLL(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                  "diff-icp_amd", "libdifficp_microbench.so"))
    out = torch.zeros(64, dtype=torch.int32, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert mb.dicp_mb_dpp(0, ctypes.c_void_p(out.data_ptr()), st) == 0
    assert out.cpu().tolist() == [(l + 1) % 64 for l in range(64)]


@pytest.mark.parametrize("M", [128, 129, 1000, 5000, 50000])
def test_sym_bwd_vs_ordered(dev, M):
    """Symmetric pair-once VJP == ordered kernel (alg 1) up to fp32 summation order, incl.
    partial last groups and quads; deterministic run to run."""
    L = _lib()
    g = torch.Generator().manual_seed(M + 1)
    q = torch.rand(M, 3, generator=g).to(dev)
    p = (0.05 * torch.randn(M, 3, generator=g)).to(dev)
    a = torch.randn(M, 3, generator=g).to(dev)
    b = torch.randn(M, 3, generator=g).to(dev)
    gd = torch.full((1,), -0.4, device=dev)
    L.set_option("bwd_alg", 1)
    try:
        gq1, gp1 = L.ode_self_bwd(q, p, a, b, gd, 0.1, 0.0)
        L.set_option("bwd_alg", 2)  # scalar rows
        gq2, gp2 = L.ode_self_bwd(q, p, a, b, gd, 0.1, 0.0)
        gq3, gp3 = L.ode_self_bwd(q, p, a, b, gd, 0.1, 0.0)
    finally:
        L.set_option("bwd_alg", BWD_ALG_DEFAULT)
    assert rel_err(gq2, gq1) < 2e-6 and rel_err(gp2, gp1) < 2e-6
    assert torch.equal(gq2, gq3) and torch.equal(gp2, gp3)
    gq4, gp4 = L.ode_self_bwd(q, p, a, b, gd, 0.1, 0.0)  # default: packed-FP32 rows
    gq5, gp5 = L.ode_self_bwd(q, p, a, b, gd, 0.1, 0.0)
    assert rel_err(gq4, gq1) < 2e-6 and rel_err(gp4, gp1) < 2e-6
    assert torch.equal(gq4, gq5) and torch.equal(gp4, gp5)


@pytest.mark.parametrize("M", [1, 127, 128, 129, 1000, 5000, 50000])
@pytest.mark.parametrize("want_div", [True, False])
@pytest.mark.parametrize("alg", [1, 2, 3, 4])
def test_sym_fwd_vs_ordered(dev, M, want_div, alg):
    """Symmetric pair-once (alg 1), packed-FP32 (alg 2) and matrix-core (alg 3) forwards == the
    ordered-row forward up to fp32 summation order (partial last groups / row pairs / row tiles
    included), every output incl. the fused Euler epilogue; deterministic run to run."""
    L = _lib()
    g = torch.Generator().manual_seed(M + 11)
    q = torch.rand(M, 3, generator=g).to(dev)
    p = (0.05 * torch.randn(M, 3, generator=g)).to(dev)
    L.set_option("fwd_alg", 0)                                        # ordered rows
    ref = L.ode_self_fwd(q, p, 0.1, 0.0, want_div, want_h=True)
    qn0, pn0, _ = L.euler_step(q, p, 0.1, 0.0, 0.1, want_div)
    L.set_option("fwd_alg", alg)
    try:
        out = L.ode_self_fwd(q, p, 0.1, 0.0, want_div, want_h=True)
        out2 = L.ode_self_fwd(q, p, 0.1, 0.0, want_div, want_h=True)
        qn1, pn1, _ = L.euler_step(q, p, 0.1, 0.0, 0.1, want_div)
    finally:
        L.set_option("fwd_alg", FWD_ALG_DEFAULT)
    # alg 3 splits z = q_i - q_j into centred row / column terms (mfma_fwd.hpp): its fp32
    # error grows with the rows' spread against sigma -> the SURVEY 8c criterion, 1e-5
    tol = 1e-5 if alg == 3 else 2e-6
    for k, (a, b) in enumerate(zip(out, ref)):
        if b is None:
            continue
        assert rel_err(a, b) < tol, (k, rel_err(a, b))
    for a, b in zip(out, out2):
        if a is not None:
            assert torch.equal(a, b)
    assert rel_err(qn1, qn0) < 1e-7 and rel_err(pn1, pn0) < tol


@pytest.mark.parametrize("extent,ordered", [(1.0, False), (1.0, True), (5.0, True), (20.0, True)])
@pytest.mark.parametrize("M", [1000, 30000])
def test_mfma_fwd_precision_vs_extent(dev, M, extent, ordered):
    """The matrix-core forward splits z = q_i - q_j into centred row / column terms; its error
    grows with the spread of a workgroup's rows against sigma (cancellation).  With the rows
    visited in spatial order (shooting.spatial_order, what LDDMMModel.Shoot passes) the error
    stays within the SURVEY 8c criterion (1e-5) for clouds of extent 10 / 50 / 200 sigma;
    unordered rows only at 10 sigma.  Against float64 sums on 256 sampled rows."""
    from difficp_amd.core.shooting import spatial_order
    L = _lib()
    g = torch.Generator().manual_seed(M + int(extent))
    q64 = extent * torch.rand(M, 3, generator=g, dtype=torch.float64)
    p64 = 0.05 * torch.randn(M, 3, generator=g, dtype=torch.float64)
    sig = 0.1
    qd = q64.float().to(dev)
    order = spatial_order(qd) if ordered else None
    L.set_option("fwd_alg", 3)
    try:
        v, mG, gdiv, h = L.ode_self_fwd(qd, p64.float().to(dev), sig, 0.0, True, want_h=True,
                                        order=order)
        qn, pn, gn = L.euler_step(qd, p64.float().to(dev), sig, 0.0, 0.1, True, order=order)
    finally:
        L.set_option("fwd_alg", FWD_ALG_DEFAULT)
    assert torch.equal(gn, gdiv)       # same kernel, same order: bitwise
    assert rel_err(qn, qd + 0.1 * v) < 1e-7
    rows = torch.randperm(M, generator=g)[:256]
    qf = q64.float().double()   # the positions the kernel sees
    z = qf[rows][:, None, :] - qf[None, :, :]
    K = torch.exp(-(z ** 2).sum(-1) / (2 * sig ** 2))
    pf = p64.float().double()
    V = K @ pf
    pp = pf[rows] @ pf.t()
    mG64 = (1 / sig ** 2) * ((K * pp)[:, :, None] * z).sum(1)        # -GenDKRed(q,q,p,p)
    Z = -(1 / sig ** 2) * (K[:, :, None] * z).sum(1)
    assert rel_err(v[rows].cpu(), V) < 1e-5, rel_err(v[rows].cpu(), V)
    assert rel_err(mG[rows].cpu(), mG64) < 1e-5, rel_err(mG[rows].cpu(), mG64)
    gd = (pf[rows] * Z).sum(1)
    assert rel_err(gdiv[rows].cpu(), gd) < 1e-5, rel_err(gdiv[rows].cpu(), gd)


def _mfma_wg_modes(q, sigma, order):
    """Which workgroups of the matrix-core forward take the MFMA branch (mfma_fwd.hpp: rows'
    spread about their mean <= kMfRmax = 4 in scaled units), replicated on the host."""
    import math
    a = math.sqrt(1.4426950408889634 / (2 * sigma * sigma))
    qs = (q.double() * a)[order.long()] if order is not None else q.double() * a
    modes = []
    for i0 in range(0, qs.shape[0], 256):
        blk = qs[i0:i0 + 256]
        modes.append(bool(((blk - blk.mean(0)) ** 2).sum(1).max() <= 16.0))
    return modes


@pytest.mark.parametrize("M", [1, 15, 255, 257, 1000, 20000])
@pytest.mark.parametrize("sigma", [0.1, 0.5])
@pytest.mark.parametrize("ordered", [False, True])
def test_mfma_fwd_modes_vs_ordered(dev, M, sigma, ordered):
    """Matrix-core forward (fwd_alg 3) in both workgroup branches (MFMA channel sums for
    compact rows, direct VALU sums for spread rows) == the ordered-row forward (alg 0) to the
    SURVEY 8c criterion, every output incl. the fused Euler epilogue, row orders honoured
    (outputs indexed by row), deterministic run to run."""
    from difficp_amd.core.shooting import spatial_order
    L = _lib()
    g = torch.Generator().manual_seed(M + 3)
    q = torch.rand(M, 3, generator=g).to(dev)
    p = (0.05 * torch.randn(M, 3, generator=g)).to(dev)
    order = spatial_order(q) if ordered else None
    modes = _mfma_wg_modes(q.cpu(), sigma, None if order is None else order.cpu())
    if ordered and (M >= 20000 or (sigma == 0.5 and M >= 1000)):
        assert any(modes)          # the case exercises the MFMA branch
    L.set_option("fwd_alg", 0)
    try:
        ref = L.ode_self_fwd(q, p, sigma, 0.0, True, want_h=True)
        L.set_option("fwd_alg", 3)
        out = L.ode_self_fwd(q, p, sigma, 0.0, True, want_h=True, order=order)
        out2 = L.ode_self_fwd(q, p, sigma, 0.0, True, want_h=True, order=order)
        qn, pn, gn = L.euler_step(q, p, sigma, 0.0, 0.1, True, order=order)
    finally:
        L.set_option("fwd_alg", FWD_ALG_DEFAULT)
    for k, (a, b) in enumerate(zip(out, ref)):
        assert rel_err(a, b) < 1e-5, (k, rel_err(a, b), modes)
    for a, b in zip(out, out2):
        assert torch.equal(a, b)
    assert torch.equal(gn, out[2])
    assert rel_err(qn, q + 0.1 * out[0]) < 1e-7 and rel_err(pn, p + 0.1 * out[1]) < 1e-6


@pytest.mark.parametrize("M", [1, 128, 129, 1000, 5000, 50000])
def test_sym_bwd_eta_vs_ordered(dev, M):
    """Symmetric pair-once eta != 0 VJP (SymBwdEta) == the ordered OpOdeSelfBwdEta up to fp32
    summation order, incl. partial last groups; deterministic run to run."""
    L = _lib()
    g = torch.Generator().manual_seed(M + 5)
    q = torch.rand(M, 3, generator=g).to(dev)
    p = (0.05 * torch.randn(M, 3, generator=g)).to(dev)
    a = torch.randn(M, 3, generator=g).to(dev)
    b = torch.randn(M, 3, generator=g).to(dev)
    gd = torch.full((1,), -0.4, device=dev)
    res = {}
    try:
        for alg in (0, 1, 2):  # ordered, symmetric scalar rows, symmetric packed-FP32 rows
            L.set_option("bwd_eta_alg", alg)
            res[alg] = [L.ode_self_bwd(q, p, a, b, gd, 0.1, 1e-3) for _ in range(2 if alg else 1)]
    finally:
        L.set_option("bwd_eta_alg", BWD_ETA_ALG_DEFAULT)
    gq0, gp0 = res[0][0]
    for alg in (1, 2):
        (gq1, gp1), (gq2, gp2) = res[alg]
        assert torch.isfinite(gq1).all() and torch.isfinite(gp1).all()
        assert rel_err(gq1, gq0) < 5e-6 and rel_err(gp1, gp0) < 5e-6, (alg, rel_err(gq1, gq0), rel_err(gp1, gp0))
        assert torch.equal(gq1, gq2) and torch.equal(gp1, gp2)
