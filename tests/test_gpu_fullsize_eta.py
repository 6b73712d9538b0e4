"""Full-size (C2: 50k support points, sigma 0.1) parity of the kernels beyond the eta = 0
self-interaction pass that tests/test_gpu_fullsize.py covers:

  * the gradcomponent model (eta = 1/lambda != 0), which ICP_two_set actually runs
    (ICP_two_set.py:203-207 leaves gradcomponent at its default True, LDDMM.py:34, 198-203):
    fused forward (v, mG, g, h) and symmetric VJP at eta = 1e-3 (lambda = 1e3, C2') and 0.02;
  * the VJP variants the shooting adjoint launches: zero mG cotangent (first adjoint step),
    gp-only (last step when q0 needs no gradient), divergence rows reused from the forward;
  * the external-point passes (custom support / LDDMMRegistration.apply, LDDMM.py:219-227):
    ode_ext_fwd (v(x), divergence rows) and ode_ext_bwd (gx and the accumulated gq, gp).

192 sampled rows (or support columns), each a reduction over ALL 50k partners, against
float64 restatements of the reference formulas (tests/fullsize_ref.py, pinned against the
oracle at small size by tests/test_fullsize_formulas.py), computed in float64 on the device.
Tolerances (norm-wise relative): 1e-5 forward, 2e-5 backward.
"""
import pytest
import torch

import fullsize_ref as F
from conftest import rel_err

pytestmark = pytest.mark.gpu

M = 50000
SIG = 0.1
NSUB = 192


@pytest.fixture(scope="module")
def pts(dev):
    g = torch.Generator().manual_seed(2025)
    q = torch.rand(M, 3, generator=g, dtype=torch.float64)
    p = 0.01 * torch.randn(M, 3, generator=g, dtype=torch.float64)
    a = torch.randn(M, 3, generator=g, dtype=torch.float64)
    b = torch.randn(M, 3, generator=g, dtype=torch.float64)
    x = torch.rand(M, 3, generator=g, dtype=torch.float64)
    ax = torch.randn(M, 3, generator=g, dtype=torch.float64)
    sub = torch.randperm(M, generator=g)[:NSUB].to(dev)
    d = {k: v.to(dev) for k, v in dict(q=q, p=p, a=a, b=b, x=x, ax=ax).items()}
    d.update({k + "f": v.float().contiguous() for k, v in list(d.items())})
    d["sub"] = sub
    return d


@pytest.mark.parametrize("eta", [1e-3, 0.02])
def test_fwd_eta_fullsize_subset(pts, eta):
    from difficp_amd import _lib
    v, mG, g, h = _lib.ode_self_fwd(pts["qf"], pts["pf"], SIG, eta, True, want_h=True)
    s = pts["sub"]
    v64, mG64, g64, h64 = F.self_terms(pts["q"][s], pts["p"][s], pts["q"], pts["p"], SIG, eta)
    assert rel_err(v[s], v64) < 1e-5
    assert rel_err(mG[s], mG64) < 1e-5
    assert rel_err(g[s], g64) < 1e-5
    assert rel_err(h[s], h64) < 1e-5


@pytest.mark.parametrize("eta", [1e-3, 0.02])
def test_bwd_eta_fullsize_subset(pts, eta, dev):
    from difficp_amd import _lib
    gam = 0.37
    gq, gp = _lib.ode_self_bwd(pts["qf"], pts["pf"], pts["af"], pts["bf"],
                               torch.full((1,), gam, device=dev), SIG, eta)
    s = pts["sub"]
    gq64, gp64 = F.self_vjp_subset(pts["q"], pts["p"], pts["a"], pts["b"], gam, s, SIG, eta)
    assert rel_err(gq[s], gq64) < 2e-5
    assert rel_err(gp[s], gp64) < 2e-5


@pytest.mark.parametrize("eta", [0.0, 1e-3])
def test_bwd_variants_fullsize_subset(pts, eta, dev):
    """Zero-mG-cotangent (lp = NULL) and gp-only (lq_next = NULL) adjoint steps, dt = 1:
    lq_next = lq + gq, lp_next = lp + gp."""
    from difficp_amd import _lib
    gam = 0.37
    gd = torch.full((1,), gam, device=dev)
    s = pts["sub"]
    q, p, a, b = pts["qf"], pts["pf"], pts["af"], pts["bf"]
    lqn, lpn = _lib.euler_adjoint_step(q, p, a, None, gd, SIG, eta, 1.0)
    gq64, gp64 = F.self_vjp_subset(pts["q"], pts["p"], pts["a"], None, gam, s, SIG, eta)
    assert rel_err(lqn[s].double() - pts["a"][s], gq64) < 2e-5
    assert rel_err(lpn[s], gp64) < 2e-5
    none, lpn = _lib.euler_adjoint_step(q, p, a, b, gd, SIG, eta, 1.0, want_lq=False)
    assert none is None
    gq64, gp64 = F.self_vjp_subset(pts["q"], pts["p"], pts["a"], pts["b"], gam, s, SIG, eta)
    assert rel_err(lpn[s].double() - pts["b"][s], gp64) < 2e-5


def test_bwd_zs_fullsize_subset(pts, dev):
    """Divergence rows written by the fused forward (zs_out) and reused by the adjoint step
    (the default shooting at eta = 0): forward outputs unchanged, VJP equal to the formula."""
    from difficp_amd import _lib
    if not _lib.zs_ok(0.0):
        pytest.skip("divergence-row variant not selected in this build")
    gam = 0.37
    s = pts["sub"]
    q, p, a, b = pts["qf"], pts["pf"], pts["af"], pts["bf"]
    Zs = torch.empty_like(q)
    qn, pn, g = _lib.euler_step(q, p, SIG, 0.0, 0.1, True, zs_out=Zs)
    qn0, pn0, g0 = _lib.euler_step(q, p, SIG, 0.0, 0.1, True)
    assert torch.equal(qn, qn0) and torch.equal(pn, pn0) and torch.equal(g, g0)
    # zs_i = sum_j K (q_i - q_j) = -sigma^2 GradKRed(q_i, q); with zero momenta and eta = 1 the
    # velocity of self_terms is v = -GradKRed, so zs = sigma^2 v
    zp = torch.zeros_like(pts["p"])
    zs64 = SIG ** 2 * F.self_terms(pts["q"][s], zp[s], pts["q"], zp, SIG, 1.0)[0]
    assert rel_err(Zs[s], zs64) < 1e-5
    lqn, lpn = _lib.euler_adjoint_step(q, p, a, b, torch.full((1,), gam, device=dev), SIG, 0.0, 1.0,
                                       zs=Zs)
    gq64, gp64 = F.self_vjp_subset(pts["q"], pts["p"], pts["a"], pts["b"], gam, s, SIG, 0.0)
    assert rel_err(lqn[s].double() - pts["a"][s], gq64) < 2e-5
    assert rel_err(lpn[s].double() - pts["b"][s], gp64) < 2e-5


@pytest.mark.parametrize("eta", [0.0, 1e-3])
@pytest.mark.parametrize("red_alg,ext_alg", [(1, 1), (0, 1), (0, 0)])   # centred / packed / generic
def test_ext_fwd_fullsize_subset_eta(pts, eta, red_alg, ext_alg):
    from difficp_amd import _lib
    _lib.set_option("red_alg", red_alg)
    _lib.set_option("ext_alg", ext_alg)
    try:
        vx, gx = _lib.ode_ext_fwd(pts["xf"], pts["qf"], pts["pf"], SIG, eta, True)
    finally:
        _lib.set_option("red_alg", 1)
        _lib.set_option("ext_alg", 1)
    s = pts["sub"]
    v64, g64 = F.ext_terms(pts["x"][s], pts["q"], pts["p"], SIG, eta)
    assert rel_err(vx[s], v64) < 1e-5
    assert rel_err(gx[s], g64) < 1e-5


@pytest.mark.parametrize("eta", [0.0, 1e-3])
@pytest.mark.parametrize("ext_alg", [1, 0])   # packed (eta = 0) / generic
def test_ext_bwd_fullsize_subset(pts, eta, dev, ext_alg):
    """ode_ext_bwd: gx rows (x side) and the gq, gp accumulated into the caller's buffers
    (support side, a column reduction over the 50k external points)."""
    from difficp_amd import _lib
    gam = 0.29
    q, p = pts["qf"], pts["pf"]
    gq0 = torch.randn_like(q)
    gq, gp = gq0.clone(), torch.zeros_like(q)
    _lib.set_option("ext_alg", ext_alg)
    try:
        gx = _lib.ode_ext_bwd(pts["xf"], q, p, pts["axf"], torch.full((1,), gam, device=dev), SIG,
                              eta, gq, gp)
    finally:
        _lib.set_option("ext_alg", 1)
    s = pts["sub"]
    gx64, gq64, gp64 = F.ext_vjp_subset(pts["x"], pts["q"], pts["p"], pts["ax"], gam, s, s, SIG, eta)
    assert rel_err(gx[s], gx64) < 2e-5
    assert rel_err(gq[s].double() - gq0[s].double(), gq64) < 2e-5    # accumulated
    assert rel_err(gp[s], gp64) < 2e-5
