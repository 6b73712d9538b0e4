"""Precision of the pair kernels against float64 as the cloud's offset and extent grow (units
of sigma).  The fused shooting kernels work by default in scaled coordinates q' = alpha (q - q_0)
with the origin at the first support point (csrc/common.hpp ld_coord), so a translation of the
data costs nothing; the rounding of q' grows with the extent (2.8e-6 at 100
sigma, 1.3e-5 at 300 sigma, profiles/r03_extent_precision.jsonl).  Their raw-coordinate
variants (library option coord_raw, per host thread) keep exact differences at any extent, and
LDDMMModel.Shoot selects them by itself beyond RAW_EXTENT_SIGMA.  KRed and the external-point
passes always use raw differences.

256 sampled rows against float64 sums over all 20k points (tests/fullsize_ref.py); inputs are
rounded to float32 first.  Criterion 1e-5 norm-wise."""
import warnings

import pytest
import torch

import fullsize_ref as F
from conftest import rel_err

pytestmark = pytest.mark.gpu
SIG = 0.1
M = 20000


def _cloud(E, off, dev, seed=0):
    g = torch.Generator().manual_seed(seed + E + off)
    q = (E * SIG * torch.rand(M, 3, generator=g, dtype=torch.float64) + off * SIG).float().double()
    p = (0.01 * torch.randn(M, 3, generator=g, dtype=torch.float64)).float().double()
    a = torch.randn(M, 3, generator=g, dtype=torch.float64).float().double()
    b = torch.randn(M, 3, generator=g, dtype=torch.float64).float().double()
    sub = torch.randperm(M, generator=g)[:256].to(dev)
    return [t.to(dev) for t in (q, p, a, b)] + [sub]


@pytest.mark.parametrize("E,off,tol", [(10, 1000, 2e-6), (10, 10000, 2e-6), (100, 0, 1e-5), (100, 1000, 1e-5)])
def test_shooting_kernels_offset_and_extent(dev, E, off, tol):
    from difficp_amd import _lib as L
    q, p, a, b, sub = _cloud(E, off, dev)
    qf, pf, af, bf = (t.float() for t in (q, p, a, b))
    v, mG, g, _ = L.ode_self_fwd(qf, pf, SIG, 0.0, True)
    v64, mG64, g64, _ = F.self_terms(q[sub], p[sub], q, p, SIG, 0.0)
    for out, ref in ((v, v64), (mG, mG64), (g, g64)):
        assert rel_err(out[sub], ref) < tol
    gq, gp = L.ode_self_bwd(qf, pf, af, bf, torch.full((1,), 0.3, device=dev), SIG, 0.0)
    gq64, gp64 = F.self_vjp_subset(q, p, a, b, 0.3, sub, SIG, 0.0)
    assert rel_err(gq[sub], gq64) < tol
    assert rel_err(gp[sub], gp64) < tol


@pytest.mark.parametrize("opts", [(1, 1), (0, 1), (0, 0), (2, 1)])   # (red_alg, ext_alg)
def test_raw_difference_kernels_any_extent(dev, opts):
    """KRed and the external-point forward at 1000 sigma extent on every path."""
    from difficp_amd import _lib as L
    q, p, _, _, sub = _cloud(1000, 0, dev)
    qf, pf = q.float(), p.float()
    xe = (q + 0.3 * SIG).float()
    kr64, _ = F.ext_terms(q[sub], q, p, SIG, 0.0)
    vx64, gx64 = F.ext_terms(xe.double()[sub], q, p, SIG, 0.0)
    L.set_option("red_alg", opts[0])
    L.set_option("ext_alg", opts[1])
    try:
        kr = L.gauss_red(L.KRED, qf, qf, SIG, b=pf)
        vx, gx = L.ode_ext_fwd(xe, qf, pf, SIG, 0.0, True)
    finally:
        L.set_option("red_alg", 1)
        L.set_option("ext_alg", 1)
    assert rel_err(kr[sub], kr64) < 1e-6
    assert rel_err(vx[sub], vx64) < 1e-6
    assert rel_err(gx[sub], gx64) < 1e-6


@pytest.mark.parametrize("E", [300, 1000])
def test_raw_coordinate_shooting_kernels(dev, E):
    """coord_raw: the packed forward (with and without the divergence rows, eta = 0 and 1e-3)
    and the packed symmetric VJP (full, zero-mG-cotangent, gp-only) at extents where the scaled
    form misses the criterion."""
    from difficp_amd import _lib as L
    q, p, a, b, sub = _cloud(E, 0, dev)
    qf, pf, af, bf = (t.float() for t in (q, p, a, b))
    gd = torch.full((1,), 0.3, device=dev)
    with L.coord_mode(True):
        v, mG, g, _ = L.ode_self_fwd(qf, pf, SIG, 0.0, True)
        ve, mGe, ge, _ = L.ode_self_fwd(qf, pf, SIG, 1e-3, True)
        Zs = torch.empty_like(qf)
        qn, pn, gz = L.euler_step(qf, pf, SIG, 0.0, 1.0, True, zs_out=Zs)
        gq, gp = L.ode_self_bwd(qf, pf, af, bf, gd, SIG, 0.0)
        lq0, lp0 = L.euler_adjoint_step(qf, pf, af, None, gd, SIG, 0.0, 1.0)
        none, lpg = L.euler_adjoint_step(qf, pf, af, bf, gd, SIG, 0.0, 1.0, want_lq=False)
    assert L.get_option("coord_raw") == 0                   # restored
    v64, mG64, g64, _ = F.self_terms(q[sub], p[sub], q, p, SIG, 0.0)
    ve64, mGe64, ge64, _ = F.self_terms(q[sub], p[sub], q, p, SIG, 1e-3)
    for out, ref in ((v, v64), (mG, mG64), (g, g64), (ve, ve64), (mGe, mGe64), (ge, ge64)):
        assert rel_err(out[sub], ref) < 1e-5
    # the fused Euler step (dt = 1): p + mG (q + v would round v against |q| ~ E sigma)
    assert rel_err(pn[sub].double() - p[sub], mG64) < 1e-5 and qn.shape == q.shape
    zp = torch.zeros_like(p)
    zs64 = SIG ** 2 * F.self_terms(q[sub], zp[sub], q, zp, SIG, 1.0)[0]
    assert rel_err(Zs[sub], zs64) < 1e-5
    gq64, gp64 = F.self_vjp_subset(q, p, a, b, 0.3, sub, SIG, 0.0)
    assert rel_err(gq[sub], gq64) < 1e-5 and rel_err(gp[sub], gp64) < 1e-5
    gq64, gp64 = F.self_vjp_subset(q, p, a, None, 0.3, sub, SIG, 0.0)
    assert rel_err(lq0[sub].double() - a[sub], gq64) < 1e-5 and rel_err(lp0[sub], gp64) < 1e-5
    gq64, gp64 = F.self_vjp_subset(q, p, a, b, 0.3, sub, SIG, 0.0)
    assert none is None and rel_err(lpg[sub].double() - b[sub], gp64) < 1e-5


def test_coord_raw_close_to_scaled_at_small_extent(dev):
    """Both coordinate forms agree to float32 rounding on the default workload's geometry."""
    from difficp_amd import _lib as L
    q, p, a, b, sub = _cloud(10, 0, dev)
    qf, pf, af, bf = (t.float() for t in (q, p, a, b))
    gd = torch.full((1,), 0.3, device=dev)
    outs = []
    for raw in (False, True):
        with L.coord_mode(raw):
            outs.append(L.ode_self_fwd(qf, pf, SIG, 0.0, True)[:3] + L.ode_self_bwd(qf, pf, af, bf, gd, SIG, 0.0))
    for u, w in zip(*outs):
        assert rel_err(u, w.double()) < 2e-6


def test_shoot_auto_mode_switches_to_raw(dev):
    """LDDMMModel.coord_mode "auto": a support spanning more than RAW_EXTENT_SIGMA shoots with
    the raw kernels (bitwise the forced "raw" shooting), a compact one with the scaled kernels."""
    from difficp_amd.core.LDDMM import LDDMMModel
    spec = {"device": dev, "dtype": torch.float32}
    for E, raw in ((50, False), (500, True)):
        g = torch.Generator().manual_seed(E)
        q0 = (E * SIG * torch.rand(2000, 3, generator=g)).to(dev)
        p0 = (0.01 * torch.randn(2000, 3, generator=g)).to(dev)
        res = {}
        for mode in ("auto", "raw", "scaled"):
            LM = LDDMMModel(sigma=SIG, D=3, lambd=1.0, version="hybrid", spec=spec, nt=3, scheme="Euler")
            LM.coord_mode = mode
            sh = LM.Shoot(q0, p0)
            res[mode] = (sh.Q.clone(), sh.P.clone())
        same = "raw" if raw else "scaled"
        assert torch.equal(res["auto"][0], res[same][0]) and torch.equal(res["auto"][1], res[same][1])
