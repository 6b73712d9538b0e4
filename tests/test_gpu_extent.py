"""Precision of the pair kernels against float64 as the cloud's offset and extent grow (units
of sigma).  The fused shooting kernels work in scaled coordinates q' = alpha (q - q_0) with the
origin at the first support point (csrc/common.hpp ld_coord), so a translation of the data
costs nothing; the rounding of q' grows with the extent (2.8e-6 at 100
sigma, 1.3e-5 at 300 sigma, profiles/r03_extent_precision.jsonl), which LDDMMModel.Optimize
reports with a warning beyond 200 sigma.  KRed and the external-point passes keep raw
differences (exact for nearby points) and stay at the reference's accuracy at any extent.

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


def test_optimize_warns_beyond_extent(dev):
    from difficp_amd.core.LDDMM import LDDMMModel
    spec = {"device": dev, "dtype": torch.float32}
    for E, expect in ((50, False), (500, True)):
        LM = LDDMMModel(sigma=SIG, D=3, lambd=1.0, version="classic", spec=spec, nt=2)
        g = torch.Generator().manual_seed(E)
        q0 = (E * SIG * torch.rand(300, 3, generator=g)).to(dev)
        p0 = torch.zeros_like(q0)
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            LM.Optimize(lambda x1: (x1 ** 2).sum() * 0, q0, p0, nmax=1)
        hit = any("spans" in str(x.message) for x in w)
        assert hit == expect, (E, [str(x.message) for x in w])
