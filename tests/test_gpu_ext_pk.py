"""Parity of the external-point passes on every path the library dispatches to (SURVEY 8(a)
a9/a10/a12 with external points x, LDDMM.py:100-138, :219-227; the apply / custom-support
path): the packed scaled-coordinate kernels (csrc/ext_pk.hpp, `ext_alg` 1, default below the
centred sizes), the generic scalar kernels (`ext_alg` 0) and, for the forward, the centred
expansion (`red_alg` 2 forces it at any size) -- against float64 restatements of the reference
formulas (tests/fullsize_ref.py, pinned against the oracle by tests/test_fullsize_formulas.py).

Ragged sizes (1 row, sizes that are not multiples of the 512-row workgroup or the 256-column
tile), D = 2 and 3, with and without the divergence cotangent.  Tolerances (norm-wise
relative): 1e-5 forward, 2e-5 backward.
"""
import contextlib

import pytest
import torch

import fullsize_ref as F
from conftest import rel_err

pytestmark = pytest.mark.gpu
SIG = 0.15


@contextlib.contextmanager
def options(**kw):
    from difficp_amd import _lib
    old = {k: _lib.get_option(k) for k in kw}
    try:
        for k, v in kw.items():
            _lib.set_option(k, v)
        yield
    finally:
        for k, v in old.items():
            _lib.set_option(k, v)


def _case(N, M, D, seed, dev):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(N, D, generator=g, dtype=torch.float64)
    q = torch.rand(M, D, generator=g, dtype=torch.float64)
    p = 0.02 * torch.randn(M, D, generator=g, dtype=torch.float64)
    a = torch.randn(N, D, generator=g, dtype=torch.float64)
    return [t.to(dev) for t in (x, q, p, a)]


PATHS = {"packed": dict(red_alg=0, ext_alg=1), "generic": dict(red_alg=0, ext_alg=0),
         "centred": dict(red_alg=2, ext_alg=1)}
SHAPES = [(1, 1), (7, 300), (513, 129), (3000, 2000), (20000, 700), (700, 20000)]


@pytest.mark.parametrize("path", sorted(PATHS))
@pytest.mark.parametrize("N,M", SHAPES)
@pytest.mark.parametrize("D", [2, 3])
@pytest.mark.parametrize("eta", [0.0, 2e-3])
def test_ext_fwd_paths(dev, path, N, M, D, eta):
    from difficp_amd import _lib
    x, q, p, _ = _case(N, M, D, N * 7 + M + D, dev)
    with options(**PATHS[path]):
        vx, gx = _lib.ode_ext_fwd(x.float(), q.float(), p.float(), SIG, eta, True)
        vx2, none = _lib.ode_ext_fwd(x.float(), q.float(), p.float(), SIG, eta, False)
    # the float64 reference sees the float32-rounded inputs
    v64, g64 = F.ext_terms(x.float().double(), q.float().double(), p.float().double(), SIG, eta)
    assert rel_err(vx, v64) < 1e-5
    assert rel_err(gx, g64) < 1e-5
    assert none is None and rel_err(vx2, v64) < 1e-5


@pytest.mark.parametrize("path", ["packed", "generic"])
@pytest.mark.parametrize("N,M", SHAPES)
@pytest.mark.parametrize("D", [2, 3])
@pytest.mark.parametrize("gam", [None, 0.41])
def test_ext_bwd_paths(dev, path, N, M, D, gam):
    """gx, and gq / gp ACCUMULATED into the caller's buffers (the adjoint adds them to the
    running cotangents)."""
    from difficp_amd import _lib
    x, q, p, a = _case(N, M, D, N * 11 + M + D, dev)
    xf, qf, pf, af = (t.float() for t in (x, q, p, a))
    gq0 = torch.randn(M, D, device=dev)
    gp0 = torch.randn(M, D, device=dev)
    gq, gp = gq0.clone(), gp0.clone()
    gd = None if gam is None else torch.full((1,), gam, device=dev)
    with options(**PATHS[path]):
        gx = _lib.ode_ext_bwd(xf, qf, pf, af, gd, SIG, 0.0, gq, gp)
    allx = torch.arange(N, device=dev)
    allq = torch.arange(M, device=dev)
    gx64, gq64, gp64 = F.ext_vjp_subset(xf.double(), qf.double(), pf.double(), af.double(),
                                        0.0 if gam is None else gam, allx, allq, SIG, 0.0)
    assert rel_err(gx, gx64) < 2e-5
    assert rel_err(gq.double() - gq0.double(), gq64) < 2e-5
    assert rel_err(gp.double() - gp0.double(), gp64) < 2e-5


def test_ext_packed_default_and_deterministic(dev):
    """ext_alg 1 is the default; two launches give the same bits."""
    from difficp_amd import _lib
    assert _lib.get_option("ext_alg") == 1
    x, q, p, a = (t.float() for t in _case(5000, 3000, 3, 5, dev))
    r1 = _lib.ode_ext_fwd(x, q, p, SIG, 0.0, True)
    r2 = _lib.ode_ext_fwd(x, q, p, SIG, 0.0, True)
    assert all(torch.equal(u, v) for u, v in zip(r1, r2))
    gq, gp = torch.zeros_like(q), torch.zeros_like(q)
    gq2, gp2 = torch.zeros_like(q), torch.zeros_like(q)
    gd = torch.full((1,), 0.3, device=dev)
    g1 = _lib.ode_ext_bwd(x, q, p, a, gd, SIG, 0.0, gq, gp)
    g2 = _lib.ode_ext_bwd(x, q, p, a, gd, SIG, 0.0, gq2, gp2)
    assert torch.equal(g1, g2) and torch.equal(gq, gq2) and torch.equal(gp, gp2)


@pytest.mark.parametrize("path", sorted(PATHS))
@pytest.mark.parametrize("N,M", SHAPES)
@pytest.mark.parametrize("D", [2, 3])
def test_kred_paths(dev, path, N, M, D):
    """KRed (kernel.py:138, :186-187) on the packed scaled-coordinate kernel (ext_alg 1 below the
    centred sizes), the generic kernel and the centred one."""
    from difficp_amd import _lib
    x, y, b, _ = _case(N, M, D, N * 13 + M + D, dev)
    xf, yf, bf = x.float(), y.float(), b.float()
    with options(**PATHS[path]):
        out = _lib.gauss_red(_lib.KRED, xf, yf, SIG, b=bf)
    ref, _ = F.ext_terms(xf.double(), yf.double(), bf.double(), SIG, 0.0)
    assert rel_err(out, ref) < 1e-5


@pytest.mark.parametrize("path", ["packed", "generic"])
def test_empty_support_and_points(dev, path):
    """No support points: v(x) = 0, divergence rows 0, gx = 0; no external points: empty gx and
    the accumulators untouched (LDDMM.py:111-112, 131-132)."""
    from difficp_amd import _lib
    x = torch.rand(37, 3, device=dev)
    a = torch.randn(37, 3, device=dev)
    q0 = torch.empty(0, 3, device=dev)
    gd = torch.full((1,), 0.3, device=dev)
    with options(**PATHS[path]):
        vx, gx = _lib.ode_ext_fwd(x, q0, q0, SIG, 0.0, True)
        assert vx.shape == (37, 3) and not vx.abs().any() and not gx.abs().any()
        gxb = _lib.ode_ext_bwd(x, q0, q0, a, gd, SIG, 0.0, torch.empty(0, 3, device=dev),
                               torch.empty(0, 3, device=dev))
        assert gxb.shape == (37, 3) and not gxb.abs().any()
        kr = _lib.gauss_red(_lib.KRED, x, q0, SIG, b=q0)
        assert kr.shape == (37, 3) and not kr.abs().any()
        q = torch.rand(11, 3, device=dev)
        gq, gp = torch.ones(11, 3, device=dev), torch.ones(11, 3, device=dev)
        e = torch.empty(0, 3, device=dev)
        gxe = _lib.ode_ext_bwd(e, q, q, e, gd, SIG, 0.0, gq, gp)
        assert gxe.shape == (0, 3) and bool((gq == 1).all()) and bool((gp == 1).all())
