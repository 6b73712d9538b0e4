"""Centred-expansion reductions (csrc/centred.hpp: Morton-sorted 64-column sub-tiles, expanded
exponent 2X.Y - |Y|^2 - |X|^2, difference-form fallback for wide sub-tiles) behind
dicp_gauss_red_f32 (KBase, KRedScal, KRed, GradKRed) and dicp_lddmm_ode_ext_fwd_f32.

Parity against the float64 oracle (SURVEY 8c criterion: 1e-5 norm-wise) with the path forced
on (red_alg 2) and against the generic skeleton (red_alg 0), on compact clouds, clouds far
wider than sigma (every sub-tile takes the fallback), ragged sizes (N not a multiple of 64,
N < 64, M = 1), 2D and 3D; full size (the north_star's 100k x 100k kernel sum) on sampled
rows; bitwise run-to-run determinism."""
import contextlib

import pytest
import torch

import fullsize_ref as F
from conftest import rel_err
from oracle import torch_ref as R

pytestmark = pytest.mark.gpu


@contextlib.contextmanager
def red_alg(v, rho=None):
    from difficp_amd import _lib
    old, old_rho = _lib.get_option("red_alg"), _lib.get_option("cx_rho_x100")
    _lib.set_option("red_alg", v)
    if rho is not None:
        _lib.set_option("cx_rho_x100", rho)
    try:
        yield
    finally:
        _lib.set_option("red_alg", old)
        _lib.set_option("cx_rho_x100", old_rho)


def _ops(L, x, y, b, d, s):
    return {"KBase": L.gauss_red(L.KBASE, x, y, s), "KRedScal": L.gauss_red(L.KREDSCAL, x, y, s, b=d),
            "KRed": L.gauss_red(L.KRED, x, y, s, b=b), "GradKRed": L.gauss_red(L.GRADK, x, y, s)}


def _ref(x, y, b, d, s):
    return {"KBase": R.KBase(x, y, s), "KRedScal": R.KRedScal(x, y, d, s), "KRed": R.KRed(x, y, b, s),
            "GradKRed": R.GradKRed(x, y, s)}


@pytest.mark.parametrize("D", [2, 3])
@pytest.mark.parametrize("M,N,sig,ext", [(1000, 700, 0.05, 1.0), (3000, 5000, 0.1, 1.0), (2000, 3000, 0.2, 1.0),
                                         (1500, 2500, 1.0, 1.0), (2000, 2000, 0.05, 50.0), (1, 777, 0.1, 1.0),
                                         (900, 63, 0.1, 1.0), (700, 1, 0.3, 1.0), (4097, 4099, 0.08, 3.0)])
def test_centred_reductions_match_oracle(dev, D, M, N, sig, ext):
    from difficp_amd import _lib as L
    g = torch.Generator().manual_seed(M * 7 + N + D)
    # the float64 reference sees the float32 inputs the kernels get (identical inputs)
    r32 = lambda t: t.float().double()
    x = r32(ext * torch.rand(M, D, generator=g, dtype=torch.float64))
    y = r32(ext * torch.rand(N, D, generator=g, dtype=torch.float64))
    b = r32(torch.randn(N, D, generator=g, dtype=torch.float64))
    d = r32(torch.randn(N, generator=g, dtype=torch.float64))
    f = lambda t: t.float().to(dev).contiguous()
    ref = _ref(x, y, b, d, sig)
    with red_alg(2):
        cx = _ops(L, f(x), f(y), f(b), f(d), sig)
        cx2 = _ops(L, f(x), f(y), f(b), f(d), sig)
    with red_alg(0):
        gen = _ops(L, f(x), f(y), f(b), f(d), sig)
    for k in ref:
        if float(ref[k].norm()) < 1e-30:    # below float32 range: nothing to compare
            continue
        assert rel_err(cx[k].cpu(), ref[k]) < 1e-5, (k, rel_err(cx[k].cpu(), ref[k]))
        assert torch.equal(cx[k], cx2[k]), k                        # deterministic
        assert rel_err(cx[k].cpu(), gen[k].cpu()) < 1e-5, k


@pytest.mark.parametrize("D", [2, 3])
def test_centred_fallback_and_compact_agree(dev, D):
    """rho_max 0 (every sub-tile in the difference form) vs the default vs the largest rho_max
    the factored exponent accepts (4 scaled units, kCxRhoCap): all within the criterion on a
    cloud whose extent is ~30 sigma, so the expanded form's cancellation is exercised."""
    from difficp_amd import _lib as L
    g = torch.Generator().manual_seed(3 + D)
    M, N, sig = 6000, 9000, 0.1
    x = 3.0 * torch.rand(M, D, generator=g, dtype=torch.float64)
    y = 3.0 * torch.rand(N, D, generator=g, dtype=torch.float64)
    b = torch.randn(N, D, generator=g, dtype=torch.float64)
    f = lambda t: t.float().to(dev).contiguous()
    ref = R.KRed(x, y, b, sig)
    for rho in (0, 150, 100000):       # 100000 is capped at 400 by the library
        with red_alg(2, rho):
            out = L.gauss_red(L.KRED, f(x), f(y), sig, b=f(b))
        assert rel_err(out.cpu(), ref) < 1e-5, (rho, rel_err(out.cpu(), ref))


@pytest.mark.parametrize("eta", [0.0, 0.02])
@pytest.mark.parametrize("div", [False, True])
@pytest.mark.parametrize("D", [2, 3])
def test_centred_ext_fwd_matches_oracle(dev, eta, div, D):
    from difficp_amd import _lib as L
    g = torch.Generator().manual_seed(11 + D)
    N, M, sig = 3000, 2500, 0.12
    x = torch.rand(N, D, generator=g, dtype=torch.float64)
    q = torch.rand(M, D, generator=g, dtype=torch.float64)
    p = 0.1 * torch.randn(M, D, generator=g, dtype=torch.float64)
    f = lambda t: t.float().to(dev).contiguous()
    v64, g64 = F.ext_terms(x, q, p, sig, eta)
    with red_alg(2):
        vx, gx = L.ode_ext_fwd(f(x), f(q), f(p), sig, eta, div)
    assert rel_err(vx.cpu(), v64) < 1e-5
    if div:
        assert rel_err(gx.cpu(), g64) < 1e-5


def test_kernel_sum_100k_fullsize(dev):
    """The north_star's 100k x 100k 3D kernel sum (KRed, x = y, sigma 0.1, the bench's probe)
    on the default (automatic) path: 192 sampled rows against float64 sums over all 100k
    columns; GradKRed likewise."""
    from difficp_amd import _lib as L
    g = torch.Generator().manual_seed(1)
    M = 100000
    x = torch.rand(M, 3, generator=g, dtype=torch.float64)
    b = 0.01 * torch.randn(M, 3, generator=g, dtype=torch.float64)
    sub = torch.randperm(M, generator=g)[:192]
    xd, bd = x.float().to(dev), b.float().to(dev)
    out = L.gauss_red(L.KRED, xd, xd, 0.1, b=bd)
    assert L.get_option("red_alg") == 1
    xg, bg = x.to(dev), b.to(dev)
    s = sub.to(dev)
    ref = torch.zeros(192, 3, dtype=torch.float64, device=dev)
    gk = torch.zeros(192, 3, dtype=torch.float64, device=dev)
    for j0 in range(0, M, 8192):
        z = xg[s][:, None] - xg[None, j0:j0 + 8192]
        K = torch.exp(-(z * z).sum(-1) / (2 * 0.01))
        ref += K @ bg[j0:j0 + 8192]
        gk += -(K[..., None] * z).sum(1) / 0.01
    assert rel_err(out[s], ref) < 1e-5
    out2 = L.gauss_red(L.KRED, xd, xd, 0.1, b=bd)
    assert torch.equal(out, out2)
    gout = L.gauss_red(L.GRADK, xd, xd, 0.1)
    assert rel_err(gout[s], gk) < 1e-5
