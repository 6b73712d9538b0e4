"""Pair-once centred sums for x = y (csrc/sym_cx.hpp: Morton-sorted 256-point groups, each
unordered pair evaluated once and scattered to both rows) behind dicp_gauss_red_f32 (KBase,
KRedScal, KRed; kernel.py:131-138 / :178-187 with the rows equal to the columns, as
LDDMMModel.v(q, q, p) and the Hamiltonian call KRed, LDDMM.py:114, :151).

Parity against the float64 oracle (1e-5 norm-wise) with the path forced on
(sym_red 2), with 4 and 8 rows per lane (sym_red_rows; 256- / 512-point groups), at ragged
sizes (1 point, a partial group, group boundaries, a partial quad),
compact and wide clouds (every group in the difference form) and clouds far from the origin;
against the ordered centred kernel; bitwise run-to-run determinism; the automatic rule takes
it for the north_star's 100k x 100k sum only when the rows are the columns."""
import contextlib

import pytest
import torch

from conftest import rel_err
from oracle import torch_ref as R

pytestmark = pytest.mark.gpu


@contextlib.contextmanager
def opts(**kv):
    from difficp_amd import _lib
    old = {k: _lib.get_option(k) for k in kv}
    for k, v in kv.items():
        _lib.set_option(k, v)
    try:
        yield
    finally:
        for k, v in old.items():
            _lib.set_option(k, v)


def _ops(L, x, b, d, s):
    return {"KBase": L.gauss_red(L.KBASE, x, x, s), "KRedScal": L.gauss_red(L.KREDSCAL, x, x, s, b=d),
            "KRed": L.gauss_red(L.KRED, x, x, s, b=b)}


@pytest.mark.parametrize("rows", [4, 8])
@pytest.mark.parametrize("D", [2, 3])
@pytest.mark.parametrize("M,sig,ext,off", [(1, 0.1, 1.0, 0.0), (77, 0.1, 1.0, 0.0), (256, 0.2, 1.0, 0.0),
                                           (257, 0.05, 1.0, 0.0), (1023, 0.1, 1.0, 0.0), (1025, 0.1, 1.0, 0.0),
                                           (5000, 0.05, 1.0, 0.0), (4097, 0.1, 40.0, 0.0),
                                           (6000, 0.1, 3.0, 100.0), (9000, 1.0, 1.0, 0.0)])
def test_sym_reductions_match_oracle(dev, D, M, sig, ext, off, rows):
    from difficp_amd import _lib as L
    g = torch.Generator().manual_seed(M * 3 + D)
    r32 = lambda t: t.float().double()      # the float64 reference sees the float32 inputs
    x = r32(off + ext * torch.rand(M, D, generator=g, dtype=torch.float64))
    b = r32(torch.randn(M, D, generator=g, dtype=torch.float64))
    d = r32(torch.randn(M, generator=g, dtype=torch.float64))
    f = lambda t: t.float().to(dev).contiguous()
    ref = {"KBase": R.KBase(x, x, sig), "KRedScal": R.KRedScal(x, x, d, sig), "KRed": R.KRed(x, x, b, sig)}
    xd, bd, dd = f(x), f(b), f(d)
    with opts(sym_red=2, sym_red_rows=rows):
        sy = _ops(L, xd, bd, dd, sig)
        sy2 = _ops(L, xd, bd, dd, sig)
    with opts(sym_red=0, red_alg=2):
        cx = _ops(L, xd, bd, dd, sig)
    for k in ref:
        assert rel_err(sy[k].cpu(), ref[k]) < 1e-5, (k, rel_err(sy[k].cpu(), ref[k]))
        assert torch.equal(sy[k], sy2[k]), k                          # deterministic
        assert rel_err(sy[k].cpu(), cx[k].cpu()) < 1e-5, k


@pytest.mark.parametrize("rows", [4, 8])
@pytest.mark.parametrize("rho", [0, 150, 400])
def test_sym_wide_and_compact_groups_agree(dev, rho, rows):
    """rho_max 0 (every group pair in the difference form), the default 1.5, the cap 4: all
    within the criterion on a 3D cloud ~30 sigma wide."""
    from difficp_amd import _lib as L
    g = torch.Generator().manual_seed(5)
    M, sig = 20000, 0.1
    x = 3.0 * torch.rand(M, 3, generator=g, dtype=torch.float64)
    b = torch.randn(M, 3, generator=g, dtype=torch.float64)
    ref = R.KRed(x.float().double(), x.float().double(), b.float().double(), sig)
    f = lambda t: t.float().to(dev).contiguous()
    with opts(sym_red=2, cx_rho_x100=rho, sym_red_rows=rows):
        out = L.gauss_red(L.KRED, f(x), f(x), sig, b=f(b))
    assert rel_err(out.cpu(), ref) < 1e-5, (rho, rel_err(out.cpu(), ref))


def test_sym_automatic_rule(dev):
    """sym_red 1 (default): x is y at the north_star's size takes the pair-once form -- its
    result equals the forced form bitwise; a copy of x (x is not y) takes the ordered one."""
    from difficp_amd import _lib as L
    g = torch.Generator().manual_seed(9)
    M = 100000
    x = torch.rand(M, 3, generator=g).to(dev)
    b = (0.01 * torch.randn(M, 3, generator=g)).to(dev)
    assert L.get_option("sym_red") == 1
    auto = L.gauss_red(L.KRED, x, x, 0.1, b=b)
    with opts(sym_red=2):
        forced = L.gauss_red(L.KRED, x, x, 0.1, b=b)
    assert torch.equal(auto, forced)
    xc = x.clone()
    other = L.gauss_red(L.KRED, x, xc, 0.1, b=b)
    with opts(sym_red=0):
        ordered = L.gauss_red(L.KRED, x, x, 0.1, b=b)
    assert torch.equal(other, ordered)
    assert rel_err(auto, ordered) < 2e-6
