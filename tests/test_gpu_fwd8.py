"""The symmetric forward with 8 or 6 rows per lane (lddmm_sym_pk.hpp SymFwdPkN /
sym_fwd_pkn_kernel, 512- / 384-point groups; dicp_set_option "sym_fwd_rows" 8 / 6 forces it)
at ragged sizes (a partial group, group and quad boundaries) and every output variant of a
whole pass (v / mG / g, the Hamiltonian rows, the divergence rows zs of the Euler step),
against the 4-row symmetric form (1e-6: fp32 summation order only) and the fp64 oracle's
ODE (max(2e-5, 2 x the float32 oracle's own deviation), as tests/test_gpu_pk_rows.py);
bitwise run-to-run determinism."""
import pytest
import torch

from conftest import rel_err
from oracle import torch_ref as R

pytestmark = pytest.mark.gpu

SIG = 0.15


class _rows:
    def __init__(self, v):
        self.v = v

    def __enter__(self):
        from difficp_amd import _lib
        self.old = (_lib.get_option("sym_fwd_rows"), _lib.get_option("fwd_alg"))
        _lib.set_option("fwd_alg", 5)          # the symmetric forward at every size
        _lib.set_option("sym_fwd_rows", self.v)

    def __exit__(self, *a):
        from difficp_amd import _lib
        _lib.set_option("sym_fwd_rows", self.old[0])
        _lib.set_option("fwd_alg", self.old[1])


@pytest.mark.parametrize("wide", [8, 6])
@pytest.mark.parametrize("M,D", [(1, 3), (300, 2), (383, 3), (385, 2), (511, 3), (512, 3), (513, 2),
                                 (1537, 3), (2049, 3), (4100, 3), (33001, 3), (70001, 2)])
def test_forward_eight_rows(dev, M, D, wide):
    from difficp_amd import _lib as L
    g = torch.Generator().manual_seed(11 * M + D)
    q = torch.rand(M, D, generator=g, dtype=torch.float64)
    p = 0.1 * torch.randn(M, D, generator=g, dtype=torch.float64)
    qf, pf = q.float().to(dev), p.float().to(dev)
    outs = {}
    for rows in (4, wide, wide):
        with _rows(rows):
            zs = torch.empty(M, D, device=dev)
            o = {"fwd": L.ode_self_fwd(qf, pf, SIG, 0.0, True),
                 "fwd_nodiv": L.ode_self_fwd(qf, pf, SIG, 0.0, False),
                 "fwd_h": L.ode_self_fwd(qf, pf, SIG, 0.0, True, want_h=True),
                 "step_zs": L.euler_step(qf, pf, SIG, 0.0, 0.1, True, zs_out=zs) + (zs,)}
            torch.cuda.synchronize()
        if rows in outs:
            for k in o:                       # deterministic
                for a, b in zip(o[k], outs[rows][k]):
                    assert (a is None and b is None) or torch.equal(a, b), k
        outs[rows] = o
    for k in outs[4]:
        for a, b in zip(outs[wide][k], outs[4][k]):
            if a is None or b is None:
                assert a is None and b is None, k
                continue
            assert rel_err(a.cpu(), b.cpu()) < 1e-6, (k, rel_err(a.cpu(), b.cpu()))
    if M > 5000:   # the dense oracle holds M x M x D float64 pairs
        return
    m = R.LDDMM(SIG, D, 50.0, False, True)
    v64, mG64, c64 = m.ODE(q, p, torch.zeros(1, dtype=torch.float64))
    m32 = R.LDDMM(SIG, D, 50.0, False, True)
    v32, mG32, c32 = m32.ODE(q.float(), p.float(), torch.zeros(1))
    tol = lambda r64, r32: max(2e-5, 2 * rel_err(r32, r64))
    v, mG, gd, _ = outs[wide]["fwd"]
    assert rel_err(v.cpu(), v64) <= tol(v64, v32)
    assert rel_err(mG.cpu(), mG64) <= tol(mG64, mG32)
    assert rel_err(gd.sum().cpu(), c64) <= tol(c64, c32)


@pytest.mark.parametrize("M,rows", [(30000, 4), (100000, 6), (200000, 8)])
def test_forward_rows_automatic_rule(dev, M, rows):
    """The default (fwd_alg 2, sym_fwd_rows 0) takes 4 rows below 40k points, 6 from 40k (the
    north_star's 100k) and 8 from 180k for a whole pass: its result equals the form forced with
    that many rows bitwise."""
    from difficp_amd import _lib as L
    g = torch.Generator().manual_seed(5)
    q = torch.rand(M, 3, generator=g).to(dev)
    p = (0.01 * torch.randn(M, 3, generator=g)).to(dev)
    assert L.get_option("sym_fwd_rows") == 0 and L.get_option("fwd_alg") == 2
    auto = L.euler_step(q, p, 0.1, 0.0, 0.1, True)
    old = L.get_option("sym_fwd_rows")
    L.set_option("sym_fwd_rows", rows)
    try:
        forced = L.euler_step(q, p, 0.1, 0.0, 0.1, True)
    finally:
        L.set_option("sym_fwd_rows", old)
    for a, b in zip(auto, forced):
        assert torch.equal(a, b)
