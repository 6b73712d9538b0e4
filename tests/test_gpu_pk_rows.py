"""Row pairs per thread of the packed fused forward (packed.hpp rowred_pk_kernel<Op, RP>,
dicp_set_option "pk_rp"): the 4-row form (RP = 2, automatic for the eta = 0 forward from 32k
rows) forced at ragged sizes, row slices (the row split) and every output variant (v / mG / g,
the divergence rows zs, the mG-less last step, the Hamiltonian rows), against the 2-row form
(1e-6: fp32 summation order of the column splits only, bitwise when both pick the same splits)
and against the fp64 oracle's ODE (2e-5, the tolerance of tests/test_gpu_kernels.py)."""
import pytest
import torch

from conftest import rel_err
from oracle import torch_ref as R

pytestmark = pytest.mark.gpu

SIG = 0.15


def _lib():
    from difficp_amd import _lib
    return _lib


class _rp:
    def __init__(self, v):
        self.v = v

    def __enter__(self):
        L = _lib()
        self.old = L.get_option("pk_rp")
        L.set_option("pk_rp", self.v)

    def __exit__(self, *a):
        _lib().set_option("pk_rp", self.old)


def _case(M, D, seed):
    g = torch.Generator().manual_seed(seed)
    q = torch.rand(M, D, generator=g, dtype=torch.float64)
    p = 0.1 * torch.randn(M, D, generator=g, dtype=torch.float64)
    return q, p


@pytest.mark.parametrize("M,D", [(1, 3), (257, 3), (1023, 2), (1025, 3), (5000, 3), (33001, 3)])
def test_forward_four_rows_vs_two_rows(dev, M, D):
    L = _lib()
    q, p = _case(M, D, 7 * M + D)
    qf, pf = q.float().to(dev), p.float().to(dev)
    outs = {}
    for rp in (1, 2):
        with _rp(rp):
            zs = torch.empty(M, D, device=dev)
            o = {"fwd": L.ode_self_fwd(qf, pf, SIG, 0.0, True),
                 "fwd_h": L.ode_self_fwd(qf, pf, SIG, 0.0, True, want_h=True),
                 "step_zs": L.euler_step(qf, pf, SIG, 0.0, 0.1, True, zs_out=zs) + (zs,),
                 "step_nog": L.euler_step(qf, pf, SIG, 0.0, 0.1, True, want_p=False)}
            torch.cuda.synchronize()
            outs[rp] = o
    for k in outs[1]:
        for a, b in zip(outs[2][k], outs[1][k]):
            if a is None or b is None:
                assert a is None and b is None, k
                continue
            assert rel_err(a.cpu(), b.cpu()) < 1e-6, (k, rel_err(a.cpu(), b.cpu()))
    if M > 5000:   # the dense oracle holds M x M x D float64 pairs
        return
    # the 4-row form against the fp64 oracle's ODE (v, -G, divergence), tolerance as
    # tests/test_gpu_kernels.py: max(2e-5, 2 x the float32 oracle's own deviation)
    m = R.LDDMM(SIG, D, 50.0, False, True)
    v64, mG64, c64 = m.ODE(q, p, torch.zeros(1, dtype=torch.float64))
    m32 = R.LDDMM(SIG, D, 50.0, False, True)
    v32, mG32, c32 = m32.ODE(q.float(), p.float(), torch.zeros(1))
    tol = lambda r64, r32: max(2e-5, 2 * rel_err(r32, r64))
    v, mG, g, _ = outs[2]["fwd"]
    assert rel_err(v.cpu(), v64) <= tol(v64, v32)
    assert rel_err(mG.cpu(), mG64) <= tol(mG64, mG32)
    assert rel_err(g.sum().cpu(), c64) <= tol(c64, c32)


@pytest.mark.parametrize("M,W", [(33001, 2), (40000, 3), (70001, 2)])
def test_forward_four_rows_row_slices(dev, M, W):
    """Row slices of the forward under the automatic choice (the full pass >= 32k rows runs 4
    rows per thread; slices below 32k rows 2, the 35k-row slices of 70001 / 2 also 4)
    concatenate to the full pass within fp32 summation order."""
    L = _lib()
    q, p = _case(M, 3, M + W)
    qf, pf = q.float().to(dev), p.float().to(dev)
    qn, pn, g = L.euler_step(qf, pf, SIG, 0.0, 0.1, True)
    per = -(-M // W)
    parts = []
    for r in range(W):
        r0 = min(per * r, M)
        n = min(per, M - r0)
        parts.append(L.euler_step_rows(qf, pf, r0, n, SIG, 0.0, 0.1, True))
    qs = torch.cat([t[0] for t in parts])
    ps = torch.cat([t[1] for t in parts])
    gs = torch.cat([t[2] for t in parts])
    assert rel_err(qs.cpu(), qn.cpu()) < 1e-6
    assert rel_err(ps.cpu(), pn.cpu()) < 1e-6
    assert rel_err(gs.cpu(), g.cpu()) < 1e-5


@pytest.mark.parametrize("N,M,D", [(1, 5, 3), (1025, 700, 3), (3001, 2049, 2), (20000, 9000, 3)])
@pytest.mark.parametrize("eta", [0.0, 0.02])
def test_external_point_passes_four_rows_vs_two_rows(dev, N, M, D, eta):
    """The packed external-point forward / VJP and the packed KRed (ext_pk.hpp) with 4 rows per
    thread forced, against 2 rows: fp32 summation order of the column splits only."""
    L = _lib()
    g = torch.Generator().manual_seed(N + M + D)
    x = torch.rand(N, D, generator=g).to(dev)
    q = torch.rand(M, D, generator=g).to(dev)
    p = (0.1 * torch.randn(M, D, generator=g)).to(dev)
    gvx = torch.randn(N, D, generator=g).to(dev)
    gdiv = torch.ones(1, device=dev)
    old = L.get_option("red_alg")
    L.set_option("red_alg", 0)   # the packed kernels at every size
    try:
        res = {}
        for rp in (1, 2):
            with _rp(rp):
                gq = torch.zeros(M, D, device=dev)
                gp = torch.zeros(M, D, device=dev)
                vx, gx = L.ode_ext_fwd(x, q, p, SIG, eta, True)
                gxb = L.ode_ext_bwd(x, q, p, gvx, gdiv, SIG, eta, gq, gp)
                kr = L.gauss_red(L.KRED, x, q, SIG, b=p)
                torch.cuda.synchronize()
                res[rp] = (vx, gx, gxb, gq, gp, kr)
    finally:
        L.set_option("red_alg", old)
    for a, b in zip(res[2], res[1]):
        assert rel_err(a.cpu(), b.cpu()) < 1e-6, rel_err(a.cpu(), b.cpu())


# --- the symmetric VJP with 4 rows per lane (lddmm_sym_pk.hpp sym_pk4_body, "sym_rp") ---

class _srp(_rp):
    def __enter__(self):
        L = _lib()
        self.old = L.get_option("sym_rp")
        L.set_option("sym_rp", self.v)

    def __exit__(self, *a):
        _lib().set_option("sym_rp", self.old)


def _vjp_variants(L, qf, pf, a, b, gd, zs, raw):
    """Every launch form of the packed eta = 0 VJP: plain (with / without the divergence
    cotangent), the adjoint steps reusing the divergence rows (full, zero momentum cotangent,
    gp only) and the pair-subset parts of a 3-way row split (summed)."""
    with L.coord_mode(raw):
        o = {"bwd": L.ode_self_bwd(qf, pf, a, b, gd, SIG, 0.0),
             "bwd_nodiv": L.ode_self_bwd(qf, pf, a, b, None, SIG, 0.0),
             "adj_zs": L.euler_adjoint_step(qf, pf, a, b, gd, SIG, 0.0, 0.1, zs=zs),
             "adj_b0": L.euler_adjoint_step(qf, pf, a, None, gd, SIG, 0.0, 0.1, zs=zs),
             "adj_gp": (L.euler_adjoint_step(qf, pf, a, b, gd, SIG, 0.0, 0.1, want_lq=False, zs=zs)[1],)}
        sq, sp = torch.zeros_like(qf), torch.zeros_like(qf)
        for r in range(3):
            pq, pp = L.ode_self_bwd_part(qf, pf, a, b, gd, SIG, 0.0, r, 3)
            sq += pq
            sp += pp
        o["parts3"] = (sq, sp)
    torch.cuda.synchronize()
    return o


@pytest.mark.parametrize("M,D", [(1, 3), (129, 2), (257, 3), (1023, 2), (1025, 3), (4700, 3), (33001, 3)])
@pytest.mark.parametrize("raw", [False, True])
def test_vjp_four_rows_vs_two_rows(dev, M, D, raw):
    """The packed symmetric VJP forced to 4 rows per lane (256-point groups, packed column sums
    over the 4 rows) against 2 rows at ragged sizes, every launch variant, scaled and raw
    coordinates: fp32 summation order only (2e-6); and against float64 autograd of the
    oracle's ODE (2e-5, tests/test_gpu_kernels.py::test_ode_self_bwd's tolerance)."""
    L = _lib()
    g = torch.Generator().manual_seed(11 * M + D)
    q = torch.rand(M, D, generator=g, dtype=torch.float64)
    p = 0.1 * torch.randn(M, D, generator=g, dtype=torch.float64)
    a = torch.randn(M, D, generator=g, dtype=torch.float64)
    b = torch.randn(M, D, generator=g, dtype=torch.float64)
    gam = torch.randn(1, generator=g, dtype=torch.float64)
    f = lambda t: t.float().to(dev)
    qf, pf, af, bf, gd = f(q), f(p), f(a), f(b), f(gam)
    zs = torch.empty(M, D, device=dev)
    L.euler_step(qf, pf, SIG, 0.0, 0.1, True, zs_out=zs)
    outs = {}
    for rp in (1, 2):
        with _srp(rp):
            outs[rp] = _vjp_variants(L, qf, pf, af, bf, gd, zs, raw)
    for k in outs[1]:
        for x4, x2 in zip(outs[2][k], outs[1][k]):
            assert rel_err(x4.cpu(), x2.cpu()) < 2e-6, (k, rel_err(x4.cpu(), x2.cpu()))
    # determinism: the 4-row kernel is bitwise reproducible run to run
    with _srp(2):
        again = _vjp_variants(L, qf, pf, af, bf, gd, zs, raw)
    for k in again:
        for x, y in zip(again[k], outs[2][k]):
            assert torch.equal(x, y), k
    if M > 5000:
        return
    qq, pp = q.clone().requires_grad_(True), p.clone().requires_grad_(True)
    m = R.LDDMM(SIG, D, 50.0, False, True)
    v, mG, c = m.ODE(qq, pp, torch.zeros(1, dtype=torch.float64))
    gq64, gp64 = torch.autograd.grad((a * v).sum() + (b * mG).sum() + (gam * c).sum(), (qq, pp))
    gq, gp = outs[2]["bwd"]
    assert rel_err(gq.cpu(), gq64) < 2e-5 and rel_err(gp.cpu(), gp64) < 2e-5
    gq, gp = outs[2]["parts3"]
    assert rel_err(gq.cpu(), gq64) < 2e-5 and rel_err(gp.cpu(), gp64) < 2e-5


def test_vjp_rows_automatic_rule(dev):
    """sym_rp 0 (automatic) picks 4 rows for whole passes from 40k points and 2 below (row-split
    parts: from 64k and 2e9 pairs per part): the automatic result equals the forced form
    bitwise on each side of the threshold (50k: the 4-row form with L = 1)."""
    L = _lib()
    for M, want in ((20000, 1), (50000, 2), (100000, 2)):
        g = torch.Generator().manual_seed(M)
        qf = torch.rand(M, 3, generator=g).to(dev)
        pf = (0.01 * torch.randn(M, 3, generator=g)).to(dev)
        a = torch.randn(M, 3, generator=g).to(dev)
        res = {}
        for rp in (0, want):
            with _srp(rp):
                res[rp] = L.ode_self_bwd(qf, pf, a, a, None, SIG, 0.0)
        assert torch.equal(res[0][0], res[want][0]) and torch.equal(res[0][1], res[want][1]), M


# --- the symmetric pair-once forward with 4 rows per lane (fwd_alg 5, SymFwdPk4) ---

class _falg(_rp):
    def __enter__(self):
        L = _lib()
        self.old = L.get_option("fwd_alg")
        L.set_option("fwd_alg", self.v)

    def __exit__(self, *a):
        _lib().set_option("fwd_alg", self.old)


@pytest.mark.parametrize("M,D", [(1, 3), (257, 3), (1023, 2), (1025, 3), (5000, 3), (33001, 3), (70001, 3)])
def test_forward_sym4_vs_ordered(dev, M, D):
    """fwd_alg 5 (each unordered pair once, 4 rows per lane, column sums rotated by DPP) against
    the packed ordered forward (fwd_alg 6) for every forward form the shooting runs -- plain,
    with the Hamiltonian rows, the Euler step writing the divergence rows, the mG-less last step
    -- within fp32 summation order (2e-6; the divergence rows 1e-5), bitwise run to run, and
    against the fp64 oracle's ODE (2e-5)."""
    L = _lib()
    q, p = _case(M, D, 3 * M + D)
    qf, pf = q.float().to(dev), p.float().to(dev)
    outs = {}
    for alg in (6, 5, 5):
        with _falg(alg):
            zs = torch.empty(M, D, device=dev)
            zs0 = torch.empty(M, D, device=dev)
            o = {"fwd": L.ode_self_fwd(qf, pf, SIG, 0.0, True),
                 "fwd_h": L.ode_self_fwd(qf, pf, SIG, 0.0, True, want_h=True),
                 "first_zs": L.ode_self_fwd(qf, pf, SIG, 0.0, True, zs_out=zs0)[:3] + (zs0,),
                 "step_zs": L.euler_step(qf, pf, SIG, 0.0, 0.1, True, zs_out=zs) + (zs,),
                 "step_nog": L.euler_step(qf, pf, SIG, 0.0, 0.1, True, want_p=False)}
            torch.cuda.synchronize()
            if alg in outs:
                for k in o:
                    for a, b in zip(o[k], outs[alg][k]):
                        assert (a is None and b is None) or torch.equal(a, b), k
            outs[alg] = o
    for k in outs[6]:
        for i, (a, b) in enumerate(zip(outs[5][k], outs[6][k])):
            if a is None or b is None:
                assert a is None and b is None, k
                continue
            tol = 1e-5 if (k in ("step_zs", "first_zs") and i == 3) else 2e-6
            assert rel_err(a.cpu(), b.cpu()) < tol, (k, i, rel_err(a.cpu(), b.cpu()))
    if M > 5000:
        return
    m = R.LDDMM(SIG, D, 50.0, False, True)
    v64, mG64, c64 = m.ODE(q, p, torch.zeros(1, dtype=torch.float64))
    v, mG, g, h = outs[5]["fwd_h"]
    assert rel_err(v.cpu(), v64) < 2e-5 and rel_err(mG.cpu(), mG64) < 2e-5
    assert abs(float(g.double().sum().cpu() - c64.sum())) <= 2e-5 * max(1.0, float(c64.abs().sum()))


def test_forward_automatic_rule(dev):
    """fwd_alg 2 (default) runs the ordered rows below 20k points and the symmetric 4-row pass
    from 20k on (whole passes; L = 1 at 20k-50k, 4 at 100k): bitwise fwd_alg 6 / fwd_alg 5 on
    each side."""
    L = _lib()
    for M, want in ((12000, 6), (20000, 5), (50000, 5), (100000, 5)):
        q, p = _case(M, 3, M)
        qf, pf = q.float().to(dev), p.float().to(dev)
        res = {}
        for alg in (2, want):
            with _falg(alg):
                zs = torch.empty(M, 3, device=dev)
                res[alg] = L.euler_step(qf, pf, SIG, 0.0, 0.1, True, zs_out=zs) + (zs,)
        for a, b in zip(res[2], res[want]):
            assert torch.equal(a, b), M
