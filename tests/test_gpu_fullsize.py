"""Parity at BASELINE full sizes (C2: 50k, the metric's 100k and C3: 200k 3D points,
sigma_LDDMM = 0.1, sigma_GMM = 0.05).

A full fp64 oracle at 50k x 50k is 2.5e9 pairs per operator -- too slow for a test -- so the
checks here are
  * row-subset parity: 192 random rows of each output, each a reduction over ALL the
    columns, against float64 torch formulas of the reference operators (the formulas are
    themselves checked against the oracle at small size, in the CPU test at the bottom);
  * size-independent properties: bitwise run-to-run determinism, invariance to the number of
    column splits, sum_c gamma_nc = 1 (column statistics add up to N and to sum_n x_n).
Tolerances: 1e-5 norm-wise relative, 2e-5 for the backward (two fp32 passes
deep), 1e-6 for split invariance (only the fp32 summation order differs).
"""
import math

import pytest
import torch

from conftest import rel_err
from oracle import torch_ref as R

M_FULL = 50000
SIG_L = 0.1
SIG_G = 0.05
NSUB = 192


def _points(M, seed):
    g = torch.Generator().manual_seed(seed)
    q = torch.rand(M, 3, generator=g, dtype=torch.float64)
    p = 0.01 * torch.randn(M, 3, generator=g, dtype=torch.float64)
    a = torch.randn(M, 3, generator=g, dtype=torch.float64)
    b = torch.randn(M, 3, generator=g, dtype=torch.float64)
    sub = torch.randperm(M, generator=g)[:NSUB]
    return q, p, a, b, sub


def _row_terms(qr, pr, qc, pc, sigma, chunk=4096):
    """v, mG, g of the rows (qr, pr) against the columns (qc, pc): LDDMM.py:100-138, 176-205
    (eta = 0): v = KRed, mG = -GenDKRed(q,q,p,p), g_i = p_i . GradKRed(q_i, q)."""
    v = torch.zeros_like(qr)
    mG = torch.zeros_like(qr)
    g = torch.zeros(qr.shape[0], dtype=qr.dtype)
    s2 = sigma * sigma
    for j0 in range(0, qc.shape[0], chunk):
        z = qr[:, None, :] - qc[None, j0:j0 + chunk, :]
        K = torch.exp(-(z * z).sum(-1) / (2 * s2))
        pcj = pc[j0:j0 + chunk]
        v = v + K @ pcj
        pp = pr @ pcj.T
        mG = mG + ((K * pp)[:, :, None] * z).sum(1) / s2
        g = g - (pr[:, None, :] * z * K[:, :, None]).sum((1, 2)) / s2
    return v, mG, g


def _bwd_subset(q, p, a, b, gam, sub, sigma):
    """d/d(q_i, p_i), i in sub, of L = sum_k a_k.v_k + b_k.mG_k + gam g_k over ALL rows k:
    row-side derivatives from the rows in `sub` (columns detached) plus column-side
    derivatives from all rows against the columns in `sub` (rows detached)."""
    qs = q[sub].clone().requires_grad_(True)
    ps = p[sub].clone().requires_grad_(True)
    v, mG, g = _row_terms(qs, ps, q, p, sigma)
    L = (a[sub] * v).sum() + (b[sub] * mG).sum() + gam * g.sum()
    for k0 in range(0, q.shape[0], 8192):
        sl = slice(k0, k0 + 8192)
        v, mG, g = _row_terms(q[sl], p[sl], qs, ps, sigma)
        L = L + (a[sl] * v).sum() + (b[sl] * mG).sum() + gam * g.sum()
    return torch.autograd.grad(L, (qs, ps))


def test_subset_formulas_match_oracle():
    """CPU: the row/column-subset formulas above equal the oracle's full computation."""
    q, p, a, b, _ = _points(300, 11)
    p = 10 * p
    sub = torch.tensor([0, 7, 150, 299])
    m = R.LDDMM(0.15, 3, 50.0, False, True)
    v64, mG64, c64 = m.ODE(q, p, torch.zeros(1, dtype=torch.float64))
    v, mG, g = _row_terms(q[sub], p[sub], q, p, 0.15)
    assert rel_err(v, v64[sub]) < 1e-12 and rel_err(mG, mG64[sub]) < 1e-12
    vall, mGall, gall = _row_terms(q, p, q, p, 0.15)
    assert abs(float(gall.sum() - c64.sum())) < 1e-10 * max(1.0, abs(float(c64.sum())))
    qq = q.clone().requires_grad_(True)
    pq = p.clone().requires_grad_(True)
    v, mG, c = m.ODE(qq, pq, torch.zeros(1, dtype=torch.float64))
    gam = 0.7
    gq, gp = torch.autograd.grad((a * v).sum() + (b * mG).sum() + gam * c.sum(), (qq, pq))
    gqs, gps = _bwd_subset(q, p, a, b, gam, sub, 0.15)
    assert rel_err(gqs, gq[sub]) < 1e-12 and rel_err(gps, gp[sub]) < 1e-12


@pytest.fixture(scope="module", params=[M_FULL, 100000, 200000], ids=["50k", "100k", "200k"])
def full(dev, request):
    q, p, a, b, sub = _points(request.param, 2024)
    f = lambda t: t.float().to(dev)
    return dict(q=q, p=p, a=a, b=b, sub=sub, qd=f(q), pd=f(p), ad=f(a), bd=f(b))


@pytest.mark.gpu
def test_fwd_fullsize_subset(full):
    from difficp_amd import _lib
    v, mG, g, h = _lib.ode_self_fwd(full["qd"], full["pd"], SIG_L, 0.0, True, want_h=True)
    sub = full["sub"]
    v64, mG64, g64 = _row_terms(full["q"][sub], full["p"][sub], full["q"], full["p"], SIG_L)
    assert rel_err(v.cpu()[sub], v64) < 1e-5
    assert rel_err(mG.cpu()[sub], mG64) < 1e-5
    assert rel_err(g.cpu()[sub], g64) < 1e-5
    h64 = 0.5 * (full["p"][sub] * v64).sum(-1)
    assert rel_err(h.cpu()[sub], h64) < 1e-5


@pytest.mark.gpu
def test_bwd_fullsize_subset(full):
    from difficp_amd import _lib
    gam = 0.37
    gdiv = torch.full((1,), gam, device=full["qd"].device)
    gq, gp = _lib.ode_self_bwd(full["qd"], full["pd"], full["ad"], full["bd"], gdiv, SIG_L, 0.0)
    gq64, gp64 = _bwd_subset(full["q"], full["p"], full["a"], full["b"], gam, full["sub"], SIG_L)
    sub = full["sub"]
    assert rel_err(gq.cpu()[sub], gq64) < 2e-5
    assert rel_err(gp.cpu()[sub], gp64) < 2e-5


@pytest.mark.gpu
def test_ext_fwd_fullsize_subset(full, dev):
    from difficp_amd import _lib
    g = torch.Generator().manual_seed(77)
    x = torch.rand(full["q"].shape[0], 3, generator=g, dtype=torch.float64)
    vx, gx = _lib.ode_ext_fwd(x.float().to(dev), full["qd"], full["pd"], SIG_L, 0.0, True)
    sub = full["sub"]
    v64 = R.KRed(x[sub], full["q"], full["p"], SIG_L)
    assert rel_err(vx.cpu()[sub], v64) < 1e-5


@pytest.mark.gpu
def test_fullsize_deterministic_and_split_invariant(full):
    from difficp_amd import _lib
    args = (full["qd"], full["pd"], full["ad"], full["bd"], torch.ones(1, device=full["qd"].device))
    outs = []
    for rounds in (0, 0, 1, 8):
        _lib.set_option("split_rounds", rounds)
        try:
            v, mG, g, _ = _lib.ode_self_fwd(full["qd"], full["pd"], SIG_L, 0.0, True)
            gq, gp = _lib.ode_self_bwd(*args, SIG_L, 0.0)
        finally:
            _lib.set_option("split_rounds", 0)
        outs.append([t.cpu() for t in (v, mG, g, gq, gp)])
    for x0, x1 in zip(outs[0], outs[1]):
        assert torch.equal(x0, x1)            # bitwise reproducible (no atomics)
    for other in outs[2:]:
        for x0, x1 in zip(outs[0], other):
            assert rel_err(x1, x0) < 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("NF", [M_FULL, 100000, 200000])
def test_estep_fullsize_subset_and_properties(dev, NF):
    """Two-set E/M passes at C2 size (50k points x 50k components, mu = xB), the headline's
    100k x 100k and C3's 200k x 200k (GMM.py:260-282): sampled rows against float64, and the
    size-independent column identities."""
    from difficp_amd import _lib
    g = torch.Generator().manual_seed(5)
    X = torch.rand(NF, 3, generator=g, dtype=torch.float64)
    mu = torch.rand(NF, 3, generator=g, dtype=torch.float64)
    w = 0.1 * torch.randn(NF, generator=g, dtype=torch.float64)
    lpi = w - w.logsumexp(0)
    lgn = 3 * (math.log(SIG_G) + 0.5 * math.log(2 * math.pi))
    f = lambda t: t.float().to(dev).contiguous()
    T, T2, stats = _lib.gmm_estep(f(X), f(mu), f(lpi / math.log(2)), f((mu * mu).sum(-1)), SIG_G, lgn, True)
    sub = torch.randperm(NF, generator=g)[:NSUB]
    D2 = ((X[sub][:, None, :] - mu[None]) ** 2).sum(-1)
    t = lpi[None] - D2 / (2 * SIG_G ** 2) - lgn
    T64 = t.logsumexp(1)
    gam = torch.exp(t - T64[:, None])
    Y64 = gam @ mu
    assert rel_err(T.cpu()[sub], T64) < 1e-5
    assert rel_err(T2.cpu()[sub], (T64 + lgn) / math.log(2)) < 1e-5     # log2, without lgn
    assert rel_err(stats.cpu()[sub, :3], Y64) < 1e-5
    # M-step column statistics: log sum_n gamma_nc and the gamma-weighted means
    col = _lib.gmm_mstep(f(X), T2, f(mu), f(lpi / math.log(2)), SIG_G).cpu().double()
    wn = col[:, 0]
    assert abs(float(wn.logsumexp(0)) - math.log(NF)) < 1e-5      # sum_nc gamma = N
    fin = torch.isfinite(wn)
    xsum = (torch.exp(wn[fin])[:, None] * col[fin, 1:]).sum(0)
    assert rel_err(xsum, X.sum(0)) < 1e-5                             # sum_c sum_n gamma x_n = sum_n x_n
