"""CPU: the float64 row/column-subset formulas of tests/fullsize_ref.py (used by the full-size
GPU parity tests) equal the oracle's full computation (oracle/torch_ref.py, itself pinned by
the reference goldens) at small size, for eta = 0 and eta != 0, self and external points."""
import math

import pytest
import torch

import fullsize_ref as F
from conftest import rel_err
from oracle import torch_ref as R


@pytest.mark.parametrize("eta", [0.0, 0.02])
def test_self_terms_and_vjp_match_oracle(eta):
    g = torch.Generator().manual_seed(3)
    M, sig = 260, 0.15
    q = torch.rand(M, 3, generator=g, dtype=torch.float64)
    p = 0.1 * torch.randn(M, 3, generator=g, dtype=torch.float64)
    a = torch.randn(M, 3, generator=g, dtype=torch.float64)
    b = torch.randn(M, 3, generator=g, dtype=torch.float64)
    sub = torch.tensor([0, 5, 77, 259])
    m = R.LDDMM(sig, 3, 1.0 / eta if eta else 50.0, eta != 0, True)
    v64, mG64, c64 = m.ODE(q, p, torch.zeros(1, dtype=torch.float64))
    v, mG, gr, h = F.self_terms(q[sub], p[sub], q, p, sig, eta, chunk=97)
    assert rel_err(v, v64[sub]) < 1e-12 and rel_err(mG, mG64[sub]) < 1e-12
    _, _, gall, hall = F.self_terms(q, p, q, p, sig, eta, chunk=97)
    assert abs(float(gall.sum() - c64.sum())) < 1e-10 * max(1.0, abs(float(c64.sum())))
    H = m.Hamiltonian(q, p)
    assert abs(float(hall.sum() - H)) < 1e-10 * max(1.0, abs(float(H)))
    gam = 0.7
    for bb in (b, None):
        qq = q.clone().requires_grad_(True)
        pq = p.clone().requires_grad_(True)
        v, mG, c = m.ODE(qq, pq, torch.zeros(1, dtype=torch.float64))
        L = (a * v).sum() + gam * c.sum() + ((bb * mG).sum() if bb is not None else 0)
        gq, gp = torch.autograd.grad(L, (qq, pq))
        gqs, gps = F.self_vjp_subset(q, p, a, bb, gam, sub, sig, eta, chunk=101)
        assert rel_err(gqs, gq[sub]) < 1e-12 and rel_err(gps, gp[sub]) < 1e-12


@pytest.mark.parametrize("eta", [0.0, 0.02])
def test_ext_terms_and_vjp_match_oracle(eta):
    g = torch.Generator().manual_seed(4)
    M, N, sig = 120, 310, 0.2
    q = torch.rand(M, 3, generator=g, dtype=torch.float64)
    p = 0.1 * torch.randn(M, 3, generator=g, dtype=torch.float64)
    x = torch.rand(N, 3, generator=g, dtype=torch.float64)
    a = torch.randn(N, 3, generator=g, dtype=torch.float64)
    m = R.LDDMM(sig, 3, 1.0 / eta if eta else 50.0, eta != 0, True)
    xs, qs = torch.tensor([1, 9, 300]), torch.tensor([0, 64, 119])
    vx, gx = F.ext_terms(x, q, p, sig, eta, chunk=37)
    assert rel_err(vx, m.v(x, q, p)) < 1e-12
    md = m.mdivsum(x, q, p)
    assert abs(float(gx.sum() - md)) < 1e-10 * max(1.0, abs(float(md)))
    gam = 0.3
    xx = x.clone().requires_grad_(True)
    qq = q.clone().requires_grad_(True)
    pq = p.clone().requires_grad_(True)
    L = (a * m.v(xx, qq, pq)).sum() + gam * m.mdivsum(xx, qq, pq)
    gxa, gqa, gpa = torch.autograd.grad(L, (xx, qq, pq))
    gxs, gqs, gps = F.ext_vjp_subset(x, q, p, a, gam, xs, qs, sig, eta, chunk=53)
    assert rel_err(gxs, gxa[xs]) < 1e-12
    assert rel_err(gqs, gqa[qs]) < 1e-12 and rel_err(gps, gpa[qs]) < 1e-12


def test_gmm_rows_and_columns_match_oracle():
    g = torch.Generator().manual_seed(6)
    N, C, sig = 900, 40, 0.07
    X = torch.rand(N, 3, generator=g, dtype=torch.float64)
    mu = torch.rand(C, 3, generator=g, dtype=torch.float64)
    w = 0.3 * torch.randn(C, generator=g, dtype=torch.float64)
    lpi = w - w.logsumexp(0)
    lgn = 3 * (math.log(sig) + 0.5 * math.log(2 * math.pi))
    Y64, _, _, st = R.em_step(X, mu, w, sig, {"mu": True, "w": True, "sigma": True, "eta0": False})
    T, Y = F.gmm_rows(X, mu, lpi, sig, lgn, chunk=128)
    Yold, *_ = R.em_step(X, mu, w, sig, {"mu": False, "w": False, "sigma": False, "eta0": False})
    assert rel_err(Y, Yold) < 1e-12
    lw, mun, sd2 = F.gmm_columns(X, mu, lpi, sig, chunk=111)
    assert rel_err(mun, st["mu"]) < 1e-12
    assert rel_err(lw, st["w"]) < 1e-12
    assert abs(math.sqrt(float(sd2) / (3 * N)) - st["sigma"]) < 1e-12
    D2 = ((X[:, None] - mu[None]) ** 2).sum(-1)
    t = lpi[None] - D2 / (2 * sig ** 2) - lgn
    assert rel_err(T, t.logsumexp(1)) < 1e-13


@pytest.mark.parametrize("version", ["hybrid", "classic", "logdet"])
def test_shoot_loss_grad_matches_oracle_autograd(version):
    """The chunked whole-shooting restatement (fullsize_ref.shoot_loss_grad_p0: Euler shoot,
    trajloss, quadratic data loss and the discrete-adjoint gradient w.r.t. p0) equals the
    oracle's Shoot / trajloss with torch autograd (float64, small size)."""
    g = torch.Generator().manual_seed(21)
    M, sig, nt, lam = 150, 0.2, 5, 30.0
    grad_comp, logdet = {"hybrid": (False, True), "classic": (False, False), "logdet": (True, True)}[version]
    eta = 1.0 / lam if grad_comp else 0.0
    q0 = torch.rand(M, 3, generator=g, dtype=torch.float64)
    p0 = 0.05 * torch.randn(M, 3, generator=g, dtype=torch.float64)
    y = q0 + 0.02 * torch.randn(M, 3, generator=g, dtype=torch.float64)
    m = R.LDDMM(sig, 3, lam, grad_comp, logdet, scheme="Euler", nt=nt)
    pr = p0.clone().requires_grad_(True)
    sh = m.Shoot(q0, pr)
    traj = m.trajloss(sh)
    loss = traj + 0.5 * ((sh[-1][0] - y) ** 2).sum()
    gref, = torch.autograd.grad(loss, (pr,))
    q1, c1, tr, lo, gp0 = F.shoot_loss_grad_p0(q0, p0, sig, nt, lam, y, eta, logdet)
    assert rel_err(q1, sh[-1][0].detach()) < 1e-12
    assert abs(float(c1 - sh[-1][2].detach().sum())) < 1e-10 * max(1.0, abs(float(c1)))
    assert abs(float(tr - traj.detach())) < 1e-10 * abs(float(traj))
    assert abs(float(lo - loss.detach())) < 1e-10 * abs(float(loss))
    assert rel_err(gp0, gref) < 1e-10
