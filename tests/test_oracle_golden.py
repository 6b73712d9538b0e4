"""Pin the CPU oracle (oracle/torch_ref.py, oracle/difficp_ref.c) against the golden
vectors produced by the reference itself (tests/golden/make_golden.py).  CPU only."""
import os

import numpy as np
import pytest
import torch

from conftest import rel_err
from oracle import torch_ref as R

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(GOLD, name + ".npz"))


def T(a):
    return torch.from_numpy(np.asarray(a))


def keys(z, suffix):
    return sorted({k.split("/")[0] for k in z.files if k.endswith(suffix)})


@pytest.mark.parametrize("fname", ["reductions", "reductions_large"])
def test_reductions_oracle_vs_reference(fname):
    z = load(fname)
    for key in keys(z, "/KRed"):
        g = lambda n: T(z[f"{key}/{n}"])
        x, y, b, c, d, dm = (g("in_" + n) for n in ("x", "y", "b", "c", "d", "dm"))
        s = float(z[f"{key}/sigma"])
        out = {"KBase": R.KBase(x, y, s), "KRedScal": R.KRedScal(x, y, d, s), "KRed": R.KRed(x, y, b, s),
               "GradKRed": R.GradKRed(x, y, s), "GradKRed_rev": R.GradKRed_rev(x, y, dm, s),
               "DDKRed": R.DDKRed(x, y, b, s), "GenDKRed": R.GenDKRed(x, y, b, c, s),
               "HessKRed": R.HessKRed(x, y, b, c, s), "LapKRed": R.LapKRed(x, y, s),
               "GradLapKRed": R.GradLapKRed(x, y, s)}
        for name, v in out.items():
            assert rel_err(v, g(name)) < 1e-12, (key, name)


def test_shoot_oracle_vs_reference():
    z = load("shoot")
    for key in keys(z, "/q1"):
        version, scheme, xs, Ds = key.split("_")
        ext, D = int(xs[1:]), int(Ds[1:])
        sig, lam, nt = z[f"{key}/params"]
        m = R.LDDMM(float(sig), D, float(lam), version == "logdet", version != "classic",
                    scheme=scheme, nt=int(nt))
        q0, tgt = T(z[f"{key}/q0"]), T(z[f"{key}/tgt"])
        p0 = T(z[f"{key}/p0"]).clone().requires_grad_(True)
        x0 = T(z[f"{key}/x0"]) if ext else None
        sh = m.Shoot(q0, p0, x0)
        last = sh[-1][-1] if ext else sh[-1][0]
        traj = m.trajloss(sh)
        L = traj + ((last - tgt) ** 2).sum()
        (gp,) = torch.autograd.grad(L, (p0,))
        assert rel_err(sh[-1][0], T(z[f"{key}/q1"])) < 1e-12, key
        assert rel_err(sh[-1][1], T(z[f"{key}/p1"])) < 1e-12, key
        assert rel_err(sh[-1][2], T(z[f"{key}/cost1"])) < 1e-10, key
        if ext:
            assert rel_err(sh[-1][3], T(z[f"{key}/x1"])) < 1e-12, key
        assert abs(float(traj) - float(z[f"{key}/trajloss"])) < 1e-10 * max(1, abs(float(traj)))
        assert rel_err(gp, T(z[f"{key}/grad_p0"])) < 1e-10, key
        assert abs(float(m.Hamiltonian(q0, p0.detach())) - float(z[f"{key}/H0"])) < 1e-12


def test_em_oracle_vs_reference():
    z = load("em")
    opts = {"all": dict(mu=True, w=True, sigma=True, eta0=True),
            "sigma": dict(mu=False, w=False, sigma=True, eta0=True),
            "mu": dict(mu=True, w=False, sigma=False, eta0=False),
            "mu_w": dict(mu=True, w=True, sigma=False, eta0=True)}
    for key in keys(z, "/X"):
        Ds, outs, oname = key.split("_", 2)
        outl = outs == "out1"
        X = T(z[f"{key}/X"])
        st = dict(mu=T(z[f"{key}/mu0"]), w=T(z[f"{key}/w0"]), sigma=float(z[f"{key}/sigma0"]),
                  outliers={"vol0": None, "eta0": 0.0} if outl else None)
        for it in range(2):
            Y, Cfe, FE, st = R.em_step(X, st["mu"], st["w"], st["sigma"], opts[oname], st["outliers"])
            assert rel_err(Y, T(z[f"{key}/it{it}/Y"])) < 1e-12, (key, it)
            assert abs(float(FE) - float(z[f"{key}/it{it}/FE"])) < 1e-9 * abs(float(FE)) + 1e-9
            assert abs(float(Cfe) - float(z[f"{key}/it{it}/Cfe"])) < 1e-9 * abs(float(Cfe)) + 1e-9
            assert rel_err(st["mu"], T(z[f"{key}/it{it}/mu"])) < 1e-12
            assert rel_err(st["w"], T(z[f"{key}/it{it}/w"])) < 1e-12
            assert abs(st["sigma"] - float(z[f"{key}/it{it}/sigma"])) < 1e-14
            if outl:
                assert abs(st["outliers"]["eta0"] - float(z[f"{key}/it{it}/eta0"])) < 1e-12
        ll = R.log_likelihoods(X, st["mu"], st["w"], st["sigma"])
        assert rel_err(ll, T(z[f"{key}/loglik"])) < 1e-12, key


def test_c_oracle_vs_torch_oracle():
    """The C restatement (cpu_baseline leg) agrees with the pinned torch oracle."""
    from oracle import c_ref
    g = torch.Generator().manual_seed(0)
    M, D, sig = 500, 3, 0.2
    q = torch.rand(M, D, generator=g, dtype=torch.float64)
    p = 0.1 * torch.randn(M, D, generator=g, dtype=torch.float64)
    m = R.LDDMM(sig, D, 10.0, False, True)
    v, mG, c = m.ODE(q, p, torch.zeros(1, dtype=torch.float64))
    vc, mGc, gc = c_ref.ode_self_fwd(q, p, sig)
    assert rel_err(vc, v) < 1e-6 and rel_err(mGc, mG) < 1e-6
    assert abs(float(gc.double().sum()) - float(c)) < 1e-5 * abs(float(c)) + 1e-6
    qq, pp = q.clone().requires_grad_(True), p.clone().requires_grad_(True)
    a, b = torch.randn(M, D, generator=g, dtype=torch.float64), torch.randn(M, D, generator=g, dtype=torch.float64)
    v, mG, c = m.ODE(qq, pp, torch.zeros(1, dtype=torch.float64))
    gq, gp = torch.autograd.grad((a * v).sum() + (b * mG).sum() + 0.7 * c.sum(), (qq, pp))
    gqc, gpc = c_ref.ode_self_bwd(q, p, a, b, 0.7, sig)
    assert rel_err(gqc, gq) < 1e-5 and rel_err(gpc, gp) < 1e-5
    X = torch.rand(300, 3, generator=g, dtype=torch.float64)
    mu = torch.rand(20, 3, generator=g, dtype=torch.float64)
    w = torch.randn(20, generator=g, dtype=torch.float64)
    Tc, _ = c_ref.gmm_estep(X, mu, w, 0.1)
    lgn = 3 * (np.log(0.1) + 0.5 * np.log(2 * np.pi))
    t = w[None] - w.logsumexp(0) - ((X[:, None] - mu[None]) ** 2).sum(-1) / (2 * 0.01) - lgn
    assert rel_err(Tc, t.logsumexp(1)) < 1e-6


DECIM_CASES = ("rand2d", "rand3d", "grid2d", "dup3d")


def test_decimate_oracle_vs_reference():
    """Greedy decimation (point_sets.py:102-133): identical kept indices, in order."""
    z = load("decim")
    for name in DECIM_CASES:
        kept, rej = R.decimate(T(z[f"{name}/x"]), float(z[f"{name}/R"]))
        assert kept == z[f"{name}/kept"].tolist(), name
        assert sorted(kept + rej) == list(range(z[f"{name}/x"].shape[0]))


def test_oracle_ridge_cg_matches_dense():
    """The restated KeOps CG (KridgeSolve_keops, kernel.py:239-241) converges to the dense
    ridge solution (KridgeSolve_torch, kernel.py:234-237) in float64."""
    g = torch.Generator().manual_seed(0)
    x = torch.rand(200, 3, generator=g, dtype=torch.float64)
    v = torch.randn(200, 3, generator=g, dtype=torch.float64)
    b, k = R.KridgeSolve_cg(x, v, 0.1, 0.5, eps=1e-10)
    ref = R.KridgeSolve_torch(x, v, 0.1, 0.5)
    assert 0 < k < 200
    assert float((b - ref).norm() / ref.norm()) < 1e-8


def test_oracle_data_distance_vs_reference():
    """data_distance (PSR_standard.py:37-58) against the reference's own values
    (tests/golden/psr_std.npz), with and without template weights."""
    z = np.load(os.path.join(GOLD, "psr_std.npz"))
    for D in (2, 3):
        x, y, w = (torch.from_numpy(z[f"dd{D}/{k}"]) for k in ("x", "y", "w"))
        assert abs(float(R.data_distance(x, y, 0.15)) - float(z[f"dd{D}/L"])) < 1e-12
        assert abs(float(R.data_distance(x, y, 0.15, w)) - float(z[f"dd{D}/Lw"])) < 1e-12
