"""The north_star-named API on the device: LDDMMRegistration.apply / backward
(registrations.py:56-87) and LDDMMModel.v / mdivsum (LDDMM.py:100-138), incl. their autograd,
against the reference goldens (x1 of Shoot with external points, produced by the reference
itself) and the float64 oracle.  Tolerances: 1e-5 forward, 2e-5 backward / gradients."""
import os

import numpy as np
import pytest
import torch

from conftest import rel_err
from oracle import torch_ref as R

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _spec(dev):
    return {"device": dev, "dtype": torch.float32}


def test_registration_apply_matches_golden_x1(dev):
    """apply(X) = Shoot(q0, a0, X)[-1][3] (registrations.py:72-77): the reference's own x1."""
    from difficp_amd.core.LDDMM import LDDMMModel
    from difficp_amd.core.registrations import LDDMMRegistration
    z = np.load(os.path.join(GOLD, "shoot.npz"))
    keys = sorted({k.split("/")[0] for k in z.files if k.endswith("/x1")})
    assert len(keys) >= 8
    for key in keys:
        version, scheme, _, Ds = key.split("_")
        sig, lam, nt = z[f"{key}/params"]
        LM = LDDMMModel(sigma=float(sig), D=int(Ds[1:]), lambd=float(lam), version=version,
                        scheme=scheme, nt=int(nt), spec=_spec(dev))
        f = lambda n: torch.from_numpy(np.asarray(z[f"{key}/{n}"])).float().to(dev)
        reg = LDDMMRegistration(LM, f("q0"), f("p0"))
        y = reg.apply(f("x0"))
        assert rel_err(y.cpu(), torch.from_numpy(z[f"{key}/x1"])) < 1e-5, key


@pytest.mark.parametrize("version", ["classic", "hybrid", "logdet"])
@pytest.mark.parametrize("scheme", ["Euler", "Ralston"])
def test_registration_backward_matches_oracle(dev, version, scheme):
    """backward(Y) = Shoot(q1, -p1, Y)[-1][3] (registrations.py:66-69, 79-87) against the
    float64 oracle; for eta = 0, backward(apply(X)) returns close to X (the flow is reversed up
    to the integrator's discretisation error)."""
    from difficp_amd.core.LDDMM import LDDMMModel
    from difficp_amd.core.registrations import LDDMMRegistration
    g = torch.Generator().manual_seed(9)
    M, N, D = 300, 900, 3
    q0 = torch.rand(M, D, generator=g, dtype=torch.float64)
    p0 = 0.02 * torch.randn(M, D, generator=g, dtype=torch.float64)
    X = torch.rand(N, D, generator=g, dtype=torch.float64)
    lam = 50.0
    LM = LDDMMModel(sigma=0.2, D=D, lambd=lam, version=version, scheme=scheme, nt=10, spec=_spec(dev))
    reg = LDDMMRegistration(LM, q0.float().to(dev), p0.float().to(dev))
    Y = reg.apply(X.float().to(dev))
    B = reg.backward(Y)
    m = R.LDDMM(0.2, D, lam, version == "logdet", version != "classic", scheme=scheme, nt=10)
    fw = m.Shoot(q0, p0, X)
    Y64 = fw[-1][3]
    bw = m.Shoot(fw[-1][0], -fw[-1][1], Y.double().cpu())
    assert rel_err(Y.cpu(), Y64) < 1e-5
    assert rel_err(B.cpu(), bw[-1][3]) < 2e-5
    if version != "logdet":
        # eta = 0: v is odd in p, so shooting from the arrival state with -p1 retraces the
        # flow; with gradcomponent the -eta GradKRed part of v does not flip (the reference's
        # backward is then not an inverse) -- only the parity above applies
        disp = float((Y64 - X).norm())
        assert float((B.double().cpu() - X).norm()) < 0.05 * disp
    # previous_forwardshoot is reused as given
    sh = reg.shoot(None)
    assert torch.equal(reg.backward(Y, previous_forwardshoot=sh), B)


@pytest.mark.parametrize("gradcomponent", [False, True])
def test_v_and_mdivsum_with_autograd(dev, gradcomponent):
    """LDDMMModel.v(x, q, p) and mdivsum(x, q, p) (rev False / True) and their gradients
    w.r.t. x, q, p against float64 autograd through the oracle."""
    from difficp_amd.core.LDDMM import LDDMMModel
    g = torch.Generator().manual_seed(12)
    M, N, D, sig, lam = 400, 700, 3, 0.15, 20.0
    q = torch.rand(M, D, generator=g, dtype=torch.float64)
    p = 0.1 * torch.randn(M, D, generator=g, dtype=torch.float64)
    x = torch.rand(N, D, generator=g, dtype=torch.float64)
    w = torch.randn(N, D, generator=g, dtype=torch.float64)
    m = R.LDDMM(sig, D, lam, gradcomponent, True)
    LM = LDDMMModel(sigma=sig, D=D, lambd=lam, gradcomponent=gradcomponent, withlogdet=True,
                    scheme="Euler", spec=_spec(dev))
    ins64 = [t.clone().requires_grad_(True) for t in (x, q, p)]
    v64 = m.v(*ins64)
    gv64 = torch.autograd.grad((v64 * w).sum(), ins64)
    ins = [t.float().to(dev).requires_grad_(True) for t in (x, q, p)]
    v = LM.v(*ins)
    assert rel_err(v.detach().cpu(), v64.detach()) < 1e-5
    gv = torch.autograd.grad((v * w.float().to(dev)).sum(), ins)
    for a, b in zip(gv, gv64):
        assert rel_err(a.cpu(), b) < 2e-5
    for rev in (False, True):
        ins64 = [t.clone().requires_grad_(True) for t in (x, q, p)]
        d64 = m.mdivsum(*ins64)
        gd64 = torch.autograd.grad(d64, ins64)
        ins = [t.float().to(dev).requires_grad_(True) for t in (x, q, p)]
        d = LM.mdivsum(*ins, rev=rev)
        assert abs(float(d.detach()) - float(d64.detach())) < 1e-5 * abs(float(d64.detach())), rev
        gd = torch.autograd.grad(d, ins)
        for a, b in zip(gd, gd64):
            assert rel_err(a.cpu(), b) < 2e-5, rev
    # empty x (LDDMM.py:111-112, 131-132)
    e = torch.empty(0, D, device=dev)
    assert LM.v(e, ins[1].detach(), ins[2].detach()).shape == (0, D)
    assert float(LM.mdivsum(e, ins[1].detach(), ins[2].detach())) == 0.0
