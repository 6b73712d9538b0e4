"""Support schemes on the device: the 3D grid support of DiffPSR (the
reference's grid is 2D only, PSR.py:472-482 -- parity-unpinned: support-point count, coverage,
free-energy monotonicity and bitwise determinism are checked), and DiffPSR_std with
decimated / grid supports and template weights (PSR_standard.py:445-503; the reference's
golden trace covers the dense support only)."""
import warnings

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _grid_run(dev):
    from difficp_amd import workloads
    from difficp_amd.core.GMM import GaussianMixtureUnif
    from difficp_amd.core.LDDMM import LDDMMModel
    from difficp_amd.core.PSR import DiffPSR
    spec = {"device": dev, "dtype": torch.float32}
    x = [f.to(dev) for f in workloads.atlas_frames(3, 3000, seed=5)]
    G = GaussianMixtureUnif(torch.zeros(64, 3), spec=spec)
    G.to_optimize = {"mu": True, "sigma": True, "w": True, "eta0": False}
    LM = LDDMMModel(sigma=0.1, D=3, lambd=1e3, version="hybrid", scheme="Euler", nt=10, spec=spec)
    torch.manual_seed(0)
    P = DiffPSR(x, G, LM, dataspec=spec, compspec=spec)
    P.printstuff = False
    P.reinitialize_GMM()
    P.set_support_scheme("grid", rho=1.0)
    fes = [P.FE]
    with warnings.catch_warnings():
        warnings.simplefilter("error", RuntimeWarning)        # uncovered points would raise
        for _ in range(2):
            P.GMM_opt(max_iterations=10, tol=1e-3)
            fes.append(P.FE)
            P.Reg_opt(nmax=1, tol=1e-3)
            fes.append(P.FE)
    return P, fes


def test_grid_support_3d_diffpsr(dev):
    from difficp_amd.core.support import bounds_with_margin
    P, fes = _grid_run(dev)
    lo, hi = bounds_with_margin(P.allx0, 3)
    R = 0.1
    n = np.prod([len(np.arange(lo[d] - R / 2, hi[d] + R / 2, R)) for d in range(3)])
    assert P.q0[0].shape == (n, 3)
    for f0, f1 in zip(fes[:-1], fes[1:]):
        assert f1 <= f0 + 1e-6 * abs(f0), fes
    P2, fes2 = _grid_run(dev)
    assert fes2 == fes
    for k in range(3):
        assert torch.equal(P.a0[k], P2.a0[k]) and torch.equal(P.x1[k, 0], P2.x1[k, 0])


@pytest.mark.parametrize("scheme", ["decim", "grid"])
@pytest.mark.parametrize("weights", [False, True])
def test_psr_std_support_schemes(dev, scheme, weights):
    from difficp_amd.core.LDDMM import LDDMMModel
    from difficp_amd.core.PSR_standard import DiffPSR_std
    from difficp_amd.tools.kernel import GaussKernel
    from difficp_amd.tools.point_sets import decimate
    spec = {"device": dev, "dtype": torch.float32}
    g = torch.Generator().manual_seed(13)
    t = torch.linspace(0, 2 * np.pi, 121)[:-1]
    y0 = torch.stack([0.5 + 0.3 * torch.cos(t), 0.5 + 0.2 * torch.sin(t)], 1)
    xs = []
    for k in range(3):
        tk = torch.rand(200, generator=g) * 2 * np.pi
        xs.append((torch.stack([0.5 + (0.3 + 0.03 * k) * torch.cos(tk), 0.5 + (0.2 - 0.02 * k) * torch.sin(tk)], 1)
                   + 0.01 * torch.randn(200, 2, generator=g)).to(dev))
    DK = GaussKernel(0.1, 2, spec=spec)
    LM = LDDMMModel(sigma=0.2, D=2, lambd=2.0, version="classic", scheme="Euler", nt=10, spec=spec)
    P = DiffPSR_std(xs, y0.to(dev), 0.05, LM, DK, template_weights=weights, dataspec=spec, compspec=spec)
    P.printstuff = False
    P.set_support_scheme(scheme, rho=1.0)
    if scheme == "decim":
        assert P.q0.shape[0] == len(decimate(y0.to(dev), 0.2)[0])
    Es = [P.E]
    for _ in range(2):
        P.Reg_opt(nmax=2, tol=1e-4)
        Es.append(P.E)
        P.Template_opt(nmax=2, tol=1e-4)
        Es.append(P.E)
    assert all(np.isfinite(Es))
    if weights:
        assert P.w0[0].shape == (120,)
    # against the reference's float64 trace of the same inputs (tests/golden/psr_std_support.npz)
    import std_support_case as C
    ref = C.reference(scheme, weights)
    assert abs(Es[0] - ref[0]) <= 1e-5 * abs(ref[0]), (Es[0], ref[0])
    if scheme == "grid":
        # the energy after each optimisation stage: an L-BFGS path whose float32 rounding is
        # amplified stage by stage.  The CPU float32 oracle drifts from float64 by FP32_DEV; the
        # GPU's float32 path (other fma contractions and reduction orders) drifts by up to 3.5x
        # that at the last stage (5.6e-3 with weights, 2.0e-3 without; the first energy 7e-7),
        # bitwise the same with every host mechanism switched off (workspace cache, graphs,
        # direct closures: profiles/r05_psr_std_trace_switches.jsonl) -- so 4x, not 2x
        tol = max(1e-3, 4 * C.FP32_DEV[(scheme, weights)])
        for a, b in zip(Es, ref):
            assert abs(a - b) <= tol * abs(b), (Es, ref)
    else:
        # the decim traces are not float32-reproducible (test_host_logic.py::
        # test_psr_std_support_fp32_oracle_deviation); the reference itself decreases the
        # energy overall -- and raises its own increase warning once without weights
        assert Es[-1] < Es[0] and ref[-1] < ref[0]
