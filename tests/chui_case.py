"""SURVEY 8c fixture: the reference's Chui ex3 two-set trace (tests/golden/chui_ex3.npz, see
make_golden.chui_case) replayed through the product API."""
import os

import numpy as np
import torch

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "chui_ex3.npz")


def run_chui(spec, iters=4, check=None):
    """ICP_two_set defaults (ICP_two_set.py:140-207, 254-282), lambda 1e2, grid support."""
    from difficp_amd.core.GMM import GaussianMixtureUnif
    from difficp_amd.core.LDDMM import LDDMMModel
    from difficp_amd.core.PSR import DiffPSR
    z = np.load(GOLD)
    T = lambda k: torch.from_numpy(np.asarray(z[k])).to(dtype=spec["dtype"], device=spec["device"])
    GM = GaussianMixtureUnif(T("xB"), sigma=0.1, spec=spec)
    GM.to_optimize = {"mu": False, "sigma": True, "w": False, "eta0": False}
    LM = LDDMMModel(sigma=0.2, D=2, lambd=1e2, withlogdet=True, gradcomponent=False, scheme="Euler",
                    nt=10, spec=spec)
    PS = DiffPSR([[T("xA")]], GM, LM, dataspec=spec, compspec=spec)
    PS.printstuff = False
    PS.set_support_scheme("grid", rho=1.0)
    check("init", -1, PS, z)
    for it in range(iters):
        PS.GMM_opt(max_iterations=10, tol=1e-3)
        check("gmm", it, PS, z)
        PS.Reg_opt(tol=1e-3, nmax=1)
        check("reg", it, PS, z)
    return PS
