"""The PSR_std grid-support energy trace of tests/test_gpu_support.py (weights on), printed as
one JSON line -- run under different environment switches (DICP_WS_POISON, DICP_SHOOT_GRAPH,
DICP_DIRECT_LOSSGRAD, DICP_WS_NOCACHE) to find what moves it.

    python tools/probes/psr_std_trace.py [grid|decim] [0|1]
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    scheme = sys.argv[1] if len(sys.argv) > 1 else "grid"
    weights = bool(int(sys.argv[2])) if len(sys.argv) > 2 else True
    from difficp_amd import _lib
    if os.environ.get("DICP_WS_NOCACHE"):
        _lib._WS_CACHE_MAX = 0
    from difficp_amd.core.LDDMM import LDDMMModel
    from difficp_amd.core.PSR_standard import DiffPSR_std
    from difficp_amd.tools.kernel import GaussKernel
    dev = torch.device("cuda:0")
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
    Es = [P.E]
    for _ in range(2):
        P.Reg_opt(nmax=2, tol=1e-4)
        Es.append(P.E)
        P.Template_opt(nmax=2, tol=1e-4)
        Es.append(P.E)
    import std_support_case as C
    ref = C.reference(scheme, weights)
    env = {k: v for k, v in os.environ.items() if k.startswith("DICP_")}
    print(json.dumps({"env": env, "scheme": scheme, "weights": weights, "Es": [float(e) for e in Es],
                      "rel_vs_fp64": [abs(a - b) / abs(b) for a, b in zip(Es, ref)]}), flush=True)


if __name__ == "__main__":
    main()
