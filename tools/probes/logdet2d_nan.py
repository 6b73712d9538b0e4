"""The logdet model's gradient (eta != 0 VJP) on 2D clouds of a few hundred / thousand points:
finite or not with each eta VJP variant (bwd_eta_alg 2 packed symmetric, 1 symmetric, 0
ordered), against the float64 oracle at 700 points.

    python tools/probes/logdet2d_nan.py > out.jsonl
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from difficp_amd import _lib  # noqa: E402
from difficp_amd.core import shooting  # noqa: E402
from difficp_amd.core.LDDMM import LDDMMModel  # noqa: E402


def rel(a, b):
    return float((a - b).norm() / b.norm())


def main():
    from oracle import torch_ref as R
    dev = torch.device("cuda:0")
    shooting._GRAPH_ON = False
    for M, D in ((700, 2), (3333, 2), (2000, 3)):
        g = torch.Generator().manual_seed(M + D)
        q0 = torch.rand(M, D, generator=g, dtype=torch.float64)
        p0 = 0.02 * torch.randn(M, D, generator=g, dtype=torch.float64)
        tgt = q0 + 0.05 * torch.randn(M, D, generator=g, dtype=torch.float64)
        ref = None
        if M <= 1000:
            LR = R.LDDMM(0.1, D, 100.0, True, True, scheme="Euler", nt=10)
            p = p0.clone().requires_grad_(True)
            sh = LR.Shoot(q0, p, None)
            L = LR.trajloss(sh) + ((sh[-1][0] - tgt) ** 2).sum()
            (ref,) = torch.autograd.grad(L, (p,))
        old = _lib.get_option("bwd_eta_alg")
        for alg in (2, 1, 0):
            _lib.set_option("bwd_eta_alg", alg)
            LM = LDDMMModel(sigma=0.1, D=D, lambd=100.0, version="logdet", nt=10, scheme="Euler",
                            spec={"device": dev, "dtype": torch.float32})
            LM.shoot_cache = None
            p = p0.float().to(dev).requires_grad_(True)
            sh = LM.Shoot(q0.float().to(dev), p, None)
            L = LM.trajloss(sh) + ((sh[-1][0] - tgt.float().to(dev)) ** 2).sum()
            L.backward()
            gr = p.grad.double().cpu()
            nan_rows = (~torch.isfinite(gr)).any(1).nonzero().flatten()
            print(json.dumps({"M": M, "D": D, "bwd_eta_alg": alg, "L": float(L),
                              "grad_finite": bool(torch.isfinite(gr).all()),
                              "nan_rows": nan_rows.numel(), "first_nan_rows": nan_rows[:8].tolist(),
                              "rel_vs_fp64": None if ref is None or not torch.isfinite(gr).all() else rel(gr, ref)}),
                  flush=True)
        _lib.set_option("bwd_eta_alg", old)


if __name__ == "__main__":
    main()
