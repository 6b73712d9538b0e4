"""Hinted vs unhinted E-step: T2 error against the hint's offset above the true T2, per kernel
(packed / scalar rows), re-reference mode and column split (force_splits)."""
import json, math, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from difficp_amd import _lib  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(5)
N, C = 1536, 40000
X = torch.rand(N, 3, generator=g, dtype=torch.float64).float().to(dev)
mu = torch.rand(C, 3, generator=g, dtype=torch.float64).float().to(dev)
w2 = torch.full((C,), -math.log2(C), device=dev)
mu2 = (mu * mu).sum(-1)
T, T2, st = _lib.gmm_estep(X, mu, w2, mu2, 0.01, 0.0, True)
for opt, vals in (("lse_pk", (1, 0)), ("lse_adapt", (0, 1000)), ("force_splits", (0, 1, 4))):
    old = _lib.get_option(opt)
    for v in vals:
        _lib.set_option(opt, v)
        for off in (0.0, 8.0, 20.0, 50.0, 100.0, 200.0, 300.0, -20.0):
            Th, T2h, sth = _lib.gmm_estep(X, mu, w2, mu2, 0.01, 0.0, True, hint=T2 + off)
            d = T2h - T2
            print(json.dumps({opt: v, "off": off, "max_abs": float(d.abs().max()), "min": float(d.min()),
                              "n_bad": int((d.abs() > 1e-3).sum())}), flush=True)
    _lib.set_option(opt, old)
