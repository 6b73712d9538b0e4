"""Does any kernel of a shooting + adjoint read workspace it did not write?  Runs the direct
path (no graphs) with the workspaces poisoned (NaN bytes before every call, _lib._WS_POISON)
and without, at ragged sizes, and reports whether the results are finite and bitwise equal.

    python tools/probes/ws_poison.py > out.jsonl
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from difficp_amd import _lib  # noqa: E402
from difficp_amd.core import shooting  # noqa: E402
from difficp_amd.core.LDDMM import LDDMMModel  # noqa: E402


def run(LM, q0, p0, tgt):
    p = p0.clone().requires_grad_(True)
    sh = LM.Shoot(q0, p, None)
    L = LM.trajloss(sh) + ((sh[-1][0] - tgt) ** 2).sum()
    L.backward()
    return [sh.Q.detach().clone(), sh.P.detach().clone(), sh.C.detach().clone(), p.grad.clone()]


def main():
    dev = torch.device("cuda:0")
    shooting._GRAPH_ON = False
    for version in ("classic", "hybrid", "logdet"):
        for M, D in ((700, 2), (257, 2), (1025, 3), (2000, 3), (3333, 2), (9000, 3)):
            g = torch.Generator().manual_seed(M + D)
            q0 = torch.rand(M, D, generator=g).to(dev)
            p0 = (0.02 * torch.randn(M, D, generator=g)).to(dev)
            tgt = (q0.cpu() + 0.05 * torch.randn(M, D, generator=g)).to(dev)
            LM = LDDMMModel(sigma=0.1, D=D, lambd=100.0, version=version, nt=10, scheme="Euler",
                            spec={"device": dev, "dtype": torch.float32})
            LM.shoot_cache = None
            _lib._WS_POISON = False
            a = run(LM, q0, p0, tgt)
            _lib._WS_POISON = True
            b = run(LM, q0, p0, tgt)
            _lib._WS_POISON = False
            names = ("Q", "P", "C", "grad")
            print(json.dumps({"version": version, "M": M, "D": D,
                              "finite": {n: bool(torch.isfinite(t).all()) for n, t in zip(names, b)},
                              "equal": {n: bool(torch.equal(x, y)) for n, x, y in zip(names, a, b)}}),
                  flush=True)


if __name__ == "__main__":
    main()
