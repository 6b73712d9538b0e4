"""E-step at 100k x 100k (two independent clouds, uniform weights) against sigma: the bound
shift (option "lse_bound" 1: min(hint - 8, max_c w2_c - 8), no sample pass, listed rows summed
again) against the sampled shift with adaptive re-referencing (0), with and without the shift
hint (the previous step's T2); the two modes' outputs against each other.

    python tools/probes/estep_bound.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from difficp_amd import _lib  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    M = 100000
    g = torch.Generator().manual_seed(1)
    X = torch.rand(M, 3, generator=g).to(dev)
    mu = torch.rand(M, 3, generator=g).to(dev)
    w2 = torch.full((M,), -16.6, device=dev)
    mu2 = (mu * mu).sum(-1)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(); fn(); fn(); e1.record(); e1.synchronize()
            best = min(best, e0.elapsed_time(e1) / 2)
        return round(best, 4)

    rel = lambda a, b: float((a - b).norm() / b.norm())
    old = _lib.get_option("lse_bound")
    for sigma in (0.05, 0.02, 0.01, 0.005):
        row = {"sigma": sigma}
        outs = {}
        for b in (0, 1):
            _lib.set_option("lse_bound", b)
            T, T2, st = _lib.gmm_estep(X, mu, w2, mu2, sigma, 0.0, True)
            Th, T2h, sth = _lib.gmm_estep(X, mu, w2, mu2, sigma, 0.0, True, hint=T2)
            outs[b] = (T, st, Th, sth)
            row[f"bound{b}_ms"] = timed(lambda: _lib.gmm_estep(X, mu, w2, mu2, sigma, 0.0, True))
            row[f"bound{b}_hint_ms"] = timed(lambda: _lib.gmm_estep(X, mu, w2, mu2, sigma, 0.0, True, hint=T2))
        row["T_rel"] = rel(outs[1][0], outs[0][0])
        row["stats_rel"] = rel(outs[1][1], outs[0][1])
        row["hint_T_rel"] = rel(outs[1][2], outs[0][2])
        print(json.dumps(row), flush=True)
    _lib.set_option("lse_bound", old)


if __name__ == "__main__":
    main()
