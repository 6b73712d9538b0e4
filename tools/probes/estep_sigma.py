"""E-step time at 100k x 100k (two independent clouds, uniform weights) against sigma: the
single sweep's re-reference events grow as sigma shrinks below the first-64-column sample's
nearest-component distance.  Swept over the adaptive re-reference threshold (option
"lse_adapt": eventful tiles before the per-pair test; 0 per pair throughout, 1000 tile-end
throughout), with and without the shift hint (the previous step's T2)."""
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
    old = _lib.get_option("lse_adapt")
    for sigma in (0.05, 0.02, 0.01, 0.005):
        for adapt in (0, 1, 2, 4, 1000):
            _lib.set_option("lse_adapt", adapt)
            T, T2, st = _lib.gmm_estep(X, mu, w2, mu2, sigma, 0.0, True)
            Th, T2h, sth = _lib.gmm_estep(X, mu, w2, mu2, sigma, 0.0, True, hint=T2)
            print(json.dumps({"sigma": sigma, "lse_adapt": adapt,
                              "estep_ms": timed(lambda: _lib.gmm_estep(X, mu, w2, mu2, sigma, 0.0, True)),
                              "estep_hint_ms": timed(lambda: _lib.gmm_estep(X, mu, w2, mu2, sigma, 0.0, True, hint=T2)),
                              "hint_vs_plain_T": rel(Th, T), "hint_vs_plain_stats": rel(sth, st)}), flush=True)
    _lib.set_option("lse_adapt", old)

if __name__ == "__main__":
    main()
