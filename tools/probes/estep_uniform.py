"""E-step outputs with uniform weights (the tile-level uniform path) against float64 at small,
single-tile shapes (the Chui two-set sizes) and large sigma; per-slot relative errors."""
import json
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from difficp_amd import _lib  # noqa: E402
from test_gpu_em import _estep64  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    for (N, C, sigma, D) in ((200, 200, 0.3, 2), (100, 150, 1.0, 2), (500, 80, 0.05, 2), (300, 300, 0.1, 2),
                             (2000, 20000, 0.05, 2)):
        g = torch.Generator().manual_seed(N + C)
        X = torch.rand(N, D, generator=g, dtype=torch.float64).float().double()
        mu = torch.rand(C, D, generator=g, dtype=torch.float64).float().double()
        for uniform in (True, False):
            w = torch.zeros(C, dtype=torch.float64) if uniform else 0.3 * torch.randn(C, generator=g, dtype=torch.float64)
            lpi = w - w.logsumexp(0)
            T64, T264, st64, lgn = _estep64(X, mu, lpi, sigma)
            f = lambda t: t.float().to(dev).contiguous()
            T, T2, st = _lib.gmm_estep(f(X), f(mu), f(lpi / math.log(2)), f((mu * mu).sum(-1)), sigma, lgn, True)
            st = st.cpu().double()
            errs = [float((st[:, k] - st64[:, k]).norm() / st64[:, k].norm()) for k in range(D + 4)]
            print(json.dumps({"N": N, "C": C, "sigma": sigma, "uniform": uniform,
                              "T": float((T.cpu().double() - T64).norm() / T64.norm()),
                              "slots": ["%.1e" % e for e in errs]}), flush=True)


if __name__ == "__main__":
    main()
