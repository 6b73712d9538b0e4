"""The E-step's bound shift against the sampled shift on the exact two-set workload's own EM
(50k x 50k points, the built problem's points and components) at the GMM's sigma and smaller
ones: one hinted E-step (the hint: the same call's T2) with option lse_bound 0 and 1 -- the
relative differences of T, T2 and the stats, and NaN counts.  One JSON line per sigma.

    python tools/probes/estep_workload_diff.py
"""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from difficp_amd import _lib, workloads  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    N = int(os.environ.get("EW_N", "50000"))
    psr = workloads.build_two_set(N, dev, seed=0, version="logdet",
                                  v2p_args={"version": "ridge_keops", "alpha": 1e-3})
    G = psr.GMMi[0]
    X = psr.x1[0, 0].detach().contiguous()
    mu = G.mu.contiguous()
    C, D = mu.shape
    rel = lambda a, b: float((a - b).norm() / b.norm().clamp_min(1e-30))
    for sig in (G.sigma, 0.05, 0.02, 0.01, 0.005):
        lpi = torch.full((C,), -math.log(C), device=dev)
        lgn = D * (math.log(sig) + 0.5 * math.log(2 * math.pi))
        outs = {}
        _lib.set_option("lse_bound", 0)
        w2, m2 = (lpi / math.log(2)).contiguous(), (mu * mu).sum(-1)
        hint = _lib.gmm_estep(X, mu, w2, m2, sig, lgn, True)[1]   # the hinted calls' hint: T2
        for b in (0, 1):
            _lib.set_option("lse_bound", b)
            outs[b] = _lib.gmm_estep(X, mu, w2, m2, sig, lgn, True, hint=hint)
        (T0, T20, st0), (T1, T21, st1) = outs[0], outs[1]
        # float64 rows (the first 2000) of the same E-step (GMM.py:260-282; tests/test_gpu_em.py
        # _estep64): which shift is nearer
        R = 2000
        Xd, mud, lpid = X[:R].double(), mu.double(), lpi.double()
        D2 = ((Xd[:, None, :] - mud[None]) ** 2).sum(-1)
        t = lpid[None] - D2 / (2 * sig ** 2) - lgn
        T64 = t.logsumexp(1)
        lg = t - T64[:, None]
        gam = lg.exp()
        st64 = torch.cat([gam @ mud, (gam * (mud * mud).sum(-1)[None]).sum(1, keepdim=True),
                          (gam * lg).sum(1, keepdim=True), (gam * lpid[None]).sum(1, keepdim=True),
                          (gam * D2).sum(1, keepdim=True)], 1)
        vs64 = {b: [rel(outs[b][2][:R, k].double(), st64[:, k]) for k in range(st64.shape[1])] for b in (0, 1)}
        print(json.dumps({"sigma": sig, "T_rel": rel(T1, T0), "T2_rel": rel(T21, T20),
                          "stats_rel": [rel(st1[:, k], st0[:, k]) for k in range(st0.shape[1])],
                          "stats_vs_fp64_sampled": vs64[0], "stats_vs_fp64_bound": vs64[1],
                          "T_vs_fp64": [rel(outs[b][0][:R].double(), T64) for b in (0, 1)],
                          "nan0": int(torch.isnan(T0).sum()), "nan1": int(torch.isnan(T1).sum()),
                          "T_maxabs": float((T1 - T0).abs().max())}), flush=True)
    _lib.set_option("lse_bound", 1)


if __name__ == "__main__":
    main()
