"""Precision of the pair kernels against float64 as the point cloud's extent and offset grow
(in units of sigma): the self ODE forward (scaled coordinates, shifted to the first support
point), the symmetric VJP, KRed and the external-point forward on every path.  256 sampled rows
against float64 sums over all points (tests/fullsize_ref.py), inputs rounded to float32 first.

    python tools/probes/extent_precision.py [--M 20000]
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

import fullsize_ref as F  # noqa: E402


def rel(a, b):
    a = a.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-300))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=20000)
    args = ap.parse_args()
    from difficp_amd import _lib as L
    dev = torch.device("cuda:0")
    sig = 0.1
    M = args.M
    out = []
    for E, off in [(10, 0), (30, 0), (100, 0), (300, 0), (1000, 0), (10, 1000), (10, 10000), (100, 1000)]:
        g = torch.Generator().manual_seed(E + off)
        # uniform cloud of extent E sigma, density kept at ~M points per (E sigma)^3
        q = (E * sig * torch.rand(M, 3, generator=g, dtype=torch.float64) + off * sig).float().double()
        p = (0.01 * torch.randn(M, 3, generator=g, dtype=torch.float64)).float().double()
        a = torch.randn(M, 3, generator=g, dtype=torch.float64).float().double()
        b = torch.randn(M, 3, generator=g, dtype=torch.float64).float().double()
        sub = torch.randperm(M, generator=g)[:256].to(dev)
        qd, pd, ad, bd = (t.to(dev) for t in (q, p, a, b))
        qf, pf, af, bf = (t.float() for t in (qd, pd, ad, bd))
        v, mG, gg, _ = L.ode_self_fwd(qf, pf, sig, 0.0, True)
        v64, mG64, g64, _ = F.self_terms(qd[sub], pd[sub], qd, pd, sig, 0.0)
        gq, gp = L.ode_self_bwd(qf, pf, af, bf, torch.full((1,), 0.3, device=dev), sig, 0.0)
        gq64, gp64 = F.self_vjp_subset(qd, pd, ad, bd, 0.3, sub, sig, 0.0)
        row = {"extent_sigma": E, "offset_sigma": off,
               "fwd_v": rel(v[sub], v64), "fwd_mG": rel(mG[sub], mG64), "fwd_g": rel(gg[sub], g64),
               "vjp_gq": rel(gq[sub], gq64), "vjp_gp": rel(gp[sub], gp64)}
        kr64, _ = F.ext_terms(qd[sub], qd, pd, sig, 0.0)
        xe = (qd + 0.3 * sig).float()
        vx64, gx64 = F.ext_terms(xe.double()[sub], qd, pd, sig, 0.0)
        # the reference's own fp32 arithmetic (torch, chunked) on the same inputs: the parity
        # criterion's yardstick, max(1e-5, 2 x this)
        v32, mG32, g32, _ = F.self_terms(qf[sub], pf[sub], qf, pf, sig, 0.0)
        row.update({"oracle32_v": rel(v32, v64), "oracle32_mG": rel(mG32, mG64), "oracle32_g": rel(g32, g64)})
        for name, opts in (("packed", (0, 1)), ("generic", (0, 0)), ("centred", (2, 1))):
            L.set_option("red_alg", opts[0])
            L.set_option("ext_alg", opts[1])
            kr = L.gauss_red(L.KRED, qf, qf, sig, b=pf)
            vx, gx = L.ode_ext_fwd(xe, qf, pf, sig, 0.0, True)
            row[f"kred_{name}"] = rel(kr[sub], kr64)
            row[f"extfwd_v_{name}"] = rel(vx[sub], vx64)
            row[f"extfwd_g_{name}"] = rel(gx[sub], gx64)
        L.set_option("red_alg", 1)
        L.set_option("ext_alg", 1)
        row = {k: (round(v_, 9) if isinstance(v_, float) else v_) for k, v_ in row.items()}
        out.append(row)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
