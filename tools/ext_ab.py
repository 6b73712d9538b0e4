"""A/B of the external-point passes: packed scaled-coordinate kernels (ext_alg 1,
csrc/ext_pk.hpp) against the generic scalar kernels (ext_alg 0), with the centred path off
(red_alg 0) so both run at every size; alternating in one process, HIP events on the launch
stream, best of reps.

    python tools/ext_ab.py [--shapes 100000:5000,...] [--reps 7] [--out file.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from cx_ab import timed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="100000:2000,100000:5000,100000:20000,20000:20000,50000:50000,5000:100000")
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    from difficp_amd import _lib as L
    dev = torch.device("cuda:0")
    L.set_option("red_alg", 0)
    rows = []
    for N, M in (tuple(int(v) for v in s.split(":")) for s in args.shapes.split(",")):
        g = torch.Generator().manual_seed(N + M)
        x = torch.rand(N, 3, generator=g).to(dev)
        a = torch.randn(N, 3, generator=g).to(dev)
        q = torch.rand(M, 3, generator=g).to(dev)
        p = (0.01 * torch.randn(M, 3, generator=g)).to(dev)
        gq, gp = torch.zeros_like(q), torch.zeros_like(q)
        gd = torch.full((1,), 0.3, device=dev)
        cases = {"ode_ext_fwd(eta=0,div)": lambda: L.ode_ext_fwd(x, q, p, 0.1, 0.0, True),
                 "ode_ext_bwd(eta=0)": lambda: L.ode_ext_bwd(x, q, p, a, gd, 0.1, 0.0, gq, gp)}
        for name, fn in cases.items():
            res = {}
            for alg in (0, 1, 0, 1):
                L.set_option("ext_alg", alg)
                res[alg] = min(res.get(alg, 1e9), timed(fn, args.reps))
            L.set_option("ext_alg", 1)
            row = {"op": name, "N_ext": N, "M_support": M, "generic_ms": round(res[0], 4),
                   "packed_ms": round(res[1], 4), "speedup": round(res[0] / res[1], 3),
                   "packed_Tpair_s": round(N * M / res[1] / 1e9 * (2 if "bwd" in name else 1), 3)}
            rows.append(row)
            print(json.dumps(row), flush=True)
    L.set_option("red_alg", 1)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
