"""A/B of the centred-expansion reductions (red_alg 1) against the generic skeleton (red_alg 0)
on one GPU, alternating in one process: KRed / GradKRed at M = N (x = y, the north_star's
kernel sum) and the external-point forward, HIP events on the launch stream, best of reps.

    python tools/cx_ab.py [--sizes 20000,50000,100000,200000] [--reps 7] [--out file.json]
    python tools/cx_ab.py --shapes 100000:5000,20000:20000 (rows:columns; KRed and the
        external-point forward with rows = external points, columns = support points)
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def timed(fn, reps):
    st = torch.cuda.current_stream()
    fn()
    best = None
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        fn()
        e1.record(st)
        e1.synchronize()
        ms = e0.elapsed_time(e1)
        best = ms if best is None else min(best, ms)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="20000,50000,100000,200000")
    ap.add_argument("--shapes", default=None)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    from difficp_amd import _lib as L
    dev = torch.device("cuda:0")
    rows = []
    if args.shapes:
        shapes = [tuple(int(v) for v in s.split(":")) for s in args.shapes.split(",")]
    else:
        shapes = [(int(s), int(s)) for s in args.sizes.split(",")]
    for Mr, M in shapes:
        g = torch.Generator().manual_seed(M)
        x = torch.rand(M, 3, generator=g).to(dev)
        b = (0.01 * torch.randn(M, 3, generator=g)).to(dev)
        xr = x if Mr == M else torch.rand(Mr, 3, generator=g).to(dev)
        xe = torch.rand(Mr, 3, generator=g).to(dev)
        cases = {"KRed": lambda: L.gauss_red(L.KRED, xr, x, 0.1, b=b),
                 "ode_ext_fwd(eta=0,div)": lambda: L.ode_ext_fwd(xe, x, b, 0.1, 0.0, True)}
        if not args.shapes:
            cases.update({"GradKRed": lambda: L.gauss_red(L.GRADK, x, x, 0.1),
                          "ode_ext_fwd(eta=1e-3,div)": lambda: L.ode_ext_fwd(xe, x, b, 0.1, 1e-3, True)})
        for name, fn in cases.items():
            res = {}
            for alg in (0, 2, 0, 2):   # 2: centred path forced whatever the size
                L.set_option("red_alg", alg)
                ms = timed(fn, args.reps)
                res[alg] = min(res.get(alg, 1e9), ms)
            L.set_option("red_alg", 1)
            row = {"op": name, "rows": Mr, "cols": M, "generic_ms": round(res[0], 4),
                   "centred_ms": round(res[2], 4), "speedup": round(res[0] / res[2], 3),
                   "centred_Tpair_s": round(Mr * M / res[2] / 1e9, 3),
                   "generic_Tpair_s": round(Mr * M / res[0] / 1e9, 3)}
            rows.append(row)
            print(json.dumps(row), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
