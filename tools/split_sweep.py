"""Sweep of the column-split count of the packed forward (euler_step, eta = 0) and of the
symmetric VJP's chunk length L, HIP-event timed on one box: is the default geometry
(launch.hpp num_splits_cap / lddmm_sym.hpp sym_geom) the fastest at the bench sizes?"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from difficp_amd import _lib  # noqa: E402
from part_timing import timeit  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    out = []
    for M in (50000, 100000, 200000):
        g = torch.Generator().manual_seed(M)
        q = torch.rand(M, 3, generator=g).to(dev)
        p = (0.05 * torch.randn(M, 3, generator=g)).to(dev)
        a = torch.randn(M, 3, generator=g).to(dev)
        b = torch.randn(M, 3, generator=g).to(dev)
        gd = torch.full((1,), 0.3, device=dev)
        reps = max(3, int(3e10 / (M * M)))
        S0 = _lib.num_splits(1, M, M)
        res = {"M": M, "default_splits": S0, "fwd": {}, "bwd": {}}
        for rnd in range(2):
            for S in [0] + sorted({max(1, S0 + d) for d in (-8, -4, -2, -1, 1, 2, 4, 8, 16)} | {8, 16, 32, 48, 64}):
                _lib.set_option("force_splits", S)
                ms = timeit(lambda: _lib.euler_step(q, p, 0.1, 0.0, 0.1, True), reps)
                res["fwd"].setdefault(S, []).append(round(ms, 4))
            _lib.set_option("force_splits", 0)
            for L in (0, 1, 2, 3, 4, 6, 8):
                _lib.set_option("sym_L", L)
                ms = timeit(lambda: _lib.ode_self_bwd(q, p, a, b, gd, 0.1, 0.0), reps)
                res["bwd"].setdefault(L, []).append(round(ms, 4))
            _lib.set_option("sym_L", 0)
        best_f = min(res["fwd"].items(), key=lambda kv: min(kv[1]))
        best_b = min(res["bwd"].items(), key=lambda kv: min(kv[1]))
        res["best_fwd"], res["best_bwd"] = best_f, best_b
        print(json.dumps(res), flush=True)
        out.append(res)
    with open("gpurun_out/split_sweep.json", "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
