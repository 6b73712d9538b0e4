"""Host-side floor of one diff-ICP iteration: per L-BFGS closure wall time at a small point count
(device work negligible) next to the default size, on one GPU.  What does not shrink with the
number of ranks of a row split.

    python tools/host_floor.py [--sizes 2000 100000] [--iters 2]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from difficp_amd import workloads  # noqa: E402
from difficp_amd.core import shooting  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", type=int, nargs="+", default=[2000, 100000])
    ap.add_argument("--iters", type=int, default=2)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    counts = {"fwd": 0}
    orig = shooting.ShootFn.forward

    def counting(*args, **kw):
        counts["fwd"] += 1
        return orig(*args, **kw)

    shooting.ShootFn.forward = staticmethod(counting)
    for N in a.sizes:
        psr = workloads.build_two_set(N, dev, seed=0)
        workloads.psr_iteration(psr)
        torch.cuda.synchronize()
        counts["fwd"] = 0
        t0 = time.perf_counter()
        for _ in range(a.iters):
            workloads.psr_iteration(psr)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.iters
        n = counts["fwd"] / a.iters
        print(json.dumps({"N": N, "ms_per_iter": round(dt * 1e3, 2), "shoots_per_iter": n,
                          "ms_per_shoot": round(dt * 1e3 / max(n, 1), 3)}), flush=True)


if __name__ == "__main__":
    main()
