"""The 2k-point PSR iteration (tools/host_floor.py's workload) under several split minimum
chunks (library option "min_chunk", default 256: at 2k columns it caps the ordered forward at
8 splits = 32 workgroups, ~20 us per pass; 64 is faster at 2k but stays forced-only, see
csrc/launch.hpp): fresh workload per measurement, settings
alternated, ms per iteration and per closure.

    python tools/probes/min_chunk_ab.py [--chunks 256 64 32] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from difficp_amd import _lib, workloads  # noqa: E402
from difficp_amd.tools import runstats  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", type=int, nargs="+", default=[256, 64, 32])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--N", type=int, default=2000)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    res = {c: [] for c in a.chunks}
    for _ in range(a.reps):
        for c in a.chunks:
            _lib.set_option("min_chunk", c)
            psr = workloads.build_two_set(a.N, dev, seed=0)
            workloads.psr_iteration(psr)
            workloads.psr_iteration(psr)
            torch.cuda.synchronize()
            s0 = runstats.snapshot()
            t0 = time.perf_counter()
            for _ in range(a.iters):
                workloads.psr_iteration(psr)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / a.iters * 1e3
            n = runstats.delta(s0).get("closures", 0) / a.iters
            res[c].append({"ms_per_iter": round(dt, 2), "closures_per_iter": n,
                           "ms_per_closure": round(dt / max(n, 1), 3)})
            print(c, res[c][-1], flush=True)
    _lib.set_option("min_chunk", 0)
    print(json.dumps({"N": a.N, "res": res,
                      "best_ms_per_iter": {c: min(r["ms_per_iter"] for r in v) for c, v in res.items()},
                      "best_ms_per_closure": {c: min(r["ms_per_closure"] for r in v) for c, v in res.items()}}),
          flush=True)


if __name__ == "__main__":
    main()
