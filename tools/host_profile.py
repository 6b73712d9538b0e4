"""cProfile of one diff-ICP iteration at a small point count (device work negligible, so the
profile is the host path: L-BFGS, autograd, wrappers, launches), on one GPU.

    python tools/host_profile.py [--N 2000] [--workload two_set|atlas] [--top 45]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from difficp_amd import workloads  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=2000)
    ap.add_argument("--top", type=int, default=45)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    psr = workloads.build_two_set(a.N, dev, seed=0)
    workloads.psr_iteration(psr)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    workloads.psr_iteration(psr)
    torch.cuda.synchronize()
    pr.disable()
    for key in ("tottime", "cumulative"):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(a.top)
        print(s.getvalue())


if __name__ == "__main__":
    main()
