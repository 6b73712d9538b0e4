"""cProfile of one diff-ICP iteration at a small point count on the GPU (device work
negligible): where the host floor of tools/host_floor.py goes, by own time and cumulative.

    python tools/host_profile.py [--N 2000] [--top 45] > profile.txt
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
    for _ in range(2):
        workloads.psr_iteration(psr)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    workloads.psr_iteration(psr)
    torch.cuda.synchronize()
    pr.disable()
    for key in ("tottime", "cumulative"):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).strip_dirs().sort_stats(key).print_stats(a.top)
        print(s.getvalue())


if __name__ == "__main__":
    main()
