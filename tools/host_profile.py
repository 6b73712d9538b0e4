"""cProfile of the host side of one timed PSR iteration of the C2 bench workload (where the
idle gaps of the device timeline come from).

    python tools/host_profile.py [--N 50000] > out.txt
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
    ap.add_argument("--N", type=int, default=50000)
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
    s = io.StringIO()
    st = pstats.Stats(pr, stream=s)
    st.sort_stats("tottime").print_stats(35)
    st.sort_stats("cumulative").print_stats(35)
    print(s.getvalue())


if __name__ == "__main__":
    main()
