"""Which torch ops (by Python call site) the 2k-point PSR iteration issues -- the host floor's
kernel count (tools/host_floor_timeline.py: ~196 device kernels per L-BFGS closure, a quarter
of them buffer copies).  torch.profiler over one iteration after a warm-up one, CPU activity
only, ops grouped by their top Python frames, sorted by call count.

    python tools/probes/host_ops.py [--N 2000] [--top 40] [--frames 4]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from difficp_amd import workloads  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=2000)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--frames", type=int, default=4)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    psr = workloads.build_two_set(a.N, dev, seed=0)
    workloads.psr_iteration(psr)
    workloads.psr_iteration(psr)
    torch.cuda.synchronize()
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU], with_stack=True) as prof:
        workloads.psr_iteration(psr)
        torch.cuda.synchronize()
    ka = prof.key_averages(group_by_stack_n=a.frames)
    rows = [e for e in ka if e.key.startswith("aten::") and e.stack]
    rows.sort(key=lambda e: -e.count)
    tot = {}
    for e in ka:
        if e.key.startswith("aten::"):
            tot[e.key] = tot.get(e.key, 0) + e.count
    print("op totals:", sorted(tot.items(), key=lambda kv: -kv[1])[:30])
    for e in rows[:a.top]:
        st = " <- ".join(s.split("/")[-1] for s in e.stack[:a.frames])
        print(f"{e.count:5d} {e.key:28s} {st}")


if __name__ == "__main__":
    main()
