"""Which torch ops (by Python call site) the 2k-point PSR iteration issues -- the host floor's
kernel count (tools/host_floor_timeline.py: ~196 device kernels per L-BFGS closure, a quarter
of them buffer copies).  a dispatch-mode counter over one iteration after two warm-up ones, ops
grouped by their top Python frames in this repository, sorted by call count.

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
    import collections
    import traceback
    from torch.utils._python_dispatch import TorchDispatchMode
    cnt = collections.Counter()
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

    class Count(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            fr = [f for f in traceback.extract_stack()[:-2] if f.filename.startswith(root)
                  or "torch/optim" in f.filename]
            site = " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in fr[::-1][:a.frames])
            cnt[(str(func.overloadpacket), site)] += 1
            return func(*args, **(kwargs or {}))

    with Count():
        workloads.psr_iteration(psr)
    torch.cuda.synchronize()
    tot = collections.Counter()
    for (op, _), c in cnt.items():
        tot[op] += c
    print("op totals:", tot.most_common(40))
    for (op, site), c in cnt.most_common(a.top):
        print(f"{c:5d} {op:28s} {site}")

if __name__ == "__main__":
    main()
