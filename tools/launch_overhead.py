"""Host cost of one library call through the Python wrappers (diff-icp_amd/_lib.py): a loop
of small euler_step / euler_adjoint_step calls (M = 512: device work of a few microseconds, so
the loop runs at the host's issue rate), wall time per call, plus a cProfile of the same loop.

    python tools/launch_overhead.py [--calls 2000]
"""
import argparse
import cProfile
import io
import json
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=2000)
    ap.add_argument("--M", type=int, default=512)
    args = ap.parse_args()
    from difficp_amd import _lib as L
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(0)
    q = torch.rand(args.M, 3, generator=g).to(dev)
    p = (0.01 * torch.randn(args.M, 3, generator=g)).to(dev)
    a = torch.randn(args.M, 3, generator=g).to(dev)
    b = torch.randn(args.M, 3, generator=g).to(dev)
    gd = torch.full((1,), 0.3, device=dev)

    def fwd():
        return L.euler_step(q, p, 0.1, 0.0, 0.1, True)

    def bwd():
        return L.euler_adjoint_step(q, p, a, b, gd, 0.1, 0.0, 0.1)

    out = {}
    for name, fn in (("euler_step", fwd), ("euler_adjoint_step", bwd)):
        for _ in range(50):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.calls):
            fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        out[name] = {"host_us_per_call": round((t1 - t0) / args.calls * 1e6, 2),
                     "wall_us_per_call": round((t2 - t0) / args.calls * 1e6, 2)}
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(500):
            fn()
        pr.disable()
        torch.cuda.synchronize()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(12)
        print(f"== {name}\n" + s.getvalue(), file=sys.stderr)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
