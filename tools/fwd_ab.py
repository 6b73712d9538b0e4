"""A/B of the eta = 0 fused ODE forward variants (fwd_alg 2 = packed-FP32 VALU rows,
3 = matrix-core channel contraction) on one box, alternating, HIP-event timed."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from difficp_amd import _lib  # noqa: E402
from difficp_amd.core.shooting import spatial_order  # noqa: E402


def timeit(fn, reps):
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record(st)
    for _ in range(reps):
        fn()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    dev = torch.device("cuda:0")
    for M in (20000, 50000, 100000, 200000):
        g = torch.Generator().manual_seed(M)
        q = torch.rand(M, 3, generator=g).to(dev)
        p = (0.05 * torch.randn(M, 3, generator=g)).to(dev)
        reps = max(3, int(4e10 / (M * M)))
        order = spatial_order(q)   # what LDDMMModel.Shoot passes
        res = {}
        outs = {}
        for rnd in range(2):
            for alg in (2, 3, 4):
                _lib.set_option("fwd_alg", alg)
                ms = timeit(lambda: _lib.euler_step(q, p, 0.1, 0.0, 0.1, True, order=order), reps)
                res.setdefault(alg, []).append(ms)
                outs[alg] = _lib.euler_step(q, p, 0.1, 0.0, 0.1, True, order=order)
        _lib.set_option("fwd_alg", 2)
        a, b, c = min(res[2]), min(res[3]), min(res[4])
        d = [float((x - y).norm() / y.norm()) for x, y in zip(outs[4], outs[2])]
        print(f"M={M}: pk {a:.3f} ms ({M * M / a / 1e9:.2f} Tpair/s)  mfma {b:.3f} ms ({a / b:.2f}x)  "
              f"sym-pk {c:.3f} ms ({M * M / c / 1e9:.2f} Tpair/s, {a / c:.2f}x)  sym-pk vs pk rel diff q/p/g "
              f"{d[0]:.1e} {d[1]:.1e} {d[2]:.1e}", flush=True)


if __name__ == "__main__":
    main()
