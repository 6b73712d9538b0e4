"""Per-rank kernel time of the row split (core/rowsplit.py) at W ranks, measured on ONE GPU:
every part's forward row slice (euler_step_rows) and VJP pair subset (ode_self_bwd_part) is
timed alone, HIP-event timed, and compared with the unsplit pass / W.  The slowest part sets a
rank's step time at W GPUs, so W * max(part) / full is the compute-side strong-scaling loss
(collectives and the replicated host work come on top)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from difficp_amd import _lib  # noqa: E402


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


def rows(M, W, r):
    base, rem = divmod(M, W)
    return r * base + min(r, rem), base + (1 if r < rem else 0)


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
        reps = max(2, int(2e10 / (M * M)))
        # the variants the timed Euler steps run: forward writing the divergence rows zs, the
        # adjoint reusing them (shooting.ShootFn)
        zs = torch.empty_like(q)
        full_f = timeit(lambda: _lib.euler_step(q, p, 0.1, 0.0, 0.1, True, zs_out=zs), reps)
        full_b = timeit(lambda: _lib.euler_adjoint_step(q, p, a, b, gd, 0.1, 0.0, 0.1, zs=zs), reps)
        for W in (2, 4, 8):
            tf, tb = [], []
            for r in range(W):
                r0, n = rows(M, W, r)
                zl = zs[r0:r0 + n]
                tf.append(timeit(lambda: _lib.euler_step_rows(q, p, r0, n, 0.1, 0.0, 0.1, True,
                                                              zs_out=zl), reps))
                tb.append(timeit(lambda: _lib.ode_self_bwd_part(q, p, a, b, gd, 0.1, 0.0, r, W, zs=zl,
                                                                zrow0=r0), reps))
            rec = {"M": M, "W": W, "fwd_full_ms": round(full_f, 4), "bwd_full_ms": round(full_b, 4),
                   "fwd_part_max_ms": round(max(tf), 4), "fwd_part_min_ms": round(min(tf), 4),
                   "bwd_part_max_ms": round(max(tb), 4), "bwd_part_min_ms": round(min(tb), 4),
                   "fwd_eff": round(full_f / (W * max(tf)), 4), "bwd_eff": round(full_b / (W * max(tb)), 4)}
            print(json.dumps(rec), flush=True)
            out.append(rec)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/part_timing.json", "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
