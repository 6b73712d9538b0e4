"""A/B of the symmetric 4-row forward (fwd_alg 5) against the packed ordered forward
(fwd_alg 6), and the automatic choice (fwd_alg 2), on the forms the shooting runs: the Euler step writing the divergence rows
(step_zs, the t >= 1 steps), the first step (ode_self_fwd with zs), the mG-less last step
(step_nog), alternating in one process, HIP events; agreement of the step outputs.

    SIZES=20000,50000,100000,200000 python tools/probes/fwd_sym4_ab.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from difficp_amd import _lib  # noqa: E402

dev = torch.device("cuda:0")
st = torch.cuda.current_stream()


def timeit(fn, reps):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        fn()
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


for M in [int(v) for v in os.environ.get("SIZES", "20000,50000,100000,200000").split(",")]:
    g = torch.Generator().manual_seed(M)
    q = torch.rand(M, 3, generator=g).to(dev)
    p = (0.01 * torch.randn(M, 3, generator=g)).to(dev)
    zs = torch.empty_like(q)
    zs0 = torch.empty_like(q)
    fns = {"step_zs": lambda: _lib.euler_step(q, p, 0.1, 0.0, 0.1, True, zs_out=zs),
           "first_zs": lambda: _lib.ode_self_fwd(q, p, 0.1, 0.0, True, zs_out=zs0),
           "step_nog": lambda: _lib.euler_step(q, p, 0.1, 0.0, 0.1, True, want_p=False)}
    reps = max(2, int(2e10 / (M * M)))
    row = {"M": M}
    for name, fn in fns.items():
        best, outs = {}, {}
        for alg in (6, 5, 2):
            _lib.set_option("fwd_alg", alg)
            outs[alg] = [t.clone() for t in fn() if isinstance(t, torch.Tensor)] + [zs.clone()]
        for _ in range(3):
            for alg in (6, 5, 2):
                _lib.set_option("fwd_alg", alg)
                best[alg] = min(best.get(alg, 1e9), timeit(fn, reps))
        _lib.set_option("fwd_alg", 2)
        err = max(float((a - b).norm() / max(float(b.norm()), 1e-30)) for a, b in zip(outs[5], outs[6]))
        row[name] = {"ordered_ms": round(best[6], 4), "sym4_ms": round(best[5], 4),
                     "auto_ms": round(best[2], 4), "speedup": round(best[6] / best[5], 4), "rel_err": err}
    print(json.dumps(row), flush=True)
