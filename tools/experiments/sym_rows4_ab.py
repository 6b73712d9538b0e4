"""Experiment: the packed eta = 0 VJP with 4 rows per lane (256-point groups, dicp_set_option
"sym_rows4" 1) against the default 2 rows (128-point groups): agreement and time per adjoint
step (divergence-row variant, first-step b0 variant), alternating in one process."""
import json
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from difficp_amd import _lib  # noqa: E402

dev = torch.device("cuda:0")
st = torch.cuda.current_stream()
for M in [int(v) for v in os.environ.get("SIZES", "3001,50000,100000").split(",")]:
    g = torch.Generator().manual_seed(M)
    q = torch.rand(M, 3, generator=g).to(dev)
    p = (0.01 * torch.randn(M, 3, generator=g)).to(dev)
    ga = torch.randn(M, 3, generator=g).to(dev)
    gb = torch.randn(M, 3, generator=g).to(dev)
    gd = torch.ones(1, device=dev)
    zs = torch.empty_like(q)
    _lib.euler_step(q, p, 0.1, 0.0, 0.1, True, zs_out=zs)
    fns = {"adj_zs": lambda: _lib.euler_adjoint_step(q, p, ga, gb, gd, 0.1, 0.0, 0.1, zs=zs),
           "adj_b0": lambda: _lib.euler_adjoint_step(q, p, ga, None, gd, 0.1, 0.0, 0.1, zs=zs),
           "bwd": lambda: _lib.ode_self_bwd(q, p, ga, gb, gd, 0.1, 0.0)}
    row = {"M": M}
    for name, fn in fns.items():
        outs, best = {}, {}
        for v in (0, 1):
            _lib.set_option("sym_rows4", v)
            outs[v] = [t.clone() for t in fn() if isinstance(t, torch.Tensor)]
        err = max(float((a - b).norm() / b.norm()) for a, b in zip(outs[1], outs[0]))
        reps = max(2, int(3e10 / (M * M)))
        for _ in range(3):
            for v in (0, 1):
                _lib.set_option("sym_rows4", v)
                fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(reps):
                    fn()
                e1.record(st)
                e1.synchronize()
                best[v] = min(best.get(v, 1e9), e0.elapsed_time(e1) / reps)
        row[name] = {"rows2_ms": round(best[0], 4), "rows4_ms": round(best[1], 4),
                     "speedup": round(best[0] / best[1], 4), "rel_err": err}
    _lib.set_option("sym_rows4", 0)
    print(json.dumps(row), flush=True)
