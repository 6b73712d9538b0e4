"""Symmetric forward, 4 vs 8 rows per lane (dicp_set_option "sym_fwd_rows"), at the bench's
point counts: the Euler step with divergence rows (the shooting's fused step) and the plain
pass with the Hamiltonian rows, alternating in one process, best of 3 passes.

    python tools/probes/fwd8_ab.py [M ...]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from difficp_amd import _lib  # noqa: E402

dev = torch.device("cuda:0")
st = torch.cuda.current_stream()
Ms = [int(a) for a in sys.argv[1:]] or [60000, 80000, 100000, 120000, 150000, 200000]
_lib.set_option("fwd_alg", 5)      # the symmetric forward whatever the size
for M in Ms:
    g = torch.Generator().manual_seed(M)
    q = torch.rand(M, 3, generator=g).to(dev)
    p = (0.01 * torch.randn(M, 3, generator=g)).to(dev)
    zs = torch.empty_like(q)
    fns = {"step_zs": lambda: _lib.euler_step(q, p, 0.1, 0.0, 0.1, True, zs_out=zs),
           "fwd_h": lambda: _lib.ode_self_fwd(q, p, 0.1, 0.0, True, want_h=True)}
    reps = max(3, int(3e10 / (M * M)))
    row = {"M": M}
    for name, fn in fns.items():
        best = {}
        for _ in range(3):
            for rows, L in ((4, 0), (8, 0), (8, 1), (8, 2)):
                _lib.set_option("sym_fwd_rows", rows)
                _lib.set_option("sym_L", L)
                fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(reps):
                    fn()
                e1.record(st)
                e1.synchronize()
                best[(rows, L)] = min(best.get((rows, L), 1e9), e0.elapsed_time(e1) / reps)
        _lib.set_option("sym_L", 0)
        row[name] = {f"rows{r}_L{L}_ms": round(v, 4) for (r, L), v in best.items()}
    _lib.set_option("sym_fwd_rows", 0)
    print(json.dumps(row), flush=True)
_lib.set_option("fwd_alg", 2)
