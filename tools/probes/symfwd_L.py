"""Symmetric forward at the north_star's 100k: column groups per workgroup (sym_L) against rows
per lane (sym_fwd_rows 4 / 8) -- the grid's fill of the chip's resident workgroup slots
(4-row: 3 workgroups of 4 waves per CU; 8-row: 2).  The fused Euler step with divergence rows
(the shooting's step), alternated in one process, best of 3 passes.

    python tools/probes/symfwd_L.py [M ...]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from difficp_amd import _lib  # noqa: E402

dev = torch.device("cuda:0")
st = torch.cuda.current_stream()
Ms = [int(a) for a in sys.argv[1:]] or [100000]
for M in Ms:
    g = torch.Generator().manual_seed(M)
    q = torch.rand(M, 3, generator=g).to(dev)
    p = (0.01 * torch.randn(M, 3, generator=g)).to(dev)
    zs = torch.empty_like(q)
    fn = lambda: _lib.euler_step(q, p, 0.1, 0.0, 0.1, True, zs_out=zs)
    reps = max(3, int(3e10 / (M * M)))
    cfgs = [(4, L) for L in (0, 2, 4)] + [(6, L) for L in (0, 1, 2, 3, 4)] + [(8, L) for L in (1, 2)]
    if os.environ.get("SYMFWD_CFGS"):   # e.g. "4:0,6:0,8:0" (rows:L)
        cfgs = [tuple(int(v) for v in c.split(":")) for c in os.environ["SYMFWD_CFGS"].split(",")]
    best = {}
    for _ in range(3):
        for rows, L in cfgs:
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
    _lib.set_option("sym_fwd_rows", 0)
    print(json.dumps({"M": M, **{f"rows{r}_L{L}_ms": round(v, 4) for (r, L), v in best.items()}}), flush=True)
