"""Pair-once centred KRed (sym_red 2, csrc/sym_cx.hpp) with 4 / 8 rows per lane
(sym_red_rows) and column groups per workgroup L (sym_L; 0 = automatic) vs the ordered
centred KRed (sym_red 0, cx_kernel) for x = y, and the ordered kernel for x != y, at 50k /
100k / 200k 3D points (sigma 0.1, uniform cube: the bench's kernel-sum probe), alternating in
one process, best of 3 passes.

    python tools/probes/sym_red_ab.py [rows:L ...]     (default 4:0 8:0)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from difficp_amd import _lib  # noqa: E402

dev = torch.device("cuda:0")
st = torch.cuda.current_stream()
cfgs = [tuple(int(v) for v in a.split(":")) for a in sys.argv[1:]] or [(4, 0), (8, 0)]


def timed(fn, reps):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        fn()
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


for M in (50000, 100000, 200000):
    g = torch.Generator().manual_seed(1)
    x = torch.rand(M, 3, generator=g).to(dev)
    b = (0.01 * torch.randn(M, 3, generator=g)).to(dev)
    y = torch.rand(M, 3, generator=g).to(dev)
    reps = max(3, int(4e10 / (M * M)))
    best = {}
    for _ in range(3):
        for rows, L in cfgs:
            _lib.set_option("sym_red", 2)
            _lib.set_option("sym_red_rows", rows)
            _lib.set_option("sym_L", L)
            k = f"sym_r{rows}_L{L}"
            best[k] = min(best.get(k, 1e9), timed(lambda: _lib.gauss_red(_lib.KRED, x, x, 0.1, b=b), reps))
        _lib.set_option("sym_L", 0)
        _lib.set_option("sym_red_rows", 0)
        _lib.set_option("sym_red", 0)
        best["cx_xx"] = min(best.get("cx_xx", 1e9), timed(lambda: _lib.gauss_red(_lib.KRED, x, x, 0.1, b=b), reps))
        best["cx_xy"] = min(best.get("cx_xy", 1e9), timed(lambda: _lib.gauss_red(_lib.KRED, x, y, 0.1, b=b), reps))
    _lib.set_option("sym_red", 1)
    best["auto_xx"] = timed(lambda: _lib.gauss_red(_lib.KRED, x, x, 0.1, b=b), reps)
    bound = max(M * M * 15 / 157.3e12, M * M / (64 / 8 * 1024 * 2.4e9)) * 1e3
    row = {"M": M, **{k: round(v, 4) for k, v in best.items()},
           "compute_bound_ms": round(bound, 4),
           **{f"frac_{k}": round(bound / v, 4) for k, v in best.items()}}
    print(json.dumps(row), flush=True)
