"""Row pairs per thread (dicp_set_option "pk_rp" 1 vs 2) for the packed external-point passes
and the packed KRed (ext_pk.hpp) at the shapes they run at (rows = external / data points,
columns = support points; below the centred sizes), alternating in one process."""
import json
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from difficp_amd import _lib  # noqa: E402

dev = torch.device("cuda:0")
st = torch.cuda.current_stream()
_lib.set_option("red_alg", 0)   # keep KRed / ext forward on the packed kernels
for N, M in [(100000, 2000), (100000, 10000), (50000, 20000), (40000, 40000), (20000, 20000)]:
    g = torch.Generator().manual_seed(N + M)
    x = torch.rand(N, 3, generator=g).to(dev)
    q = torch.rand(M, 3, generator=g).to(dev)
    p = (0.01 * torch.randn(M, 3, generator=g)).to(dev)
    gvx = torch.randn(N, 3, generator=g).to(dev)
    gdiv = torch.ones(1, device=dev)
    gq = torch.zeros(M, 3, device=dev)
    gp = torch.zeros(M, 3, device=dev)
    fns = {"ext_fwd": lambda: _lib.ode_ext_fwd(x, q, p, 0.1, 0.0, True),
           "ext_bwd": lambda: _lib.ode_ext_bwd(x, q, p, gvx, gdiv, 0.1, 0.0, gq, gp),
           "kred": lambda: _lib.gauss_red(_lib.KRED, x, q, 0.1, b=p)}
    reps = max(3, int(2e10 / (N * M)))
    row = {"rows": N, "cols": M}
    for name, fn in fns.items():
        best = {}
        for _ in range(3):
            for rp in (1, 2):
                _lib.set_option("pk_rp", rp)
                fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(reps):
                    fn()
                e1.record(st)
                e1.synchronize()
                best[rp] = min(best.get(rp, 1e9), e0.elapsed_time(e1) / reps)
        row[name] = {"rp1_ms": round(best[1], 4), "rp2_ms": round(best[2], 4),
                     "rp2_speedup": round(best[1] / best[2], 4)}
    _lib.set_option("pk_rp", 0)
    print(json.dumps(row), flush=True)
_lib.set_option("red_alg", 1)
