"""Row pairs per thread of the packed fused forward (dicp_set_option "pk_rp" 1 vs 2) across
sizes: the Euler step with divergence rows (the shooting's hot variant) and the mG-less last
step, alternating in one process, HIP events, best of reps -- the data behind the automatic
threshold (packed.hpp DICP_PK_RP2_ROWS)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from difficp_amd import _lib  # noqa: E402

dev = torch.device("cuda:0")
st = torch.cuda.current_stream()
out = []
RPS = tuple(int(v) for v in os.environ.get("RPS", "1,2").split(","))
for M in [int(v) for v in os.environ.get("SIZES", "20000,30000,40000,50000,70000,100000,200000").split(",")]:
    g = torch.Generator().manual_seed(M)
    q = torch.rand(M, 3, generator=g).to(dev)
    p = (0.01 * torch.randn(M, 3, generator=g)).to(dev)
    zs = torch.empty_like(q)
    fns = {"step_zs": lambda: _lib.euler_step(q, p, 0.1, 0.0, 0.1, True, zs_out=zs),
           "step_nog": lambda: _lib.euler_step(q, p, 0.1, 0.0, 0.1, True, want_p=False)}
    reps = max(2, int(3e10 / (M * M)))
    row = {"M": M}
    for name, fn in fns.items():
        best = {}
        for _ in range(3):
            for rp in RPS:
                _lib.set_option("pk_rp", rp)
                fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(reps):
                    fn()
                e1.record(st)
                e1.synchronize()
                best[rp] = min(best.get(rp, 1e9), e0.elapsed_time(e1) / reps)
        row[name] = {f"rp{rp}_ms": round(best[rp], 4) for rp in RPS}
        row[name].update({f"rp{rp}_speedup": round(best[1] / best[rp], 4) for rp in RPS if rp > 1})
    _lib.set_option("pk_rp", 0)
    print(json.dumps(row), flush=True)
    out.append(row)
