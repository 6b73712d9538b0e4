"""Packed ordered forward (fwd_alg 2, default) vs the packed symmetric pair-once forward
(fwd_alg 4) at 100k, with the symmetric kernel's column groups per workgroup swept (sym_L);
alternating in one process, HIP events, best of reps.  ode_self_fwd(eta 0, divergence)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from difficp_amd import _lib  # noqa: E402

dev = torch.device("cuda:0")
M = int(os.environ.get("M", "100000"))
g = torch.Generator().manual_seed(0)
q = torch.rand(M, 3, generator=g).to(dev)
p = (0.01 * torch.randn(M, 3, generator=g)).to(dev)
fn = lambda: _lib.ode_self_fwd(q, p, 0.1, 0.0, True)
cases = [(2, 0), (4, 2), (4, 4), (4, 8), (4, 0)]
res = {}
ref = None
for alg, L in cases:
    _lib.set_option("fwd_alg", alg)
    _lib.set_option("sym_L", L)
    out = fn()
    if ref is None:
        ref = out
    else:
        res.setdefault(f"maxdiff_v alg{alg} L{L}", float((out[0] - ref[0]).abs().max() / ref[0].abs().max()))
st = torch.cuda.current_stream()
for _ in range(4):
    for alg, L in cases:
        _lib.set_option("fwd_alg", alg)
        _lib.set_option("sym_L", L)
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(3):
            fn()
        e1.record(st)
        e1.synchronize()
        k = f"alg{alg} L{L}"
        res[k] = min(res.get(k, 1e9), round(e0.elapsed_time(e1) / 3, 4))
_lib.set_option("fwd_alg", 2)
_lib.set_option("sym_L", 0)
print(json.dumps(res))
