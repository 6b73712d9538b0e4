"""A/B of the symmetric VJP's column groups per workgroup (dicp_set_option "sym_L") at 100k,
alternating in one process, HIP events, the divergence-row adjoint step."""
import json, os, sys, torch
sys.path.insert(0, os.getcwd())
from difficp_amd import _lib
dev = torch.device("cuda:0")
M = 100000
g = torch.Generator().manual_seed(0)
q = torch.rand(M, 3, generator=g).to(dev); p = (0.01 * torch.randn(M, 3, generator=g)).to(dev)
ga = torch.randn(M, 3, generator=g).to(dev); gb = torch.randn(M, 3, generator=g).to(dev)
gd = torch.ones(1, device=dev); zs = torch.empty_like(q)
_lib.euler_step(q, p, 0.1, 0.0, 0.1, True, zs_out=zs)
fn = lambda: _lib.euler_adjoint_step(q, p, ga, gb, gd, 0.1, 0.0, 0.1, zs=zs)
st = torch.cuda.current_stream()
res = {}
Ls = tuple(int(v) for v in os.environ.get("SYM_LS", "4,6,8,3").split(","))
for L in Ls:
    _lib.set_option("sym_L", L); fn()
torch.cuda.synchronize()
for _ in range(4):
    for L in Ls:
        _lib.set_option("sym_L", L)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(4): fn()
        e1.record(st); e1.synchronize()
        res.setdefault(L, []).append(round(e0.elapsed_time(e1) / 4, 4))
print(json.dumps({str(k): sorted(v) for k, v in res.items()}))
