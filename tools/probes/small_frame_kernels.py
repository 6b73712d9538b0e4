"""The atlas frame's pair passes at 20k points (C4), for a rocprofv3 kernel trace: the pair
kernels and their merges separately (the bench's live timer sees one library call).

    rocprofv3 --kernel-trace --stats -d OUT -o frame --output-format csv -- \
        python3 tools/probes/small_frame_kernels.py
"""
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from difficp_amd import _lib  # noqa: E402

dev = torch.device("cuda:0")
M = int(os.environ.get("M", "20000"))
reps = int(os.environ.get("REPS", "50"))
g = torch.Generator().manual_seed(M)
q = torch.rand(M, 3, generator=g).to(dev)
p = (0.01 * torch.randn(M, 3, generator=g)).to(dev)
lq = torch.randn(M, 3, generator=g).to(dev)
lp = torch.randn(M, 3, generator=g).to(dev)
gd = torch.full((1,), 0.3, device=dev)
zs = torch.empty_like(q)
qn, pn = torch.empty_like(q), torch.empty_like(q)
_lib.euler_step(q, p, 0.1, 0.0, 0.1, True, zs_out=zs)
for _ in range(reps):
    _lib.euler_step(q, p, 0.1, 0.0, 0.1, True, q_out=qn, p_out=pn, zs_out=zs)
    _lib.euler_adjoint_step(q, p, lq, lp, gd, 0.1, 0.0, 0.1, zs=zs)
torch.cuda.synchronize()
print("done", M, reps)
