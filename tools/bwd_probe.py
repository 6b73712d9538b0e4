"""Launch the symmetric VJP a few times at M points (rocprofv3 --kernel-trace A/B of library
builds via DICP_LIB_PATH)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from difficp_amd import _lib  # noqa: E402

M = int(os.environ.get("PMC_M", "50000"))
dev = torch.device("cuda:0")
torch.manual_seed(0)
q = torch.rand(M, 3, device=dev)
p = 0.01 * torch.randn(M, 3, device=dev)
a = torch.randn(M, 3, device=dev)
gd = torch.ones(1, device=dev)
for _ in range(5):
    _lib.ode_self_bwd(q, p, a, a, gd, 0.1, 0.0)
torch.cuda.synchronize()
