"""A few KRed 100k x 100k launches on the centred path (for rocprofv3 --kernel-trace --stats)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from difficp_amd import _lib as L  # noqa: E402

M = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
g = torch.Generator().manual_seed(1)
x = torch.rand(M, 3, generator=g).cuda()
b = (0.01 * torch.randn(M, 3, generator=g)).cuda()
for _ in range(10):
    L.gauss_red(L.KRED, x, x, 0.1, b=b)
torch.cuda.synchronize()
