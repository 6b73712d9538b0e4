"""Launch the ordered forward (fwd_alg 0), the symmetric forward (fwd_alg 1) and the symmetric
VJP once each at M points, for per-kernel rocprofv3 PMC passes, e.g.

    rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY ... --output-format csv -d gpurun_out/pmc_sq -- python tools/pmc_fwd_ab.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from difficp_amd import _lib  # noqa: E402


def main():
    M = int(os.environ.get("PMC_M", "50000"))
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    q = torch.rand(M, 3, device=dev)
    p = 0.01 * torch.randn(M, 3, device=dev)
    a = torch.randn(M, 3, device=dev)
    gd = torch.ones(1, device=dev)
    for alg in (0, 1):
        _lib.set_option("fwd_alg", alg)
        _lib.ode_self_fwd(q, p, 0.1, 0.0, True)
    _lib.set_option("fwd_alg", 1)
    _lib.ode_self_bwd(q, p, a, a, gd, 0.1, 0.0)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
