"""Launch each hot kernel a few times at the bench's sizes (100k support points, 100k x 100k
E-step), in the variants the bench's timed steps run, for rocprofv3 PMC passes, e.g.

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc -o fetch --output-format csv -- python tools/pmc_probe.py
    rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc -o write --output-format csv -- python tools/pmc_probe.py
    python tools/pmc_traffic.py gpurun_out/pmc > profiles/pmc_traffic.json
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from difficp_amd import _lib  # noqa: E402


def main():
    M = int(os.environ.get("PMC_M", "100000"))
    if os.environ.get("PMC_SYM_L"):   # A/B of the VJP's column groups per workgroup
        _lib.set_option("sym_L", int(os.environ["PMC_SYM_L"]))
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    q = torch.rand(M, 3, device=dev)
    p = 0.01 * torch.randn(M, 3, device=dev)
    a = torch.randn(M, 3, device=dev)
    gd = torch.ones(1, device=dev)
    mu2 = (q * q).sum(-1)
    w2 = torch.zeros(M, device=dev)
    zs = torch.empty_like(q)
    if os.environ.get("PMC_OPS") == "symfwd":  # ordered vs symmetric packed forward (fwd_alg 2 / 4)
        for alg in (2, 4, 2, 4):
            _lib.set_option("fwd_alg", alg)
            _lib.ode_self_fwd(q, p, 0.1, 0.0, True)
        _lib.set_option("fwd_alg", 2)
        torch.cuda.synchronize()
        return
    if os.environ.get("PMC_OPS") == "ksum":   # the kernel sum x = y (pair-once) and x != y (ordered)
        y = torch.rand(M, 3, device=dev)
        for _ in range(5):
            _lib.gauss_red(_lib.KRED, q, q, 0.1, b=p)
            _lib.gauss_red(_lib.KRED, q, y, 0.1, b=p)
        torch.cuda.synchronize()
        return
    if os.environ.get("PMC_OPS") == "kred":   # the north_star's kernel sum alone (centred path)
        for _ in range(5):
            _lib.gauss_red(_lib.KRED, q, q, 0.1, b=p)
        torch.cuda.synchronize()
        return
    if os.environ.get("PMC_OPS") == "estep":  # the E-step as the EM loop runs it: unhinted, then hinted
        T2 = _lib.gmm_estep(q, q, w2, mu2, 0.05, 0.0, True)[1]
        for _ in range(3):
            _lib.gmm_estep(q, q, w2, mu2, 0.05, 0.0, True, hint=T2)
        torch.cuda.synchronize()
        return
    # the variants the bench's timed Euler steps run (shooting.ShootFn, t = 1..nt-2): the fused
    # forward step writing the divergence rows zs, and the full adjoint step reusing them
    T2 = _lib.gmm_estep(q, q, w2, mu2, 0.05, 0.0, True)[1]
    for _ in range(3):
        _lib.euler_step(q, p, 0.1, 0.0, 0.1, True, zs_out=zs)
        _lib.euler_adjoint_step(q, p, a, a, gd, 0.1, 0.0, 0.1, zs=zs)
        _lib.gmm_estep(q, q, w2, mu2, 0.05, 0.0, True, hint=T2)   # the EM loop's later E-steps
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
