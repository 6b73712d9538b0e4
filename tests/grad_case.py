"""Shared body of the reduction-gradient tests (CPU spec: tests/test_host_logic.py; GPU:
tests/test_gpu_model.py): autograd through GaussKernel's GenDKRed, HessKRed, GradLapKRed,
DDKRed and GradKRed_rev (kernel.py:147-168, :194-207, :284-292) against float64 torch
autograd through the oracle, w.r.t. every input."""
import torch

from conftest import rel_err
from oracle import torch_ref as R


def check_reduction_grads(dev, D, M=150, N=230, sig=0.3, tol_f=1e-5, tol_g=2e-5):
    from difficp_amd.tools.kernel import GaussKernel
    g = torch.Generator().manual_seed(40 + D)
    mk = lambda *s, scale=1.0: (scale * torch.randn(*s, generator=g, dtype=torch.float64))
    x = torch.rand(M, D, generator=g, dtype=torch.float64)
    y = torch.rand(N, D, generator=g, dtype=torch.float64)
    b = mk(N, D)
    c = mk(M, D)
    dm = mk(M, D)
    GK = GaussKernel(sig, D, spec={"device": dev, "dtype": torch.float32})
    cases = [
        ("GenDKRed", (x, y, b, c), lambda X, Y, B, C: GK.GenDKRed(X, Y, B, C),
         lambda X, Y, B, C: R.GenDKRed(X, Y, B, C, sig)),
        ("HessKRed", (x, y, b, c), lambda X, Y, B, C: GK.HessKRed(X, Y, B, C),
         lambda X, Y, B, C: R.HessKRed(X, Y, B, C, sig)),
        ("GradLapKRed", (x, y), lambda X, Y: GK.GradLapKRed(X, Y),
         lambda X, Y: R.GradLapKRed(X, Y, sig)),
        ("DDKRed", (x, y, b), lambda X, Y, B: GK.DDKRed(X, Y, B),
         lambda X, Y, B: R.DDKRed(X, Y, B, sig)),
        ("GradKRed_rev", (x, y, dm), lambda X, Y, Dm: GK.GradKRed_rev(X, Y, Dm),
         lambda X, Y, Dm: R.GradKRed_rev(X, Y, Dm, sig)),
    ]
    for name, ins, fh, fr in cases:
        i64 = [t.clone().requires_grad_(True) for t in ins]
        o64 = fr(*i64)
        wt = torch.randn(o64.shape, generator=g, dtype=torch.float64)
        g64 = torch.autograd.grad((o64 * wt).sum(), i64)
        ih = [t.float().to(dev).requires_grad_(True) for t in ins]
        oh = fh(*ih)
        assert oh.shape == o64.shape, name
        assert rel_err(oh.detach().cpu(), o64.detach()) < tol_f, name
        gh = torch.autograd.grad((oh * wt.float().to(dev)).sum(), ih)
        for k, (a, r) in enumerate(zip(gh, g64)):
            e = rel_err(a.cpu(), r)
            assert e < tol_g, (name, k, e)
