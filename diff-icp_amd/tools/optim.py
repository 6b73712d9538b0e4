"""L-BFGS wrapper with divergence fallback (semantics of diffICP/tools/optim.py:10-110).

The optimizer is torch.optim.LBFGS's algorithm (same control flow, memory rule, strong-Wolfe
line search) with the inverse-Hessian product in compact form (tools/lbfgs.py CompactLBFGS:
~10 device kernels per iteration instead of ~5 per stored pair); the closure's cost is the
HIP shooting + its fused backward.
"""
import math

import torch

from . import runstats
from .lbfgs import CompactLBFGS


FALLBACK_SEED = 0x5EED


def LBFGS_optimization(p0, lossfunc, nmax=10, tol=1e-3, errthresh=1e8, generator=None, lossgrad=None):
    """Returns (best_p list, best_L, nsteps, change) exactly as optim.py:10-110:
    L-BFGS(max_iter=20, max_eval=100, history_size=100, strong_wolfe) steps; on NaN /
    increase / > errthresh fall back to the best parameters seen (or a 1% random
    perturbation) and restart without line search; stop when the RMS parameter change is
    below tol x RMS parameter value.

    The perturbation (optim.py:85 draws it from torch's global RNG) is drawn from `generator`,
    by default a dedicated one seeded with FALLBACK_SEED at the first fallback of this call:
    the result then does not depend on the global RNG state, ranks of a row split (which must
    stay in lockstep) draw the same numbers, and concurrent frames (one host thread each)
    do not race on a shared generator.

    lossgrad (extension): optional callable p -> (loss, [dL/dp]) computing the same loss and
    gradient as lossfunc(*p).backward() without autograd's engine (core/shooting.py
    shoot_loss_grad, used by the lockstep frame batches); the closure then sets p.grad itself."""
    p = [a.clone().contiguous().detach().requires_grad_(True) for a in p0]
    optimizer = CompactLBFGS(p, max_iter=20, max_eval=100, history_size=100,
                             line_search_fn="strong_wolfe")
    iter_L, best_L, best_p = [], math.inf, None
    optimizer.on_loss = lambda Ld: record(Ld)

    def closure():
        runstats.add("closures")
        optimizer.zero_grad()
        if lossgrad is not None:
            L, grads = lossgrad(*p)
            for a, g in zip(p, grads):
                a.grad = g
            return L
        L = lossfunc(*p)
        # backward is queued BEFORE the host reads the loss (optim.py:41-47 reads it first): the
        # gradient does not depend on the read and p is not modified by backward, so results are
        # unchanged, but the host no longer drains the stream between the forward shooting and
        # its adjoint.  The loss itself is read by the optimizer together with the line
        # search's scalars (one transfer) and handed to record() below.
        L.backward()
        return L

    def record(Ld):
        # optim.py:39-45 (iter_L, best_p), while p still holds the evaluated point
        nonlocal best_L, best_p
        iter_L.append(Ld)
        if Ld < best_L:
            best_L = Ld
            best_p = [a.clone().detach() for a in p]

    i, keepOn, L = 0, True, math.inf
    change = None
    while i < nmax and keepOn:
        i += 1
        p_prev = [a.clone().detach() for a in p]
        optimizer.step(closure)
        Lprev, L = L, iter_L[-1]
        if L > Lprev or L > errthresh or math.isnan(L):
            if math.isnan(L):
                print("WARNING: NaN value for loss L during L-BFGS optimization.")
            elif L > errthresh:
                print("WARNING: Aberrantly large value for loss L during L-BFGS optimization.")
            elif L > Lprev:
                print("WARNING: Increase of loss L during L-BGFS optimization.")
            if best_L < Lprev:
                p = [a.clone() for a in best_p]
                L = best_L
                print("L-BFGS optimization. Found an intermediate 'best_p' value for this iteration.")
            else:
                rmod = 0.01
                if generator is None:
                    generator = torch.Generator(device=best_p[0].device)
                    generator.manual_seed(FALLBACK_SEED)
                p = [a + rmod * a.std() * torch.randn(a.shape, dtype=a.dtype, device=a.device,
                                                      generator=generator)
                     for a in best_p]
                L = lossfunc(*p)
                print("L-BFGS optimization. Trying a random perturbation of parameter from its "
                      f"current value, with relative strength {rmod}.")
            change = "None (divergent iteration step)"
            p = [a.detach().requires_grad_(True) for a in p]
            optimizer = CompactLBFGS(p, max_iter=20, max_eval=100, history_size=100,
                                     line_search_fn=None)
            optimizer.on_loss = lambda Ld: record(Ld)
        else:
            changes = [((a - a_prev) ** 2).mean().sqrt().detach().cpu().numpy()
                       for a, a_prev in zip(p, p_prev)]
            refs = [(a_prev ** 2).mean().sqrt().detach().cpu().numpy() for a_prev in p_prev]
            keepOn = any(c > tol * r for c, r in zip(changes, refs))
            change = max(changes)
    best_p = [a.detach() for a in best_p]
    return best_p, best_L, i, change
