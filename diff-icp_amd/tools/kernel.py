"""Gaussian kernel and its N x M reductions, bound to the gfx950 HIP kernels.

Mirror of diffICP/tools/kernel.py (GenKernel :58, GaussKernel :254).  The reference binds
ten reduction aliases in `set_computversion` (kernel.py:91-110) to KeOps or torch
implementations; here they are bound to `computversion="hip"`: hand-written gfx950 kernels
reached through the C-ABI library (include/difficp_hip.h, dicp_gauss_red_f32).  "keops"
is accepted as an alias of "hip" (this is the backend that replaces KeOps); "torch" is
mapped to "hip" with a warning -- the product path has no CPU implementation.

Every reduction is differentiable w.r.t. every input, as the reference's are through KeOps /
torch autodiff: each input gradient is one more tiled HIP reduction (KRed / GradKRed /
HessKRed forms of the existing pair ops, or the five gradient pair ops of
dicp_gauss_red_grad_f32 for the second and third kernel derivatives).  The LDDMM ODE itself
is differentiated through the fused kernels of core/shooting.py.
"""
from __future__ import annotations

import math
import warnings

import numpy as np
import torch

from .. import _lib
from .spec import defspec, getspec


def SVDpow(M, alpha, rcond=None):
    """SVD-based (pseudo-)power of a hermitian matrix (kernel.py:31-44)."""
    U, S, Vh = torch.linalg.svd(M)
    keep = S > rcond * S[0] if rcond is not None else slice(None)
    return U[:, keep] @ torch.diag(S[keep] ** alpha) @ Vh[keep, :]


# ---------------------------------------------------------------------------------------
# autograd wrappers of the reductions
# ---------------------------------------------------------------------------------------
class _KBase(torch.autograd.Function):
    """X_i = sum_j K(x_i-y_j).  dX/dx_i = g_i sum_j gradK ; dX/dy_j = sum_i g_i gradK(y_j-x_i)."""

    @staticmethod
    def forward(ctx, x, y, sigma):
        ctx.sigma = sigma
        ctx.save_for_backward(x, y)
        return _lib.gauss_red(_lib.KBASE, x, y, sigma)

    @staticmethod
    def backward(ctx, g):
        x, y = ctx.saved_tensors
        s = ctx.sigma
        g = g.contiguous()
        gx = gy = None
        if ctx.needs_input_grad[0]:
            gx = g[:, None] * _lib.gauss_red(_lib.GRADK, x, y, s)
        if ctx.needs_input_grad[1]:
            gy = _lib.gauss_red(_lib.GRADKSCAL, y, x, s, b=g)
        return gx, gy, None


class _KRedScal(torch.autograd.Function):
    """X_i = sum_j K d_j."""

    @staticmethod
    def forward(ctx, x, y, d, sigma):
        ctx.sigma = sigma
        ctx.save_for_backward(x, y, d)
        return _lib.gauss_red(_lib.KREDSCAL, x, y, sigma, b=d)

    @staticmethod
    def backward(ctx, g):
        x, y, d = ctx.saved_tensors
        s = ctx.sigma
        g = g.contiguous()
        gx = gy = gd = None
        if ctx.needs_input_grad[0]:
            gx = g[:, None] * _lib.gauss_red(_lib.GRADKSCAL, x, y, s, b=d)
        if ctx.needs_input_grad[1]:
            gy = d[:, None] * _lib.gauss_red(_lib.GRADKSCAL, y, x, s, b=g)
        if ctx.needs_input_grad[2]:
            gd = _lib.gauss_red(_lib.KREDSCAL, y, x, s, b=g)
        return gx, gy, gd, None


class _KRed(torch.autograd.Function):
    """X_i = sum_j K b_j.  dx_i = GenDKRed(x,y,b,g) ; dy_j = GenDKRed(y,x,g,b) ; db = KRed(y,x,g)."""

    @staticmethod
    def forward(ctx, x, y, b, sigma):
        ctx.sigma = sigma
        ctx.save_for_backward(x, y, b)
        return _lib.gauss_red(_lib.KRED, x, y, sigma, b=b)

    @staticmethod
    def backward(ctx, g):
        x, y, b = ctx.saved_tensors
        s = ctx.sigma
        g = g.contiguous()
        gx = gy = gb = None
        if ctx.needs_input_grad[0]:
            gx = _lib.gauss_red(_lib.GENDK, x, y, s, b=b, c=g)
        if ctx.needs_input_grad[1]:
            gy = _lib.gauss_red(_lib.GENDK, y, x, s, b=g, c=b)
        if ctx.needs_input_grad[2]:
            gb = _lib.gauss_red(_lib.KRED, y, x, s, b=g)
        return gx, gy, gb, None


class _GradKRed(torch.autograd.Function):
    """X_i = sum_j gradK(x_i - y_j).  dx_i = sum_j HessK g_i ; dy_j = -sum_i HessK(y_j-x_i) g_i."""

    @staticmethod
    def forward(ctx, x, y, sigma):
        ctx.sigma = sigma
        ctx.save_for_backward(x, y)
        return _lib.gauss_red(_lib.GRADK, x, y, sigma)

    @staticmethod
    def backward(ctx, g):
        x, y = ctx.saved_tensors
        s = ctx.sigma
        g = g.contiguous()
        gx = gy = None
        if ctx.needs_input_grad[0]:
            gx = _lib.gauss_red(_lib.HESSK, x, y, s, b=torch.zeros_like(y), c=g)
        if ctx.needs_input_grad[1]:
            gy = _lib.gauss_red(_lib.HESSK, y, x, s, b=g, c=torch.zeros_like(y))
        return gx, gy, None


class _LapKRed(torch.autograd.Function):
    """X_i = sum_j LapK(x_i - y_j).  dx_i = g_i GradLapKRed_i ; dy_j = sum_i g_i gradLapK(y_j-x_i)."""

    @staticmethod
    def forward(ctx, x, y, sigma):
        ctx.sigma = sigma
        ctx.save_for_backward(x, y)
        return _lib.gauss_red(_lib.LAPK, x, y, sigma)

    @staticmethod
    def backward(ctx, g):
        x, y = ctx.saved_tensors
        s = ctx.sigma
        g = g.contiguous()
        gx = gy = None
        if ctx.needs_input_grad[0]:
            gx = g[:, None] * _lib.gauss_red(_lib.GRADLAPK, x, y, s)
        if ctx.needs_input_grad[1]:
            gy = _lib.gauss_red(_lib.GRADLAPKSCAL, y, x, s, b=g)
        return gx, gy, None


# The five reductions below are differentiated by one more tiled row reduction per input
# gradient (dicp_gauss_red_grad_f32, csrc/grad_ops.hpp; the pair formulas are derived in
# DESIGN.md section 3): the reference gets these gradients from KeOps / torch autodiff
# (kernel.py:147-168, :194-207, :284-292).  z = x_i - y_j; g = the output cotangent.
def _neg(t):
    return None if t is None else -t


class _GradKRedRev(torch.autograd.Function):
    """Y_j = sum_i gradK(x_i - y_j).d_i  (N,).
    dx_i = sum_j g_j [s^2 (z.d_i) z - s d_i] K ; dy_j = -g_j sum_i [s^2 (z.d_i) z - s d_i] K ;
    dd_i = sum_j g_j gradK(z)."""

    @staticmethod
    def forward(ctx, x, y, d, sigma):
        ctx.sigma = sigma
        ctx.save_for_backward(x, y, d)
        return _lib.gauss_red(_lib.GRADK_REV, y, x, sigma, b=d)

    @staticmethod
    def backward(ctx, g):
        x, y, d = ctx.saved_tensors
        s = ctx.sigma
        g = g.contiguous()
        gx = gy = gd = None
        if ctx.needs_input_grad[0]:
            gx = _lib.gauss_red_grad(_lib.GRAD_HESSW, x, y, s, r1=d, cw=g)
        if ctx.needs_input_grad[1]:
            gy = g[:, None] * _lib.gauss_red_grad(_lib.GRAD_HESSW, y, x, s, c1=d)
        if ctx.needs_input_grad[2]:
            gd = _lib.gauss_red(_lib.GRADKSCAL, x, y, s, b=g)
        return gx, gy, gd, None


class _DDKRed(torch.autograd.Function):
    """X_i^d = sum_j -s z^d K b_j^d.  With w = g_i * b_j (elementwise):
    dx_i = sum_j [s^2 (z.w) z - s w] K ; dy_j = -sum_i [...] ; db_j^d = sum_i s z^d K g_i^d."""

    @staticmethod
    def forward(ctx, x, y, b, sigma):
        ctx.sigma = sigma
        ctx.save_for_backward(x, y, b)
        return _lib.gauss_red(_lib.DDK, x, y, sigma, b=b)

    @staticmethod
    def backward(ctx, g):
        x, y, b = ctx.saved_tensors
        s = ctx.sigma
        g = g.contiguous()
        gx = gy = gb = None
        if ctx.needs_input_grad[0]:
            gx = _lib.gauss_red_grad(_lib.GRAD_HESSWP, x, y, s, r1=g, c1=b)
        if ctx.needs_input_grad[1]:
            gy = -_lib.gauss_red_grad(_lib.GRAD_HESSWP, y, x, s, r1=b, c1=g)
        if ctx.needs_input_grad[2]:
            gb = -_lib.gauss_red(_lib.DDK, y, x, s, b=g)
        return gx, gy, gb, None


class _GenDKRed(torch.autograd.Function):
    """X_i = sum_j gradK(z) (c_i.b_j).
    dx_i = sum_j (c_i.b_j) [s^2 (z.g_i) z - s g_i] K ; dy_j = -sum_i (same) ;
    dc_i = sum_j -s (z.g_i) K b_j ; db_j = sum_i -s (z.g_i) K c_i."""

    @staticmethod
    def forward(ctx, x, y, b, c, sigma):
        ctx.sigma = sigma
        ctx.save_for_backward(x, y, b, c)
        return _lib.gauss_red(_lib.GENDK, x, y, sigma, b=b, c=c)

    @staticmethod
    def backward(ctx, g):
        x, y, b, c = ctx.saved_tensors
        s = ctx.sigma
        g = g.contiguous()
        gx = gy = gb = gc = None
        if ctx.needs_input_grad[0]:
            gx = _lib.gauss_red_grad(_lib.GRAD_HESSW, x, y, s, r1=g, r2=c, c2=b)
        if ctx.needs_input_grad[1]:
            gy = _lib.gauss_red_grad(_lib.GRAD_HESSW, y, x, s, c1=g, r2=b, c2=c)
        if ctx.needs_input_grad[2]:
            gb = _lib.gauss_red_grad(_lib.GRAD_ZDOTV, y, x, s, c1=_neg(g), c2=c)
        if ctx.needs_input_grad[3]:
            gc = _lib.gauss_red_grad(_lib.GRAD_ZDOTV, x, y, s, r1=g, c2=b)
        return gx, gy, gb, gc, None


class _HessKRed(torch.autograd.Function):
    """X_i = sum_j [s^2 (z.u) z - s u] K, u = c_i - b_j.
    dx_i = sum_j grad_z{ g_i . [...] K } (third kernel derivative, HESS3) ; dy_j = -sum_i (same);
    dc_i = sum_j [s^2 (z.g_i) z - s g_i] K ; db_j = -sum_i [...]."""

    @staticmethod
    def forward(ctx, x, y, b, c, sigma):
        ctx.sigma = sigma
        ctx.save_for_backward(x, y, b, c)
        return _lib.gauss_red(_lib.HESSK, x, y, sigma, b=b, c=c)

    @staticmethod
    def backward(ctx, g):
        x, y, b, c = ctx.saved_tensors
        s = ctx.sigma
        g = g.contiguous()
        gx = gy = gb = gc = None
        if ctx.needs_input_grad[0]:
            gx = _lib.gauss_red_grad(_lib.GRAD_HESS3, x, y, s, r1=c, c1=b, r2=g)
        if ctx.needs_input_grad[1]:
            gy = _lib.gauss_red_grad(_lib.GRAD_HESS3, y, x, s, r1=_neg(b), c1=_neg(c), c2=g)
        if ctx.needs_input_grad[2]:
            gb = _lib.gauss_red_grad(_lib.GRAD_HESSW, y, x, s, c1=g)
        if ctx.needs_input_grad[3]:
            gc = _lib.gauss_red_grad(_lib.GRAD_HESSW, x, y, s, r1=g)
        return gx, gy, gb, gc, None


class _GradLapKRed(torch.autograd.Function):
    """X_i = sum_j -z (s^3 r2 - (D+2) s^2) K.
    dx_i = -sum_j K [phi g_i + s^3 (D + 4 - s r2)(g_i.z) z] ; dy_j = -sum_i (same)."""

    @staticmethod
    def forward(ctx, x, y, sigma):
        ctx.sigma = sigma
        ctx.save_for_backward(x, y)
        return _lib.gauss_red(_lib.GRADLAPK, x, y, sigma)

    @staticmethod
    def backward(ctx, g):
        x, y = ctx.saved_tensors
        s = ctx.sigma
        g = g.contiguous()
        gx = gy = None
        if ctx.needs_input_grad[0]:
            gx = _lib.gauss_red_grad(_lib.GRAD_GRADLAP3, x, y, s, r1=g)
        if ctx.needs_input_grad[1]:
            gy = _lib.gauss_red_grad(_lib.GRAD_GRADLAP3, y, x, s, c1=-g)
        return gx, gy, None


# ---------------------------------------------------------------------------------------
class GenKernel:
    """Generic kernel with the ten reduction aliases (kernel.py:58-242)."""

    _ALIASES = ("KBase", "KRed", "KRedScal", "GradKRed", "DDKRed", "GenDKRed", "HessKRed",
                "LapKRed", "GradLapKRed", "GradKRed_rev")

    def K_torch(self, x, y):
        raise NotImplementedError()

    def set_computversion(self, version):
        """Bind the reduction aliases (kernel.py:91-110).  Backends: "hip" (and its alias
        "keops").  "torch" is redirected to "hip" with a warning."""
        if version == "torch":
            warnings.warn("computversion='torch' is served by the HIP backend in difficp_amd "
                          "(no CPU path).")
            version = "hip"
        if version == "keops":
            version = "hip"
        if version != "hip":
            raise ValueError(f"unkown computversion : {version}. Choices are 'hip' (or 'keops')")
        for name in self._ALIASES:
            setattr(self, name, getattr(self, name + "_hip"))
        self.computversion = version

    def __init__(self, D, computversion="hip"):
        self.computversion = None
        for name in self._ALIASES:
            setattr(self, name, None)
        self.set_computversion(computversion)

    # Dense-matrix solves (kernel.py:227-242).  These are set-up helpers, not the hot path.
    def KpinvSolve(self, x, v, rcond=None):
        """Min-norm least-squares solution of K(x,x) b = v (np.linalg.lstsq semantics,
        kernel.py:227-232), computed on the device by SVD.  v == 0 short-circuits to 0
        (the exact min-norm solution), which keeps zero-speed initialisation O(M)."""
        spec = getspec(x, v)
        if not bool(torch.any(v != 0)):
            return torch.zeros_like(v)
        K = self.K_torch(x, x).double()
        U, S, Vh = torch.linalg.svd(K)
        cut = (rcond if rcond is not None else np.finfo(np.float64).eps * max(K.shape)) * S[0]
        Sinv = torch.where(S > cut, 1.0 / S, torch.zeros_like(S))
        b = Vh.t() @ (Sinv[:, None] * (U.t() @ v.double()))
        return b.to(**spec).contiguous()

    def KridgeSolve_torch(self, x, v, alpha=1e-4):
        """Dense ridge solve (K + alpha I) b = v (kernel.py:234-237), on the device."""
        K = self.K_torch(x, x)
        return torch.linalg.solve(K + alpha * torch.eye(K.shape[0], dtype=K.dtype, device=K.device), v)

    KridgeSolve_pytorch = KridgeSolve_torch   # LDDMM.py:251 calls this (missing in the reference)

    # KeOps-style iterative ridge solve (kernel.py:239-241: LazyTensor.solve = conjugate
    # gradients with the kernel mat-vec): HIP CG with the KRed reduction, O(M) memory, so it
    # scales to the 50k-200k support sets where the dense solves cannot run.
    cg_eps = 1e-6
    cg_maxiter = 5000

    def KridgeSolve_keops(self, x, v, alpha=1e-4):
        getspec(x, v)
        b, info = _lib.kernel_ridge_cg(x.detach(), v.detach(), self.sigma, alpha,
                                       eps=self.cg_eps, maxiter=self.cg_maxiter)
        self.last_solve_info = info
        if info["status"] != "converged":
            warnings.warn(f"KridgeSolve_keops: CG stopped ({info})")
        return b

    KridgeSolve = KridgeSolve_keops


class GaussKernel(GenKernel):
    """K(z) = exp(-|z|^2 / 2 sigma^2) (kernel.py:248-337)."""

    def __init__(self, sigma, D, computversion="hip", spec=defspec):
        self.sigma = sigma
        self.D = D
        self.spec = spec
        super().__init__(D, computversion)

    # dense helpers (kernel.py:259-267) -- used by set-up code only (pinv solve, random_p)
    def K_torch(self, x, y):
        return (-((x[:, None, :] - y[None, :, :]) ** 2) / (2 * self.sigma ** 2)).sum(-1).exp()

    def GradK_torch(self, x, y):
        return self.K_torch(x, y)[:, :, None] * (y[None, :, :] - x[:, None, :]) / self.sigma ** 2

    def LapK_torch(self, x, y):
        D2 = torch.sum((x[:, None, :] - y[None, :, :]) ** 2, -1)
        return torch.exp(-D2 / (2 * self.sigma ** 2)) * (D2 / self.sigma ** 4 - self.D / self.sigma ** 2)

    # ---- the ten reductions (USAGE comments of kernel.py:130-168) ----
    def KBase_hip(self, x, y):
        getspec(x, y)
        return _KBase.apply(x, y, self.sigma)

    def KRedScal_hip(self, x, y, d):
        getspec(x, y, d)
        return _KRedScal.apply(x, y, d, self.sigma)

    def KRed_hip(self, x, y, b):
        getspec(x, y, b)
        return _KRed.apply(x, y, b, self.sigma)

    def GradKRed_hip(self, x, y):
        getspec(x, y)
        return _GradKRed.apply(x, y, self.sigma)

    def GradKRed_rev_hip(self, x, y, d):
        """Y_j = sum_i sum_d (d_d K)(x_i - y_j) d_i^d, shape (N,) -- column reduction done as
        a row reduction over y (kernel.py:147, :194-195)."""
        getspec(x, y, d)
        return _GradKRedRev.apply(x, y, d, self.sigma)

    def DDKRed_hip(self, x, y, b):
        getspec(x, y, b)
        return _DDKRed.apply(x, y, b, self.sigma)

    def GenDKRed_hip(self, x, y, b, c):
        getspec(x, y, b, c)
        return _GenDKRed.apply(x, y, b, c, self.sigma)

    def HessKRed_hip(self, x, y, b, c):
        getspec(x, y, b, c)
        return _HessKRed.apply(x, y, b, c, self.sigma)

    def LapKRed_hip(self, x, y):
        getspec(x, y)
        return _LapKRed.apply(x, y, self.sigma)

    def GradLapKRed_hip(self, x, y):
        getspec(x, y)
        return _GradLapKRed.apply(x, y, self.sigma)

    def check_coverage(self, X, Y, Rthreshold):
        """Boolean (N,) mask of points X at distance > Rthreshold*sigma from every Y
        (kernel.py:324-329; the reference's torch branch is broken, this is the intended
        result, computed by a min-reduction kernel)."""
        getspec(X, Y)
        if Y.shape[0] == 0:
            return torch.ones(X.shape[0], dtype=torch.bool, device=X.device)
        d2 = _lib.gauss_red(_lib.MIN_SQDIST, X.detach(), Y.detach(), self.sigma)
        return d2 > (Rthreshold * self.sigma) ** 2

    def __setstate__(self, state):
        self.__dict__.update(state)
        self.spec = defspec
