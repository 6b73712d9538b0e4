"""ORACLE -- test infrastructure only, never shipped, never the measured product.

CPU restatement (torch, any dtype; float64 by default) of the reference's runnable path
(AdrienWohrer/diff-icp, computversion="torch").  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this module.  Each function cites the reference
file:line it restates.  Pinned against the golden vectors in tests/golden/ that were
produced by importing the reference itself (tests/golden/make_golden.py, this container
only); see tests/test_oracle_golden.py.

Large inputs are processed in row chunks so memory stays O(chunk x N).
"""
from __future__ import annotations

import math

import numpy as np
import torch

CHUNK = 2048


def _rows(fn, x, *row_args, chunk=CHUNK):
    """Apply fn(x_chunk, *row_arg_chunks) over row chunks of x and concatenate."""
    M = x.shape[0]
    if M <= chunk:
        return fn(x, *row_args)
    outs = []
    for a in range(0, M, chunk):
        b = min(M, a + chunk)
        outs.append(fn(x[a:b], *[None if r is None else r[a:b] for r in row_args]))
    return torch.cat(outs, 0)


# ---------------------------------------------------------------------------------------
# Gaussian kernel and reductions  (diffICP/tools/kernel.py:177-292)
# ---------------------------------------------------------------------------------------
def K(x, y, sigma):                                   # kernel.py:259-260
    return (-(x[:, None, :] - y[None, :, :]) ** 2 / (2 * sigma ** 2)).sum(-1).exp()


def GradK(x, y, sigma):                               # kernel.py:262-263
    return K(x, y, sigma)[:, :, None] * (y[None, :, :] - x[:, None, :]) / sigma ** 2


def LapK(x, y, sigma):                                # kernel.py:265-267
    D = x.shape[1]
    D2 = torch.sum((x[:, None, :] - y[None, :, :]) ** 2, -1)
    return torch.exp(-D2 / (2 * sigma ** 2)) * (D2 / sigma ** 4 - D / sigma ** 2)


def KBase(x, y, sigma):                               # kernel.py:178-179
    return _rows(lambda xc: torch.sum(K(xc, y, sigma), 1), x)


def KRedScal(x, y, d, sigma):                         # kernel.py:182-183
    return _rows(lambda xc: torch.sum(K(xc, y, sigma) * d[None, :], 1), x)


def KRed(x, y, b, sigma):                             # kernel.py:186-187
    return _rows(lambda xc: torch.sum(K(xc, y, sigma)[:, :, None] * b[None, :, :], 1), x)


def GradKRed(x, y, sigma):                            # kernel.py:190-191
    return _rows(lambda xc: torch.sum(GradK(xc, y, sigma), 1), x)


def GradKRed_rev(x, y, d, sigma):                     # kernel.py:194-195 (column reduction)
    out = 0
    for a in range(0, x.shape[0], CHUNK):
        out = out + torch.sum((GradK(x[a:a + CHUNK], y, sigma) * d[a:a + CHUNK, None, :]).sum(-1), 0)
    return out


def DDKRed(x, y, b, sigma):                           # kernel.py:198-199
    return _rows(lambda xc: torch.sum(GradK(xc, y, sigma) * b[None, :, :], 1), x)


def GenDKRed(x, y, b, c, sigma):                      # kernel.py:202-203
    return _rows(lambda xc, cc: torch.sum(GradK(xc, y, sigma) *
                                          (b[None, :, :] * cc[:, None, :]).sum(-1)[:, :, None], 1), x, c)


def LapKRed(x, y, sigma):                             # kernel.py:206-207
    return _rows(lambda xc: torch.sum(LapK(xc, y, sigma), 1), x)


def HessKRed(x, y, b, c, sigma):                      # kernel.py:284-286
    def f(xc, cc):
        z = xc[:, None, :] - y[None, :, :]
        u = cc[:, None, :] - b[None, :, :]
        yo = (z * u).sum(-1)[:, :, None] * z
        return torch.sum((yo / sigma ** 4 - u / sigma ** 2) * K(xc, y, sigma)[:, :, None], 1)
    return _rows(f, x, c)


def GradLapKRed(x, y, sigma):                         # kernel.py:289-292
    D = x.shape[1]

    def f(xc):
        D2 = torch.sum((xc[:, None, :] - y[None, :, :]) ** 2, -1)[:, :, None]
        return torch.sum(torch.exp(-D2 / (2 * sigma ** 2)) * (y[None, :, :] - xc[:, None, :])
                         * (D2 / sigma ** 6 - (D + 2) / sigma ** 4), 1)
    return _rows(f, x)


def MinSqDist(x, y):                                  # kernel.py:324-329 (intended result)
    return _rows(lambda xc: ((xc[:, None, :] - y[None, :, :]) ** 2).sum(-1).min(dim=1).values, x)


def SqDistF32(x, y):                                  # point_sets.py:114-116 (float32 arithmetic)
    x, y = x.float(), y.float()
    return ((x[:, None, :] - y[None, :, :]) ** 2).sum(-1)


def MinSqDistOther(x):                                # point_sets.py:22-23, Kmin(2)[:, 1]
    d = SqDistF32(x, x)
    return d.sort(dim=1).values[:, 1] if x.shape[0] > 1 else torch.full((x.shape[0],), float("inf"))


def intrinsic_scale(x):                               # point_sets.py:13-26
    return MinSqDistOther(x).mean().sqrt().item()


def decimate(x, R):                                   # point_sets.py:102-133, restated as written
    """Greedy covering decimation: O(N^2) per kept point, small N only."""
    import numpy as np
    M = (SqDistF32(x, x) <= R ** 2).numpy()
    N = x.shape[0]
    notcovered = np.arange(N)
    kept = []
    while len(notcovered) > 0:
        i = notcovered[M[np.ix_(notcovered, notcovered)].sum(axis=0).argmax()]
        kept.append(int(i))
        notcovered = notcovered[~M[i, notcovered]]
    kept_set = set(kept)
    return kept, [i for i in range(N) if i not in kept_set]


# ---------------------------------------------------------------------------------------
# LDDMM (diffICP/core/LDDMM.py:100-227, 286-334)
# ---------------------------------------------------------------------------------------
def data_distance(x, y, sigma, w=None):              # PSR_standard.py:37-58
    Nx, Ny = x.shape[0], y.shape[0]
    if w is None:
        return (KBase(x, x, sigma).sum() / Nx ** 2 + KBase(y, y, sigma).sum() / Ny ** 2
                - 2 * KBase(y, x, sigma).sum() / (Nx * Ny))
    return (KBase(x, x, sigma).sum() / Nx ** 2 + (KRedScal(y, y, w, sigma) * w).sum()
            - 2 * (KBase(y, x, sigma) * w).sum() / Nx)


def KridgeSolve_torch(x, v, sigma, alpha):            # kernel.py:234-237 (dense ridge)
    Kxx = K(x, x, sigma)
    return torch.linalg.solve(Kxx + alpha * torch.eye(Kxx.shape[0], dtype=Kxx.dtype), v)


def KridgeSolve_cg(x, v, sigma, alpha, eps=1e-6, maxiter=100000):
    """kernel.py:239-241 KridgeSolve_keops = K_keops(Vi(x),Vj(x)).solve(Vi(v), alpha).  The
    algorithm lives in the third-party pykeops (absent here, no pinned version, setup.py:3-10):
    its published ConjugateGradientSolver runs ONE CG on the flattened (M,D) system with
    linop(p) = K p + alpha p and stops when |r|^2 < size(v) * eps^2.  Restated as written;
    returns (b, iterations)."""
    delta = v.numel() * eps ** 2
    r = v.clone()
    nr2 = (r ** 2).sum()
    if nr2 < delta:
        return 0 * r, 0
    a = torch.zeros_like(v)
    p = r.clone()
    k = 0
    while k < maxiter:
        Mp = KRed(x, x, p, sigma) + alpha * p
        alp = nr2 / (p * Mp).sum()
        a += alp * p
        r -= alp * Mp
        nr2new = (r ** 2).sum()
        k += 1
        if nr2new < delta:
            break
        p = r + (nr2new / nr2) * p
        nr2 = nr2new
    return a, k


class LDDMM:
    """Functional restatement of LDDMMModel's numerics (no optimizer state)."""

    def __init__(self, sigma, D, lam, gradcomponent, withlogdet, scheme="Euler", nt=10):
        self.sigma, self.D, self.lam, self.nt, self.scheme = sigma, D, lam, nt, scheme
        self.gradcomponent, self.withlogdet = gradcomponent, withlogdet
        self.eta = 1.0 / lam if gradcomponent else 0.0          # LDDMM.py:53-56

    def v(self, x, q, p):                                    # LDDMM.py:100-116
        if self.gradcomponent:
            return KRed(x, q, p, self.sigma) - self.eta * GradKRed(x, q, self.sigma)
        return KRed(x, q, p, self.sigma)

    def mdivsum(self, x, q, p):                              # LDDMM.py:120-138 (rev=False)
        r = (p * GradKRed(q, x, self.sigma)).sum()
        if self.gradcomponent:
            r = r + self.eta * LapKRed(q, x, self.sigma).sum()
        return r

    def Hamiltonian(self, q, p):                             # LDDMM.py:142-159
        H = 0.5 * (p * KRed(q, q, p, self.sigma)).sum()
        if self.gradcomponent:
            H = H - self.eta * (p * GradKRed(q, q, self.sigma)).sum() \
                - 0.5 * self.eta ** 2 * LapKRed(q, q, self.sigma).sum()
        return H

    def ODE(self, q, p, cost, x=None):                       # LDDMM.py:176-227
        vq = self.v(q, q, p)
        Gq = GenDKRed(q, q, p, p, self.sigma)
        if self.eta != 0:
            Gq = Gq - self.eta * HessKRed(q, q, p, p, self.sigma) \
                - self.eta ** 2 * GradLapKRed(q, q, self.sigma)
        zero = torch.zeros(1, dtype=q.dtype, device=q.device)
        if x is None:
            dcost = self.mdivsum(q, q, p).reshape(1) if self.withlogdet else zero
            return vq, -Gq, dcost
        dcost = self.mdivsum(x, q, p).reshape(1) if self.withlogdet else zero
        return vq, -Gq, dcost, self.v(x, q, p)

    def Shoot(self, q0, p0, x0=None):                         # LDDMM.py:286-299 + integrators.py
        cost0 = torch.zeros(1, dtype=q0.dtype, device=q0.device)
        st = (q0, p0, cost0) if x0 is None else (q0, p0, cost0, x0)
        x = tuple(t.clone() for t in st)
        dt = 1.0 / self.nt
        out = [x]
        for _ in range(self.nt):
            k1 = self.ODE(*x)
            if self.scheme == "Euler":                        # integrators.py:20-31
                x = tuple(a + dt * b for a, b in zip(x, k1))
            else:                                             # integrators.py:36-51
                xi = tuple(a + (2 * dt / 3) * b for a, b in zip(x, k1))
                k2 = self.ODE(*xi)
                x = tuple(a + (0.25 * dt) * (b + 3 * c) for a, b, c in zip(x, k1, k2))
            out.append(x)
        return out

    def trajloss(self, shoot):                               # LDDMM.py:318-334
        q0, p0 = shoot[0][:2]
        return self.lam * self.Hamiltonian(q0, p0) + shoot[-1][2]


# ---------------------------------------------------------------------------------------
# GMM EM step, torch semantics (diffICP/core/GMM.py:236-325) and log-likelihood (:714-721)
# ---------------------------------------------------------------------------------------
def log_ratio_to_proba(eta):                                  # GMM.py:205-217
    Z = torch.stack((torch.zeros_like(eta), eta), dim=0).logsumexp(dim=0)
    return eta - Z, -Z


def em_step(X, mu, w, sigma, to_optimize, outliers=None, skip_M=False):
    """Returns (Y, Cfe, FE, new_state) with new_state = dict(mu, w, sigma, outliers).
    Dense (N, C) -- fine at oracle sizes."""
    X = X.detach()
    N, D = X.shape
    dt = X.dtype
    outliers = None if outliers is None else dict(outliers)
    D2_nc = ((X[:, None, :] - mu[None, :, :]) ** 2).sum(-1)                   # :263
    lgn = D * (np.log(sigma) + 0.5 * np.log(2 * math.pi))                      # :264
    Zw = w.logsumexp(dim=0)
    t_nc = w[None, :] - Zw - D2_nc / (2 * sigma ** 2) - lgn                    # :269
    T_n = t_nc.logsumexp(dim=1)
    lgamma_nc = t_nc - T_n[:, None]
    gamma_nc = lgamma_nc.exp()
    if outliers is not None:                                                   # :275-282
        eta0 = outliers["eta0"]
        if outliers["vol0"] is None:
            outliers["vol0"] = (X.max(dim=0)[0] - X.min(dim=0)[0]).prod().item()
        logJ0 = -np.log(outliers["vol0"])
        eta0_n = eta0 + logJ0 - T_n
        lgamma0_n, lgammaT_n = log_ratio_to_proba(eta0_n)
    if not skip_M and to_optimize["mu"]:                                       # :286-287
        mu = torch.softmax(lgamma_nc, dim=0).t() @ X
    if not skip_M and outliers is not None and to_optimize.get("eta0", True):  # :289-290
        outliers["eta0"] = (lgamma0_n.logsumexp(dim=0) - lgammaT_n.logsumexp(dim=0)).item()
    if not skip_M and to_optimize["w"]:                                        # :292-293
        w = lgamma_nc.logsumexp(dim=0)
    if not skip_M and to_optimize["sigma"]:                                    # :295-297
        sigma = ((gamma_nc * D2_nc).sum() / (D * N)).sqrt().item()
    Y = (gamma_nc[:, :, None] * mu[None, :, :]).sum(1).reshape(N, D)          # :303
    lpi_c = w - w.logsumexp(dim=0)                                             # :312
    Cfe_n_comp = (gamma_nc * (((mu ** 2).sum(-1)[None, :] - (Y ** 2).sum(-1)[:, None])
                              / (2 * sigma ** 2) + lgamma_nc - lpi_c[None, :])).sum(dim=1) + lgn
    if outliers is None:
        Cfe = Cfe_n_comp.sum()
        FE = Cfe + (((X - Y) ** 2).sum(-1)).sum().item() / (2 * sigma ** 2)
    else:
        gamma0_n, gammaT_n = lgamma0_n.exp(), lgammaT_n.exp()
        lpi0, lpiT = log_ratio_to_proba(torch.tensor(outliers["eta0"], dtype=dt))
        Cfe = (gammaT_n * (Cfe_n_comp + lgammaT_n - lpiT)
               + gamma0_n * (-logJ0 + lgamma0_n - lpi0)).sum().item()
        FE = Cfe + (gammaT_n * ((X - Y) ** 2).sum(-1)).sum().item() / (2 * sigma ** 2)
    return Y, Cfe, FE, dict(mu=mu, w=w, sigma=sigma, outliers=outliers)


def log_likelihoods(X, mu, w, sigma):                          # GMM.py:714-721 (+:702-704)
    D = X.shape[1]
    weights_log = torch.log_softmax(w, 0) - D * math.log(sigma)
    return (-((X[:, None, :] - mu[None, :, :]) ** 2).sum(-1) / (2 * sigma ** 2)
            + weights_log[None, :]).logsumexp(dim=1) - D * (np.log(sigma) + 0.5 * np.log(2 * math.pi))


def em_step_keops_semantics(X, mu, w, sigma, to_optimize, skip_M=False):
    """KeOps-path EM (GMM.py:402-529) restated densely: sigma from the NEW mu (:453-456),
    lgn in Cfe from the NEW sigma (:483).  No outliers.  PARITY UNPINNED (KeOps absent)."""
    N, D = X.shape
    D2 = ((X[:, None, :] - mu[None, :, :]) ** 2).sum(-1)
    lgn = D * (np.log(sigma) + 0.5 * np.log(2 * math.pi))
    t = w[None, :] - D2 / (2 * sigma ** 2) - w.logsumexp(0) - lgn
    lg = t - t.logsumexp(1, keepdim=True)
    g = lg.exp()
    if not skip_M:
        if to_optimize["mu"]:
            mu = torch.softmax(lg, 0).t() @ X
        if to_optimize["w"]:
            w = lg.logsumexp(0)
        if to_optimize["sigma"]:
            D2n = ((X[:, None, :] - mu[None, :, :]) ** 2).sum(-1)
            sigma = ((g * D2n).sum() / (D * N)).sqrt().item()
    Y = g @ mu
    lpi = w - w.logsumexp(0)
    lgn2 = D * (np.log(sigma) + 0.5 * np.log(2 * math.pi))
    Cn = (g * (((mu ** 2).sum(-1)[None, :] - (Y ** 2).sum(-1)[:, None]) / (2 * sigma ** 2)
               + lg - lpi[None, :])).sum(1) + lgn2
    Cfe = Cn.sum()
    FE = Cfe + ((X - Y) ** 2).sum() / (2 * sigma ** 2)
    return Y, Cfe, FE, dict(mu=mu, w=w, sigma=sigma)
