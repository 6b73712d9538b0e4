"""Isotropic uniform-sigma Gaussian mixture with optional uniform outlier class; EM on gfx950.

Mirror of diffICP/core/GMM.py `GaussianMixtureUnif` (:40-383, :700-721): same state
(mu, sigma, w, outliers, to_optimize, ensure_continuum, spec), same EM_step return values
(Y, Cfe, FE) and the same EM_optimization stopping rule.  EM_step is bound to the HIP
implementation (`computversion="hip"`, alias "keops"): three fused N x C passes
(E-step LSE + weighted row sums, M-step column statistics, targets) instead of the
reference's dense (N, C) torch tensors or 5-6 separate KeOps reductions.

Semantics follow the reference's *torch* EM path (EM_step_torch, GMM.py:236-325), which is
the runnable, golden-pinned one: sigma from the OLD centroids (:296), lgn in Cfe from the
OLD sigma (:264/:314).  `em_semantics="keops"` selects the KeOps-path variant
(GMM.py:453-456, :483: sigma from the NEW centroids, lgn from the NEW sigma) -- parity
unpinned, since KeOps cannot run here.

Distributed (frame-sharded atlas): if `comm` is set (a torch.distributed process group
or the default group via comm=True), the per-rank sufficient statistics are exchanged with
all_gather and combined in rank order, so every rank holds bit-identical parameters.
"""
from __future__ import annotations

import copy
import os
import math
import weakref

import numpy as np
import torch
from torch.nn.functional import log_softmax, softmax

from .. import _lib
from ..tools.point_sets import intrinsic_scale
from ..tools import runstats
from ..tools.spec import defspec

# A/B switch (tools/probes/rowsplit_fe.py): DICP_ESTEP_HINT_ANY=1 restores the round-5 hint rule
_HINT_ANY = os.environ.get("DICP_ESTEP_HINT_ANY", "0") != "0"

_LOG2E = 1.4426950408889634


def _comm_active(comm):
    if comm is None or comm is False:
        return False
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized() and dist.get_world_size(
        None if comm is True else comm) > 1


def _group(comm):
    return None if comm is True else comm


def _gather_rows(t, comm):
    """all_gather a same-shaped tensor -> stacked (W, ...) in rank order."""
    import torch.distributed as dist
    W = dist.get_world_size(_group(comm))
    out = [torch.empty_like(t) for _ in range(W)]
    with runstats.collective():
        dist.all_gather(out, t.contiguous(), group=_group(comm))
    return torch.stack(out, 0)


def _comm_device():
    """Device the collectives run on: the current GPU for RCCL ("nccl"), else the CPU."""
    import torch.distributed as dist
    if dist.is_initialized() and dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def _sum_ranks(x, comm):
    """Deterministic cross-rank sum (gather + rank-ordered sum, float64)."""
    if not _comm_active(comm):
        return torch.as_tensor(x, dtype=torch.float64).reshape(1)[0]
    dev = x.device if isinstance(x, torch.Tensor) else _comm_device()
    t = torch.as_tensor(x, dtype=torch.float64).reshape(1).to(dev)
    return _gather_rows(t, comm).sum(0)[0]


def _sum_ranks_many(xs, comm):
    """Deterministic cross-rank sums of several scalars in ONE collective: each is taken to
    float64 (as _sum_ranks does), gathered, and summed in rank order."""
    dev = next((x.device for x in xs if isinstance(x, torch.Tensor)), None) or _comm_device()
    t = torch.stack([torch.as_tensor(x, dtype=torch.float64, device=dev).reshape(())
                     for x in xs]).reshape(-1, 1)
    g = _gather_rows(t, comm)                       # (W, n, 1)
    return [g[:, i].sum(0)[0] for i in range(len(xs))]


def _exchange(parts, comm):
    """ONE all_gather of several tensors: each is taken to float64 and flattened into one
    buffer (exact for the float32 statistics), gathered, and handed back per name as a
    (W, *shape) tensor of its own dtype, in rank order."""
    names = list(parts)
    dev = parts[names[0]].device
    flat = [parts[k].detach().to(device=dev, dtype=torch.float64).reshape(-1) for k in names]
    g = _gather_rows(torch.cat(flat), comm)         # (W, L)
    out, off = {}, 0
    for k, f in zip(names, flat):
        n = f.numel()
        out[k] = g[:, off:off + n].reshape((g.shape[0],) + tuple(parts[k].shape)).to(parts[k].dtype)
        off += n
    return out


class GaussianMixtureUnif(torch.nn.Module):

    def __init__(self, mu, sigma=None, use_outliers=False, spec=defspec, computversion="hip"):
        """Same arguments and defaults as GMM.py:42-109."""
        super().__init__()
        self.params = {}
        self.spec = spec
        self.mu = mu.clone().detach().to(**spec)
        self.C, self.D = self.mu.shape
        self.sigma = sigma
        if self.sigma is None:
            r = self.mu.var(0).sum().sqrt().item()
            self.sigma = 0.1 * (r / self.C ** (1 / self.D))
            self.sigma = max(self.sigma, 1e-6)
        self.w = torch.zeros(self.C, **spec)
        self.to_optimize = {"sigma": True, "mu": True, "w": True, "eta0": True}
        self.outliers = {"vol0": None, "eta0": 0.0} if use_outliers else None
        self.ensure_continuum = False
        self.em_semantics = "torch"
        self.comm = None
        self.set_computversion(computversion)

    def __deepcopy__(self, memo):
        G2 = GaussianMixtureUnif(self.mu, spec=self.spec, computversion=self.computversion)
        G2.sigma = self.sigma
        G2.w = self.w.clone().detach()
        G2.to_optimize = copy.deepcopy(self.to_optimize)
        G2.outliers = copy.deepcopy(self.outliers)
        G2.ensure_continuum = self.ensure_continuum
        G2.em_semantics = self.em_semantics
        G2.comm = self.comm
        return G2

    def set_computversion(self, version):
        """GMM.py:126-144.  "hip" (alias "keops"; "torch" is redirected to "hip")."""
        if version in ("keops", "torch"):
            version = "hip"
        if version != "hip":
            raise ValueError(f"unkown computversion : {version}. Choices are 'hip' (or 'keops')")
        self.EM_step = self.EM_step_hip
        self.computversion = version
        return self

    def fix(self):
        self.to_optimize = {"sigma": False, "mu": False, "w": False, "eta0": False}
        return self

    def set_vol0(self, X):
        """Outlier reference volume = bounding-box volume of X (GMM.py:163-171); global
        bounding box across ranks when sharded."""
        if self.outliers is not None:
            if X.shape[0] == 0:     # empty shard: neutral bounds for the cross-rank min / max
                lo = torch.full((X.shape[1],), float("inf"), dtype=X.dtype, device=X.device)
                hi = torch.full((X.shape[1],), float("-inf"), dtype=X.dtype, device=X.device)
            else:
                lo = X.min(dim=0)[0]
                hi = X.max(dim=0)[0]
            if _comm_active(self.comm):
                lo = _gather_rows(lo, self.comm).min(0)[0]
                hi = _gather_rows(hi, self.comm).max(0)[0]
            self.outliers["vol0"] = (hi - lo).prod().item()
        return self

    def __str__(self):
        s = super().__str__()
        s += ": Gaussian Mixture with Uniform covariances. Parameters:\n"
        s += "    C [# components] : " + str(self.C) + "\n"
        s += "    sigma [unif. std] : " + str(self.sigma) + "\n"
        s += "    mu_c [centroids] :" + str(self.mu) + "\n"
        s += "    w_c [component scores]:" + str(self.w) + "\n"
        if self.outliers is not None:
            s += "    vol0 [ref. volume for outliers]:" + str(self.outliers["vol0"]) + "\n"
            s += "    eta0 [outlier vs GMM log-ratio]:" + str(self.outliers["eta0"]) + "\n"
        return s

    def __getstate__(self):
        d = self.__dict__.copy()
        d.pop("_estep_hint", None)   # a weak reference to a point set: not state
        return d

    def __setstate__(self, state):
        self.__dict__.update(state)
        self.spec = defspec

    # ------------------------------------------------------------------------------------
    def log_ratio_to_proba(self, eta):
        """log p, log q of a Bernoulli with log-odds eta (GMM.py:205-217), on eta's device."""
        if not isinstance(eta, torch.Tensor):
            eta = torch.tensor(eta, **self.spec)
        Z = torch.stack((torch.zeros_like(eta), eta), dim=0).logsumexp(dim=0)
        return eta - Z, -Z

    def log_responsibilities(self, X):
        """(N,C) log-responsibilities (GMM.py:221-232).  Dense by definition (returns N x C)."""
        X = X.detach()
        D2_nc = ((X[:, None, :] - self.mu[None, :, :]) ** 2).sum(-1)
        return log_softmax(self.w[None, :] - D2_nc / (2 * self.sigma ** 2), dim=1)

    def _columns(self, mu, w):
        Zw = w.logsumexp(dim=0)
        lpi = (w - Zw).contiguous()
        return lpi, (lpi * _LOG2E).contiguous(), (mu * mu).sum(-1).contiguous()

    # ------------------------------------------------------------------------------------
    def EM_step_hip(self, X, skip_M=False):
        """One E + M step (GMM.py:236-325).  Returns (Y (N,D), Cfe, FE) like EM_step_torch."""
        X_in = X           # the caller's tensor object: the E-step hint's key (below)
        X = X.detach().contiguous()
        N, D = X.shape
        comm = self.comm
        dist_on = _comm_active(comm)
        keops_sem = self.em_semantics == "keops"

        mu_old = self.mu.contiguous()
        w_old = self.w
        sigma_old = float(self.sigma)
        lgn_old = self.D * (np.log(sigma_old) + 0.5 * np.log(2 * math.pi))
        lpi_old, w2_old, mu2_old = self._columns(mu_old, w_old)

        # ---- E step: T_n and responsibility-weighted row sums (old params) ----
        # the previous E-step's T2 over the same rows shifts the single exp sweep (a change of
        # reference: dicp_gmm_estep_hint_f32 -- without it a small sigma re-references most rows'
        # tiles; any hint is safe, a stale one only costs re-referencing)
        # The hint is taken only from an earlier E-step over the SAME X tensor object, unmodified
        # (weak reference to the caller's tensor + version counter): the steps of one
        # EM_optimization loop.  An E-step
        # result then depends on its inputs and the loop's own history only, never on EM calls
        # made earlier on other point sets of the same size.
        prev = getattr(self, "_estep_hint", None)
        hint = (prev[2] if (prev is not None and prev[0]() is X_in and prev[1] == X_in._version)
                else None)
        if _HINT_ANY and hint is None and prev is not None and prev[2].shape[0] == N:
            hint = prev[2]      # A/B only: the round-5 rule (any earlier E-step of the same size)
        T, T2, stats = _lib.gmm_estep(X, mu_old, w2_old, mu2_old, sigma_old, lgn_old, True, hint=hint)
        self._estep_hint = (weakref.ref(X_in), X_in._version, T2)
        E_row = stats[:, D + 1]                   # sum_c gamma lgamma

        if self.outliers is not None:
            eta0 = self.outliers["eta0"]
            if self.outliers["vol0"] is None:
                self.set_vol0(X)
            logJ0 = -np.log(self.outliers["vol0"])
            eta0_n = eta0 + logJ0 - T
            lgamma0_n, lgammaT_n = self.log_ratio_to_proba(eta0_n)

        # ---- M step ----
        need_col = (not skip_M) and (self.to_optimize["mu"] or self.to_optimize["w"])
        need_eta0 = not skip_M and self.outliers is not None and self.to_optimize["eta0"]
        need_sigma = not skip_M and self.to_optimize["sigma"]
        if need_col:
            colstats = _lib.gmm_mstep(X, T2, mu_old, w2_old, sigma_old)   # (C, D+1)
        if need_eta0:
            a = lgamma0_n.logsumexp(dim=0)
            b = lgammaT_n.logsumexp(dim=0)
        if need_sigma and not keops_sem:
            nds = stats[:, D + 3].sum()
        if dist_on and (need_col or need_eta0 or need_sigma):
            # ONE collective for everything the M step needs from the other ranks (SURVEY
            # 8(e)): the column statistics, the outlier LSE terms, the sigma numerator (torch
            # semantics: from the E-step rows) and the point count, packed into one buffer
            parts = {}
            if need_col:
                parts["col"] = colstats
            if need_eta0:
                parts["a"], parts["b"] = a, b
            if need_sigma:
                if not keops_sem:
                    parts["nds"] = nds.double()       # summed over ranks in float64
                parts["N"] = torch.tensor(float(N), dtype=torch.float64, device=X.device)
            ex = _exchange(parts, comm)
            if need_col:
                g = ex["col"]                                             # (W, C, D+1)
                lw = g[:, :, 0]
                Wg = lw.logsumexp(0)
                wt = torch.exp(lw - Wg[None, :])
                wt = torch.where(torch.isfinite(wt), wt, torch.zeros_like(wt))
                mu_new = (wt[:, :, None] * g[:, :, 1:]).sum(0) / wt.sum(0)[:, None]
                w_new = Wg
            if need_eta0:
                a = ex["a"].reshape(-1, 1).logsumexp(0)[0]
                b = ex["b"].reshape(-1, 1).logsumexp(0)[0]
            if need_sigma:
                if not keops_sem:
                    nds = ex["nds"].reshape(-1, 1).sum(0)[0]
                Ntot = int(ex["N"].reshape(-1, 1).sum(0)[0].item())
        elif need_col:
            w_new = colstats[:, 0].contiguous()
            mu_new = colstats[:, 1:].contiguous()
        if need_col and self.to_optimize["mu"]:
            self.mu = mu_new.contiguous()
        if need_eta0:
            self.outliers["eta0"] = (a - b).item()
        if need_col and self.to_optimize["w"]:
            self.w = w_new.contiguous()

        changed = need_col   # mu or w changed -> second row pass with the new columns
        if changed or keops_sem:
            lpi_new, _, _ = self._columns(self.mu, self.w)
            rows = _lib.gmm_targets(X, T2, mu_old, w2_old, sigma_old, self.mu.contiguous(), lpi_new)
            # renormalise by sum_c gamma (= 1 exactly; removes the bias that the fp32
            # rounding of the stored log-normaliser T2 would put on every weighted sum)
            inv = 1.0 / rows[:, D + 2]
            Y = rows[:, :D] * inv[:, None]
            P_row = rows[:, D + 1] * inv
            D2new_row = rows[:, D + 3] * inv
        else:
            Y = stats[:, :D]
            P_row = stats[:, D + 2]
            D2new_row = None

        if need_sigma:
            if keops_sem:
                # KeOps semantics: sigma from the NEW centroids' rows -- a second exchange
                nds = D2new_row.sum()
                if dist_on:
                    nds = _sum_ranks(nds, comm)
            if not dist_on:
                Ntot = N
            self.sigma = torch.sqrt(nds / (self.D * Ntot)).item()
            if self.ensure_continuum:      # (experimental) GMM.py:298-299 / :457-458
                self.sigma = max(self.sigma, intrinsic_scale(self.mu))

        # ---- targets and free energy (GMM.py:303-323) ----
        Y = Y.contiguous()
        sig2x2 = 2 * self.sigma ** 2
        lgn_c = self.D * (np.log(self.sigma) + 0.5 * np.log(2 * math.pi)) if keops_sem else lgn_old
        # sum_c gamma (|mu_c|^2 - |Y_n|^2) (GMM.py:313) evaluated shift-invariantly about x_n:
        # = sum_c gamma |mu_c - x_n|^2 - |Y_n - x_n|^2 (identical in exact arithmetic since
        # sum_c gamma = 1; avoids the fp32 cancellation of two O(|x|^2) terms).
        DD_row = D2new_row if (changed or keops_sem) else stats[:, D + 3]
        quad_n = ((X - Y) ** 2).sum(-1)
        Cfe_n_comp = (DD_row - quad_n) / sig2x2 + E_row - P_row + lgn_c
        if self.outliers is None:
            Cfe = Cfe_n_comp.sum()
            q = quad_n.sum()
            if dist_on:       # one scalar exchange for the free energy's two sums
                Cfe, q = _sum_ranks_many((Cfe, q), comm)
                Cfe = Cfe.to(X.dtype)
            FE = Cfe + q.item() / sig2x2
        else:
            gamma0_n = lgamma0_n.exp()
            gammaT_n = lgammaT_n.exp()
            lpi0, lpiT = self.log_ratio_to_proba(self.outliers["eta0"])
            Cfe = (gammaT_n * (Cfe_n_comp + lgammaT_n - lpiT)
                   + gamma0_n * (-logJ0 + lgamma0_n - lpi0)).sum()
            q = (gammaT_n * quad_n).sum()
            if dist_on:
                Cfe, q = _sum_ranks_many((Cfe, q), comm)
            Cfe = Cfe.item()
            FE = Cfe + q.item() / sig2x2
        return Y, Cfe, FE

    # ------------------------------------------------------------------------------------
    def EM_optimization(self, X, max_iterations=100, tol=1e-5):
        """Iterated EM until |FE - FE_prev| < tol |FE_prev| (GMM.py:330-357).
        Returns (Y, Cfe, FE, number of EM steps)."""
        if X.shape[0] == 0 and not _comm_active(self.comm):
            return torch.empty(X.shape, **defspec), torch.tensor(0.0), torch.tensor(0.0), 0
        Y, Cfe, FE, last_FE = None, None, None, None
        for i in range(max_iterations):
            runstats.add("em_steps")
            Y, Cfe, FE = self.EM_step(X)
            if last_FE is not None and tol is not None and abs(FE - last_FE) < tol * abs(last_FE):
                return Y, Cfe, FE, i + 1
            last_FE = FE
        print(f"GMM optimization - reached maximum number of iterations : {max_iterations}")
        return Y, Cfe, FE, i + 1

    @staticmethod
    def get_GMM_model(X, C, fixed_sigma=None, optimize_w=False, use_outliers=False,
                      max_iterations=100, tol=1e-5, spec=defspec, computversion="hip"):
        """C centroids drawn from X, then EM (GMM.py:361-383)."""
        mu = X[torch.randint(0, X.shape[0], (C,)), :]
        GMM = GaussianMixtureUnif(mu, use_outliers=use_outliers, spec=spec,
                                  computversion=computversion)
        GMM.to_optimize = {"mu": True, "sigma": True, "w": optimize_w, "eta0": True}
        if fixed_sigma is not None:
            GMM.to_optimize["sigma"] = False
            GMM.sigma = fixed_sigma
        GMM.EM_optimization(X, max_iterations=max_iterations, tol=tol)
        return GMM

    # ------------------------------------------------------------------------------------
    def pi(self):
        return softmax(self.w, dim=0)

    def update_covariances(self):
        pass

    def weights(self):
        return softmax(self.w, 0) / self.sigma ** self.D

    def weights_log(self):
        return log_softmax(self.w, 0) - self.D * math.log(self.sigma)

    def log_likelihoods(self, sample):
        """Log-density on a point cloud (GMM.py:714-721): LSE_c(-D2/2s^2 + weights_log)
        - D (log s + 0.5 log 2pi) = T_n - D log s  (the reference divides by sigma^D twice;
        reproduced)."""
        sample = sample.to(**self.spec).contiguous()
        lpi, w2, mu2 = self._columns(self.mu.contiguous(), self.w)
        lgn = self.D * (np.log(self.sigma) + 0.5 * np.log(2 * math.pi))
        T, _, _ = _lib.gmm_estep(sample, self.mu.contiguous(), w2, mu2, float(self.sigma), lgn, False)
        return T - self.D * np.log(self.sigma)

    def likelihoods(self, sample):
        return self.log_likelihoods(sample).exp()

    def get_sample(self, N):
        """N points from the mixture, same RNG call order as GMM.py:543-550."""
        samp = self.sigma * torch.randn(N, self.D, **self.spec)
        c = torch.distributions.categorical.Categorical(logits=self.w).sample((N,))
        return samp + self.mu[c.to(self.mu.device)]
