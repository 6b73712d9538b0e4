"""Standard (Glaunes-style) point-set registration with template estimation: mirror of
diffICP/core/PSR_standard.py on the HIP path.

The data attachment is the RKHS distance between point clouds seen as signed measures
(`data_distance`, PSR_standard.py:37-58), built from the KBase / KRedScal reductions
(dicp_gauss_red_f32, differentiable through tools/kernel.py); the registrations are the
fused LDDMM shootings (core/shooting.py) -- dense support: warped template = q1; other
support schemes: the template is carried as external points (x).  `MultiPSR_std` /
`DiffPSR_std` keep the reference's attributes (y0, y1, x, Nx, Ny, w0, a0, q0, shoot,
regloss, dataloss, E), call order and energy bookkeeping.  AffinePSR_std (affine
registrations, not on the kernel hot path) is out of scope.

Reference quirks kept or fixed:
  * the loss accumulators of Reg_opt / Template_opt start from `torch.tensor([0.0])`, a
    float32 CPU tensor (PSR_standard.py:235, :519): their sums are float32 in the reference,
    kept float32 here but created on the computation device (the reference's breaks on GPU);
  * data_distance(x, x) terms do not depend on the optimised variables; they are still
    evaluated (same values, same energy), once per call as in the reference.
"""
from __future__ import annotations

import warnings

import numpy as np
import torch

from ..tools.in_out import read_point_sets
from ..tools.kernel import GenKernel
from ..tools.optim import LBFGS_optimization
from ..tools.point_sets import decimate
from ..tools.spec import defspec
from .LDDMM import LDDMMModel
from .registrations import LDDMMRegistration


def data_distance(Kernel: GenKernel, x, y, w=None):
    """RKHS distance between the data cloud x (weights 1/Nx) and the template y (weights 1/Ny,
    or -w) -- PSR_standard.py:37-58:
        L = sum_ij c_i c_j K(X_i, X_j),  X = (y, x)."""
    KB = Kernel.KBase
    Nx = x.shape[0]
    Ny = y.shape[0]
    if w is None:
        return KB(x, x).sum() / Nx ** 2 + KB(y, y).sum() / Ny ** 2 - 2 * KB(y, x).sum() / (Nx * Ny)
    KRS = Kernel.KRedScal
    return (KB(x, x).sum() / Nx ** 2 + (KRS(y, y, w).flatten() * w).sum()
            - 2 * (KB(y, x).flatten() * w).sum() / Nx)


def _acc_zero(spec):
    # torch.tensor([0.0]) of the reference: float32, here on the computation device
    return torch.zeros(1, dtype=torch.float32, device=spec["device"])


class MultiPSR_std:
    """Base class (PSR_standard.py:67-357)."""

    def __init__(self, x, y_template, noise_std, DataKernel: GenKernel, template_weights=False,
                 dataspec=defspec, compspec=defspec):
        self.dataspec, self.compspec = dataspec, compspec
        self.DataKernel = DataKernel
        self.printstuff = True
        x, self.K, self.S, self.D = read_point_sets(x)
        if isinstance(y_template, torch.Tensor):
            self.y0 = [y_template.clone().contiguous().detach().to(**self.dataspec) for _ in range(self.S)]
        else:
            if not isinstance(y_template, list) or len(y_template) != self.S:
                raise ValueError("y_template should be a single point set (torch tensor), or a list with S point sets")
            self.y0 = [y.clone().contiguous().detach().to(**self.dataspec) for y in y_template]
        self.noise_std = noise_std if isinstance(noise_std, list) else [noise_std] * self.S
        assert len(self.noise_std) == self.S
        self.y1 = np.empty((self.K, self.S), dtype=object)
        self.x = np.empty((self.K, self.S), dtype=object)
        for s in range(self.S):
            for k in range(self.K):
                self.x[k, s] = x[k][s].contiguous().detach().to(**self.dataspec)
                self.y1[k, s] = self.y0[s].clone().contiguous().detach().to(**self.dataspec)
        self.Nx = np.array([[self.x[k, s].shape[0] for s in range(self.S)] for k in range(self.K)])
        self.Ny = np.array([self.y0[s].shape[0] for s in range(self.S)])
        self.ally0 = torch.cat(tuple(self.y0), dim=0).clone().to(**self.compspec).detach().contiguous()
        self.template_weights = template_weights
        if self.template_weights:
            self.w0 = [torch.ones(int(self.Ny[s]), **self.compspec) / int(self.Ny[s]) for s in range(self.S)]
        else:
            self.w0 = [None] * self.S
        self.shoot = [None] * self.K
        self.regloss = [0] * self.K
        self.dataloss = np.zeros((self.K, self.S))
        for k in range(self.K):
            for s in range(self.S):
                self.dataloss[k, s] = float(data_distance(self.DataKernel, self.x[k, s], self.y0[s],
                                                          self.w0[s])) / self.noise_std[s] ** 2
        self.E = sum(float(r) for r in self.regloss) + self.dataloss.sum().item()

    def __setstate__(self, state):
        self.__dict__.update(state)
        self.dataspec = defspec
        self.compspec = defspec

    def get_template(self, s=0):
        return self.y0[s]

    def get_warped_template(self, k=0, s=0):
        return self.y1[k, s]

    def get_data_points(self, k=0, s=0):
        return self.x[k, s]

    def Registration(self, k=0):
        """Registration object of frame k (PSR_standard.py:211-224)."""
        if isinstance(self, DiffPSR_std):
            return LDDMMRegistration(self.LMi, self.q0, self.a0[k])
        raise NotImplementedError("AffinePSR_std is out of scope of difficp_amd")

    def Template_opt(self, nmax=10, tol=1e-3, errthresh=1e8):
        """Optimise each template y0[s] (and its weights) through all frames' registrations
        (PSR_standard.py:226-257)."""
        for s in range(self.S):

            def lossfunc(y0s, ws):
                L = _acc_zero(self.compspec)
                for k in range(self.K):
                    L += data_distance(self.DataKernel, self.x[k, s], self.Registration(k).apply(y0s), ws)
                return L

            if self.template_weights:
                p, L, nsteps, change = LBFGS_optimization([self.y0[s], self.w0[s]], lossfunc, nmax=nmax,
                                                          tol=tol, errthresh=errthresh)
                self.y0[s] = p[0]
                self.w0[s] = p[1]
            else:
                p, L, nsteps, change = LBFGS_optimization([self.y0[s]], lambda y0s: lossfunc(y0s, None),
                                                          nmax=nmax, tol=tol, errthresh=errthresh)
                self.y0[s] = p[0]
            self.update_state(s=s, caller=self.Template_opt)
            if self.printstuff:
                print(f"Template {s} : {nsteps} optim steps, loss={L:.4}, change={change:.4}.".ljust(70)
                      + f"Total energy = {self.E:.8}")

    def Reg_opt(self, tol=1e-5):
        raise NotImplementedError("function Reg_opt must be written in derived classes.")

    def update_state(self, k=None, s=None, caller=None):
        """Recompute warped templates, data losses, regloss, support points and E
        (PSR_standard.py:269-318)."""
        klist = range(self.K) if k is None else [k]
        slist = range(self.S) if s is None else [s]
        for kk in klist:
            for ss in slist:
                if caller != self.Reg_opt:
                    self.y1[kk, ss] = self.Registration(kk).apply(self.y0[ss]).detach()
                self.dataloss[kk, ss] = float(data_distance(self.DataKernel, self.x[kk, ss], self.y1[kk, ss],
                                                            self.w0[ss])) / self.noise_std[ss] ** 2
        if caller is None and isinstance(self, DiffPSR_std):
            for kk in klist:
                self.regloss[kk] = float(self.LMi.trajloss(self.Registration(kk).shoot(None)))
        if caller == self.Template_opt:
            self.ally0 = torch.cat(tuple(self.y0), dim=0).clone().to(**self.compspec).detach().contiguous()
            if isinstance(self, DiffPSR_std):
                q0_prev = self.q0
                if self.support_scheme is None:
                    self.q0 = self.ally0
                    self.update_a0(q0_prev, rcond=1e-1)
                elif self.support_scheme == "decim":
                    self.set_support_scheme("decim", self.rho)
        E = sum(float(r) for r in self.regloss) + self.dataloss.sum().item()
        if self.E is not None and E > self.E:
            warnings.warn("WARNING: measured increase in optimization energy ! Should not happen.")
            print("WARNING: measured increase in optimization energy ! Should not happen.")
        self.E = E


class DiffPSR_std(MultiPSR_std):
    """MultiPSR_std with LDDMM registrations (PSR_standard.py:364-566)."""

    def __init__(self, x, y_template, noise_std, LMi: LDDMMModel, DataKernel: GenKernel,
                 template_weights=False, dataspec=defspec, compspec=defspec, v2p_args=None):
        super().__init__(x, y_template, noise_std, DataKernel=DataKernel, template_weights=template_weights,
                         dataspec=dataspec, compspec=compspec)
        if LMi.Kernel.spec != compspec:
            raise ValueError("Spec (dtype+device) error : LDDMMmodel 'spec' and diffPSR 'compspec' "
                             "attributes should be the same")
        self.LMi = LMi
        self.v2p_args = dict(v2p_args or {})   # as DiffPSR (core/PSR.py): None = reference defaults
        self.support_scheme = None
        self.q0 = self.ally0
        self.a0 = [None] * self.K
        self.initialize_a0()

    def initialize_a0(self, **v2p_args):
        """a0 at zero speeds (PSR_standard.py:422-428)."""
        v2p_args = v2p_args or self.v2p_args
        for k in range(self.K):
            v0 = torch.zeros(self.q0.shape, **self.compspec)
            self.a0[k] = self.LMi.v2p(self.q0, v0, **v2p_args)

    def update_a0(self, q0_prev, a0_prev=None, **v2p_args):
        """Project the previous field on the new support (PSR_standard.py:430-443)."""
        if self.v2p_args and not v2p_args.get("version"):
            v2p_args = {**self.v2p_args, **{k: v for k, v in v2p_args.items() if k != "rcond"}}
        if a0_prev is None:
            a0_prev = self.a0
        for k in range(self.K):
            v0 = self.LMi.v(self.q0, q0_prev, a0_prev[k])
            self.a0[k] = self.LMi.v2p(self.q0, v0, **v2p_args)

    def set_support_scheme(self, scheme="decim", rho=1.0, xticks=None, yticks=None, q0=None):
        """Support points of the template (PSR_standard.py:445-503): "decim" (device greedy
        decimation, point_sets.py:102-133), "grid" (2D) or "custom"."""
        self.rho = rho
        Rcover = rho * self.LMi.Kernel.sigma
        self.support_scheme = scheme
        q0_prev = self.q0
        if scheme == "decim":
            supp_ids = [decimate(self.y0[s].to(**self.compspec), Rcover)[0] for s in range(self.S)]
            Ndecim = sum(len(i) for i in supp_ids)
            if self.printstuff:
                print(f"Decimation : {Ndecim} support points ({Ndecim / sum(self.Ny):.0%} of original sets)")
            self.q0 = torch.cat(tuple(self.y0[s][supp_ids[s]] for s in range(self.S)),
                                dim=0).to(**self.compspec).contiguous()
        elif scheme == "grid":
            if self.D != 2:
                raise ValueError("grid support scheme is 2D only (as in the reference)")
            if xticks is None or yticks is None:
                # get_bounds(*y0, relmargin=0.1) (visualization/visu.py:35-50)
                ys = [a.detach().cpu() for a in self.y0 if len(a) > 0]
                mins = torch.cat(tuple(a.min(0).values.reshape(1, 2) for a in ys), 0).min(0).values.numpy()
                maxs = torch.cat(tuple(a.max(0).values.reshape(1, 2) for a in ys), 0).max(0).values.numpy()
                gmin = (1 + 0.1) * mins - 0.1 * maxs
                gmax = (1 + 0.1) * maxs - 0.1 * mins
                xmin, xmax, ymin, ymax = gmin[0], gmax[0], gmin[1], gmax[1]
            if xticks is None:
                xticks = np.arange(xmin - Rcover / 2, xmax + Rcover / 2, Rcover)
            if yticks is None:
                yticks = np.arange(ymin - Rcover / 2, ymax + Rcover / 2, Rcover)
            gp = np.stack(np.meshgrid(xticks, yticks), axis=2)
            self.q0 = torch.tensor(gp.reshape((-1, 2), order="F"), **self.compspec).contiguous()
        elif scheme == "custom":
            assert q0 is not None, "For a custom support scheme, please specify argument q0"
            self.q0 = q0.clone().detach().to(**self.compspec).contiguous()
        else:
            raise ValueError(f"Unknown value of support point scheme : {scheme}. Only values available "
                             "are 'decim', 'grid' and 'custom'.")
        self.update_a0(q0_prev, rcond=1e-2)

    def Reg_opt(self, nmax=10, tol=1e-3):
        """LDDMM registration of the template to each frame (PSR_standard.py:507-566)."""
        for k in range(self.K):

            def dataloss_func(y):
                L = _acc_zero(self.compspec)
                last = 0
                for s in range(self.S):
                    first, last = last, last + int(self.Ny[s])
                    L += data_distance(self.DataKernel, self.x[k, s], y[first:last], self.w0[s]) / self.noise_std[s] ** 2
                return L

            if self.support_scheme is None:
                self.a0[k], self.shoot[k], self.regloss[k], datal, isteps, change = \
                    self.LMi.Optimize(dataloss_func, self.q0, self.a0[k], tol=tol, nmax=nmax)
                ally1k = self.shoot[k][-1][0]
            else:
                self.a0[k], self.shoot[k], self.regloss[k], datal, isteps, change = \
                    self.LMi.Optimize(dataloss_func, self.q0, self.a0[k], self.ally0, tol=tol, nmax=nmax)
                ally1k = self.shoot[k][-1][-1]
            last = 0
            for s in range(self.S):
                first, last = last, last + int(self.Ny[s])
                self.y1[k, s] = ally1k[first:last].to(**self.dataspec)
            if self.support_scheme is not None:
                Rcoverwarning = 2.0
                for t in range(len(self.shoot[k])):
                    qk, yk = self.shoot[k][t][0], self.shoot[k][t][-1]
                    unc = self.LMi.Kernel.check_coverage(yk, qk, Rcoverwarning)
                    if unc.any():
                        print(f"WARNING : shooting, time step {t} : {unc.sum()} uncovered points "
                              f"({unc.sum() / yk.shape[0]:.2%})")
                        warnings.warn("Uncovered points during LDDMM shooting. Choose a smaller rho when "
                                      "defining the support scheme.", RuntimeWarning)
            self.update_state(k=k, caller=self.Reg_opt)
            if self.printstuff:
                print(f"Frame {k} : {isteps} optim steps, loss={float(self.regloss[k]) + float(datal):.4}, "
                      f"change={change:.4}.".ljust(70) + f"Total energy = {self.E:.8}")
