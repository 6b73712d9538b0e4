"""LDDMM model for point sets (classic / hybrid / logdet), HIP-backed.

Mirror of diffICP/core/LDDMM.py:28-398 (`LDDMMModel`): same constructor, attributes and
methods (v, mdivsum, Hamiltonian, dtrajcost, ODE, v2p, random_p, Shoot, trajloss,
BasicQuadLossFunctor, Optimize), same return conventions.  The vector field is
    v(x) = sum_j [p_j K(x - q_j) - eta (grad K)(x - q_j)],  eta = 1/lambda or 0.
What changes is where the arithmetic happens: Shoot() runs the fused trajectory of
core/shooting.py (one fused HIP pass per ODE evaluation, exact discrete adjoint for the
backward) instead of the reference's per-reduction integrator loop.
"""
from __future__ import annotations

import math
import os
import threading
import weakref

import torch

from .. import _lib
from ..tools.integrators import EulerIntegrator, RalstonIntegrator
from ..tools.kernel import GaussKernel, SVDpow
from ..tools.optim import LBFGS_optimization
from ..tools.spec import defspec, getspec
from .shooting import (HamiltonianFn, OdeExtFn, OdeFn, RowOrderCache, ShootCache, ShootFn,
                       complete_p1, row_order_for, skip_p1)



# per host thread: (q0 weak reference, q0 version, sigma, extent / sigma) of the last support
# whose extent was read (LDDMMModel._raw_for): one device read per new q0 tensor
_EXTENT_MEMO = threading.local()

# Optimize's closures form loss and gradient without the autograd engine where the loss allows
# (shooting.shoot_loss_grad; env DICP_DIRECT_LOSSGRAD=0: always through autograd)
_DIRECT_LOSSGRAD = os.environ.get("DICP_DIRECT_LOSSGRAD", "1") != "0"

class Shoot(list):
    """A "shoot" variable: list of (q, p, cost[, x]) states at the nt+1 integration times
    (LDDMM.py:286-299).  The states are views into stacked trajectory tensors Q, P, C[, X]
    that stay resident on the device."""

    # The state views are formed when read: a closure reads shoot[-1] (and trajloss shoot[0]),
    # and forming all 3 (nt+1) views of every shooting was ~1500 tensor selects per diff-ICP
    # iteration, ~8% of the host floor at 2k points (tools/host_floor.py).  Indexing by an int
    # forms (and keeps) that state only.  Any other list operation first fills the list's own
    # storage with every state; from then on (`_full`) the storage is authoritative, so list
    # mutators, concatenation and comparisons behave as on a plain list.
    def __init__(self, Q, P, C, X=None, H0=None):
        super().__init__()
        self.Q, self.P, self.C, self.X = Q, P, C, X
        self.H0 = H0   # H(q0, p0) from the first ODE evaluation (differentiable), or None
        self._n = Q.shape[0]
        self._states = {}
        self._full = False

    def _state(self, t):
        if t < 0:
            t += self._n
        if not 0 <= t < self._n:
            raise IndexError("shoot index out of range")
        s = self._states.get(t)
        if s is None:
            Q, P, C, X = self.Q, self.P, self.C, self.X
            s = (Q[t], P[t], C[t]) if X is None else (Q[t], P[t], C[t], X[t])
            self._states[t] = s
        return s

    def _fill(self):
        if not self._full:
            items = [self._state(t) for t in range(self._n)]
            super().clear()
            super().extend(items)
            self._full = True

    def __getitem__(self, k):
        if self._full:
            return super().__getitem__(k)
        if isinstance(k, int):
            return self._state(k)
        self._fill()
        return super().__getitem__(k)

    def __len__(self):
        return super().__len__() if self._full else self._n

    def __iter__(self):
        if self._full:
            return super().__iter__()
        return (self._state(t) for t in range(self._n))

    def __reversed__(self):
        if self._full:
            return super().__reversed__()
        return (self._state(t) for t in reversed(range(self._n)))

    def __bool__(self):
        return len(self) > 0

    __hash__ = None

    def __radd__(self, other):
        # other + shoot: list.__add__ would read this object's (possibly unfilled) storage
        return list(other) + list(self)

    def copy(self):
        return list(self)

    def __reduce__(self):
        """Pickle / deepcopy: the stacked tensors and attributes, plus the states themselves
        once the list was filled (it may have been mutated since)."""
        state = {k: v for k, v in self.__dict__.items() if k != "_states"}
        if self._full:
            state["_items"] = list(super().__iter__())
        return (Shoot, (self.Q, self.P, self.C, self.X, self.H0), state)

    def __setstate__(self, state):
        items = state.pop("_items", None)
        self.__dict__.update(state)
        self._states = {}
        super().clear()
        if items is not None:
            super().extend(items)
            self._full = True
        else:
            self._full = False

    def detach(self):
        d = lambda t: None if t is None else t.detach()
        sh = Shoot(d(self.Q), d(self.P), d(self.C), d(self.X), d(self.H0))
        for k in ("p1_missing", "raw", "q0_key"):     # LDDMMModel.complete_shoot's inputs
            if hasattr(self, k):
                setattr(sh, k, getattr(self, k))
        return sh


def _fill_first(name):
    """list method `name` on a Shoot, after its storage is filled with every state."""
    base = getattr(list, name)

    def f(self, *a, **k):
        self._fill()
        for o in a:   # list's C methods read another Shoot's storage directly
            if isinstance(o, Shoot):
                o._fill()
        return base(self, *a, **k)

    f.__name__ = name
    f.__doc__ = base.__doc__
    return f


for _m in ("append", "extend", "insert", "pop", "remove", "sort", "reverse", "clear", "index",
           "count", "__setitem__", "__delitem__", "__iadd__", "__imul__", "__add__", "__mul__",
           "__rmul__", "__contains__", "__eq__", "__ne__", "__lt__", "__le__", "__gt__", "__ge__",
           "__repr__"):
    setattr(Shoot, _m, _fill_first(_m))
del _m


class LDDMMModel:

    def __init__(self, sigma=1.0, D=2, lambd=2.0, spec=defspec, gradcomponent=True,
                 withlogdet=True, version=None, computversion="hip", scheme="Ralston",
                 nonsupprev=False, nt=10):
        """Same arguments as LDDMM.py:33-65.  `version` in {classic, logdet, hybrid}
        overrides (gradcomponent, withlogdet)."""
        self.Kernel = GaussKernel(sigma, D, computversion=computversion, spec=spec)
        self.D = D
        self.lam = lambd
        self.nt = nt
        if version == "classic":
            gradcomponent, withlogdet = False, False
        elif version == "logdet":
            gradcomponent, withlogdet = True, True
        elif version == "hybrid":
            gradcomponent, withlogdet = False, True
        self.withlogdet = withlogdet
        self.gradcomponent = gradcomponent
        self.eta = 1.0 / lambd if gradcomponent else 0
        self.nonsupprev = nonsupprev
        self.scheme, self.Integrator = None, None
        self.set_integration_scheme(scheme)
        self.try_trajcost_optim = False
        self.row_split = None
        # spatial visit order of the support rows for the fused forward passes (shooting.py
        # spatial_order), memoised per q0 (the support points are fixed over an L-BFGS run);
        # only the matrix-core forward (library option fwd_alg 3) uses it: set
        # `row_orders = RowOrderCache()` together with that option
        self.row_orders = None
        # the latest trajectory per q0, reused bitwise when the same shooting is asked for
        # again (shooting.ShootCache: the first closure of each Reg_opt L-BFGS run)
        self.shoot_cache = ShootCache()

    def set_row_split(self, group=None, enable=True, exact_reduce=None, verify=None, overlap=None):
        """Split every dense Euler shooting of this model over the ranks of a torch.distributed
        group (extension; core/rowsplit.py): all ranks must make the same
        calls (the host logic runs replicated).  enable=False restores single-device shooting.
        exact_reduce / verify / overlap: see RowSplit (rank-ordered VJP sums / cross-rank bit
        checks / forward steps in column phases overlapping the all-gathers).
        The L-BFGS divergence fallback draws from a generator seeded identically on every rank
        (tools/optim.py), so the replicated iterates stay in lockstep whatever each rank's
        global RNG state is."""
        from .rowsplit import RowSplit
        self.row_split = (RowSplit(group, exact_reduce=exact_reduce, verify=verify, overlap=overlap)
                          if enable else None)

    def set_integration_scheme(self, scheme: str):
        self.scheme = scheme
        if scheme == "Euler":
            self.Integrator = EulerIntegrator
        elif scheme == "Ralston":
            self.Integrator = RalstonIntegrator
        else:
            raise ValueError(f"Unkown numerical scheme : {scheme}")

    def __setstate__(self, state):
        self.__dict__.update(state)
        if self.__dict__.get("row_orders") is not None:
            self.row_orders = RowOrderCache()
        self.shoot_cache = ShootCache()
        self.Kernel = GaussKernel(self.Kernel.sigma, self.Kernel.D, self.Kernel.computversion,
                                  spec=defspec)

    @property
    def sigma(self):
        return self.Kernel.sigma

    # ------------------------------------------------------------------------------------
    def v(self, x, q, p):
        """v(x) = KRed(x,q,p) - eta GradKRed(x,q)   (LDDMM.py:100-116)."""
        spec = getspec(x, q, p)
        if x.numel() == 0:
            return torch.empty(x.shape, **spec)
        if self.gradcomponent:
            return self.Kernel.KRed(x, q, p) - self.eta * self.Kernel.GradKRed(x, q)
        return self.Kernel.KRed(x, q, p)

    def mdivsum(self, x, q, p, rev=False):
        """-sum_k div v(x_k), shape (1,)-compatible scalar (LDDMM.py:120-138)."""
        spec = getspec(x, q, p)
        if x.numel() == 0:
            return torch.tensor([0.0], **spec)
        if rev:
            r = self.Kernel.GradKRed_rev(q, x, p).sum()
        else:
            r = (p * self.Kernel.GradKRed(q, x)).sum()
        if self.gradcomponent:
            r = r + self.eta * self.Kernel.LapKRed(q, x).sum()
        return r

    def Hamiltonian(self, q, p):
        """H(q,p) = 1/2 sum_ij [p_i.p_j K - eta (p_i-p_j).gradK - eta^2 LapK]  (LDDMM.py:142-159),
        one fused HIP pass."""
        getspec(q, p)
        return HamiltonianFn.apply(q.contiguous(), p.contiguous(), self.Kernel.sigma, float(self.eta))

    def dtrajcost(self, q, p):
        """lambda*H(q,p) + mdivsum(q,q,p) variant (LDDMM.py:163-172)."""
        getspec(q, p)
        return 0.5 * self.lam * (p * self.Kernel.KRed(q, q, p)).sum() \
            + 0.5 * self.eta * self.Kernel.LapKRed(q, q).sum()

    def ODE(self, q, p, cost, x=None):
        """d/dt (q, p, cost[, x]) (LDDMM.py:176-227); one fused HIP pass (+1 for x)."""
        spec = getspec(q, p, cost, x)
        want_div = bool(self.withlogdet)
        if self.try_trajcost_optim and self.withlogdet and self.gradcomponent and x is None:
            vq, mG, _ = OdeFn.apply(q.contiguous(), p.contiguous(), self.Kernel.sigma,
                                    float(self.eta), False)
            return vq, mG, self.dtrajcost(q, p).reshape(1)
        if x is None:
            vq, mG, dcost = OdeFn.apply(q.contiguous(), p.contiguous(), self.Kernel.sigma,
                                        float(self.eta), want_div)
            if not want_div:
                dcost = torch.tensor([0.0], **spec)
            return vq, mG, dcost
        vq, mG, dcost, vx = OdeExtFn.apply(q.contiguous(), p.contiguous(), x.contiguous(),
                                           self.Kernel.sigma, float(self.eta), want_div)
        if not want_div:
            dcost = torch.tensor([0.0], **spec)
        return vq, mG, dcost, vx

    # ------------------------------------------------------------------------------------
    def v2p(self, q, v, rcond=1e-3, alpha=1e-4, version="pinv"):
        """Momenta p with v(q,q,p) ~= v (LDDMM.py:235-253)."""
        getspec(q, v)
        rhs = v if self.eta == 0 else v + self.eta * self.Kernel.GradKRed(q, q)
        if version == "pinv":
            return self.Kernel.KpinvSolve(q, rhs, rcond)
        elif version in ("ridge_keops", "ridge_hip"):
            # device CG with the KRed mat-vec (KeOps LazyTensor.solve semantics)
            return self.Kernel.KridgeSolve_keops(q, rhs, alpha)
        elif version == "ridge_pytorch":
            return self.Kernel.KridgeSolve_pytorch(q, rhs, alpha)
        raise ValueError("unknown version")

    def random_p(self, q, rcond=1e-3, alpha=1e-4, version="svd"):
        """Momenta drawn from exp(-lambda H(q,p)) (LDDMM.py:257-280)."""
        spec = getspec(q)
        if self.eta != 0:
            raise ValueError("random_p not implemented yet when gradcomponent=True.")
        K = (-(q[:, None, :] - q[None, :, :]) ** 2 / (2 * self.Kernel.sigma ** 2)).sum(-1).exp()
        zeta = torch.randn(q.shape, **spec) / math.sqrt(self.lam)
        if version == "svd":
            return (SVDpow(K, -0.5, rcond) @ zeta).contiguous()
        elif version == "ridge":
            return torch.linalg.solve(torch.linalg.cholesky(
                K + alpha * torch.eye(K.shape[0], **spec)), zeta).contiguous()
        raise ValueError("Unknown version")

    # ------------------------------------------------------------------------------------
    def Shoot(self, q0, p0, x0=None, need_p1=True):
        """Geodesic shooting from (q0, p0[, x0]); returns the list of (q, p, cost[, x])
        at the nt+1 times (LDDMM.py:286-299).  need_p1=False (extension, used by Optimize's
        loss closures): the final momenta may be left unformed (NaN; `shoot.p1_missing`) --
        the loss never reads them, and the last step then skips the momentum update's sums."""
        getspec(q0, p0, x0)
        if self.try_trajcost_optim and self.withlogdet and self.gradcomponent and x0 is None:
            # rarely used reference variant: generic integrator over the per-step ODE
            cost0 = torch.zeros(1, dtype=q0.dtype, device=q0.device)
            return self.Integrator(self.ODE, (q0, p0, cost0), self.nt)
        q0c = q0.contiguous()
        raw = self._raw_for(q0)
        outs = ShootFn.apply(q0c, p0.contiguous(),
                             None if x0 is None else x0.contiguous(), self.Kernel.sigma,
                             float(self.eta), int(self.nt), self.scheme, bool(self.withlogdet),
                             self.row_split, getattr(self, "row_orders", None),
                             getattr(self, "shoot_cache", None), bool(need_p1), raw)
        if x0 is None:
            Q, P, C, H0 = outs
            sh = Shoot(Q, P, C, None, H0)
        else:
            sh = Shoot(*outs)
        sh.p1_missing = skip_p1(need_p1, self.scheme, x0 is not None, float(self.eta),
                                self._split(), int(self.nt))
        if sh.p1_missing:
            # what complete_shoot needs to form P[nt] exactly as this shooting would have: the
            # coordinate mode its kernels ran in and the support tensor its row order is keyed on
            sh.raw, sh.q0_key = raw, q0c
        return sh

    def _split(self):
        return self.row_split if (self.row_split is not None and self.row_split.world > 1) else None

    def complete_shoot(self, shoot):
        """Form the final momenta of a shoot made with need_p1=False (no-op otherwise)."""
        if getattr(shoot, "p1_missing", False):
            # the row visit order (fwd_alg 3 with row_orders, keyed on the shooting's own q0
            # tensor, not a view of the trajectory) and the coordinate mode (raw beyond
            # RAW_EXTENT_SIGMA) the shooting itself used, so the completed P[nt] is bitwise the
            # one a full shooting would have produced
            split = self._split()
            key = getattr(shoot, "q0_key", None)
            raw = getattr(shoot, "raw", None)
            if key is None:
                key = shoot.Q[0]
            if raw is None:
                raw = self._raw_for(key)
            order, order_l = row_order_for(getattr(self, "row_orders", None), key,
                                           float(self.eta), split, shoot.Q.shape[1])
            with _lib.coord_mode(raw):
                complete_p1(shoot.Q, shoot.P, self.Kernel.sigma, float(self.eta),
                            bool(self.withlogdet), int(self.nt),
                            order=order_l if split is not None else order, split=split,
                            C=shoot.C)
            shoot.p1_missing = False
            shoot.q0_key = None
        return shoot

    def BasicQuadLossFunctor(self, y, cmul=1):
        y = y.detach()

        def dataloss(x):
            return ((x - y) ** 2).sum() * cmul / 2
        return dataloss

    def trajloss(self, shoot):
        """lambda*H(q0,p0) + cost_1  (LDDMM.py:318-334)."""
        arrival = shoot[-1]
        cost = arrival[2]
        is_x = len(arrival) == 4
        if not is_x and self.withlogdet and self.gradcomponent and self.try_trajcost_optim:
            return cost
        q0, p0 = shoot[0][:2]
        H0 = getattr(shoot, "H0", None)
        if H0 is None:
            H0 = self.Hamiltonian(q0, p0)
        return self.lam * H0 + cost

    # Coordinates of the fused shooting kernels (library option coord_raw).  "scaled": q' =
    # alpha (q - q_0), one packed multiply per two pairs fewer, float32-exact differences only
    # while the support spans up to ~200 sigma (2.8e-6 at 100 sigma, 1.3e-5 at 300 sigma
    # against float64, profiles/r03_extent_precision.jsonl); "raw": original units, the
    # reference's accuracy at any extent; "auto" (default): raw when q0 spans more than
    # RAW_EXTENT_SIGMA sigma (one small device read per new q0 tensor, per host thread).
    coord_mode = "auto"
    RAW_EXTENT_SIGMA = 128.0

    def _raw_for(self, q0):
        mode = self.coord_mode
        if mode == "raw":
            return True
        if mode != "auto" or q0.numel() == 0 or q0.device.type != "cuda":
            return False
        last = getattr(_EXTENT_MEMO, "last", None)
        if (last is not None and last[0]() is q0 and last[1] == q0._version
                and last[2] == float(self.Kernel.sigma)):
            return last[3] > self.RAW_EXTENT_SIGMA
        ext = float((q0.amax(0) - q0.amin(0)).norm()) / float(self.Kernel.sigma)
        _EXTENT_MEMO.last = (weakref.ref(q0), q0._version, float(self.Kernel.sigma), ext)
        return ext > self.RAW_EXTENT_SIGMA

    def Optimize(self, dataloss, q0, p0, x0=None, nmax=10, tol=1e-3, errthresh=1e8):
        """min_p0 trajloss + dataloss(q1 or x1) with L-BFGS (LDDMM.py:338-398).
        Returns (p0, shoot, trajl, datal, nsteps, change)."""
        getspec(q0, p0, x0)
        is_x = x0 is not None
        q0 = q0.detach()
        if is_x:
            x0 = x0.detach()

        last_eval = {}

        def lossfunc(p0):
            shoot = self.Shoot(q0, p0, x0, need_p1=False)   # the loss never reads p1
            last = shoot[-1][-1] if is_x else shoot[-1][0]
            last_eval["p0"], last_eval["shoot"] = p0.detach().clone(), shoot.detach()
            last_eval["p1_missing"] = getattr(shoot, "p1_missing", False)
            return self.trajloss(shoot) + dataloss(last)

        lossgrad = None
        batcher = getattr(_lib._tl, "batcher", None)
        # the closure forms loss and gradient directly (shooting.shoot_loss_grad: ShootFn's
        # forward and exact adjoint on THIS thread, bitwise the values of
        # lossfunc(p0).backward()) for a frame of a lockstep launch batch (core/batching.py),
        # whose adjoint must run on the frame's thread, and for every dense Euler shooting on
        # the device whose loss is lam H0 + cost + data: no autograd engine (its device-thread
        # hand-off and graph bookkeeping, ~0.1 ms of host time per closure -- the host floor,
        # tools/host_floor.py), and concurrent frames' adjoints no longer queue on the
        # engine's one device thread
        direct = (_DIRECT_LOSSGRAD and not is_x and self.scheme == "Euler" and self.row_split is None
                  and not (self.withlogdet and self.gradcomponent and self.try_trajcost_optim)
                  and q0.is_cuda)
        if (batcher is not None and not is_x) or direct:
            from .shooting import shoot_loss_grad

            def lossgrad(p0):
                if batcher is None:
                    L, g, shoot = shoot_loss_grad(self, dataloss, q0, p0)
                else:
                    with batcher.closure():   # a member of the launch batches while it evaluates
                        L, g, shoot = shoot_loss_grad(self, dataloss, q0, p0)
                last_eval["p0"], last_eval["shoot"] = p0.detach().clone(), shoot
                last_eval["p1_missing"] = getattr(shoot, "p1_missing", False)
                return L, [g]
        p0, _, nsteps, change = LBFGS_optimization([p0], lossfunc, nmax=nmax, tol=tol,
                                                   errthresh=errthresh, lossgrad=lossgrad)
        p0 = p0[0]
        with torch.no_grad():
            # final shoot (LDDMM.py:390): the kernels are deterministic, so when L-BFGS's
            # last closure evaluation was at the returned p0 its trajectory is reused
            if "p0" in last_eval and torch.equal(last_eval["p0"], p0):
                shoot = last_eval["shoot"]
                shoot.p1_missing = last_eval["p1_missing"]
                self.complete_shoot(shoot)              # the returned shoot is complete
            else:
                shoot = self.Shoot(q0, p0, x0)
            trajl = self.trajloss(shoot).item()
            datal = dataloss(shoot[-1][-1] if is_x else shoot[-1][0]).item()
        return p0, shoot, trajl, datal, nsteps, change
