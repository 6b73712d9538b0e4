"""Fused geodesic shooting and its discrete adjoint on gfx950.

The reference integrates the Hamiltonian ODE with generic Euler / Ralston loops
(diffICP/tools/integrators.py:20-51) over `LDDMMModel.ODE` (LDDMM.py:176-227), which calls
3-7 separate KeOps reductions per step, and differentiates the whole trajectory with torch
autograd + KeOps autodiff (optim.py:46).

Here one ODE evaluation is ONE fused HIP pass over the M x M support pairs
(dicp_lddmm_ode_self_fwd_f32; + one M x N pass for external points), and the trajectory is
a single autograd node whose backward runs the exact discrete adjoint of the same
integrator with one fused VJP pass per ODE evaluation (dicp_lddmm_ode_self_bwd_f32).
The result is the same gradient autograd would produce through the reference's
integrator (up to fp32 rounding); the trajectory (nt+1 states) stays resident in HBM.
"""
from __future__ import annotations

import contextlib
import os
import threading
import weakref
from collections import OrderedDict

import torch

from .. import _lib


def spatial_order(x: torch.Tensor) -> torch.Tensor:
    """Morton (Z-order) visit order of the rows of x (N, D), as an int32 permutation on x's
    device: rows that are close in space get close positions, so the workgroups of the
    matrix-core forward (csrc/mfma_fwd.hpp) hold compact groups of rows and the fp32 error of
    its centred channel split stays at the ordered-pair kernels' level whatever the cloud's
    extent.  10 (3D) / 16 (2D) bits per coordinate over the bounding box; a stable sort, so
    the order (hence every result) is deterministic."""
    N, D = x.shape
    bits = 10 if D == 3 else 16
    xd = x.detach()
    lo = xd.amin(0)
    ext = (xd.amax(0) - lo).clamp_min(1e-30)
    c = ((xd - lo) * ((2 ** bits - 1) / ext)).to(torch.int64).clamp_(0, 2 ** bits - 1)
    if D == 3:   # spread 10 bits to every third bit
        c = (c | (c << 16)) & 0x030000FF
        c = (c | (c << 8)) & 0x0300F00F
        c = (c | (c << 4)) & 0x030C30C3
        c = (c | (c << 2)) & 0x09249249
    else:        # spread 16 bits to every second bit
        c = (c | (c << 8)) & 0x00FF00FF
        c = (c | (c << 4)) & 0x0F0F0F0F
        c = (c | (c << 2)) & 0x33333333
        c = (c | (c << 1)) & 0x55555555
    code = (c << torch.arange(D, device=x.device, dtype=torch.int64)).sum(1)   # disjoint bits
    return torch.argsort(code, stable=True).to(torch.int32)


class RowOrderCache:
    """spatial_order of the support points, memoised per tensor (q0 is fixed over an L-BFGS
    run: every closure reuses the order).  Keyed on (storage pointer, version counter, shape,
    slice); each entry holds a strong reference to the keyed tensor, so its storage cannot be
    freed and handed to another tensor while the entry lives (no stale hit by address reuse).
    Least-recently-used eviction beyond `maxsize` entries."""

    def __init__(self, maxsize=32):
        self._d = OrderedDict()
        self._lock = threading.Lock()
        self.maxsize = maxsize

    # a cache: copies and pickles start empty
    def __getstate__(self):
        return {"maxsize": self.maxsize}

    def __setstate__(self, state):
        self.__init__(state.get("maxsize", 32))

    def __deepcopy__(self, memo):
        return RowOrderCache(self.maxsize)

    def __len__(self):
        return len(self._d)

    def get(self, x: torch.Tensor, row0: int = 0, n: int = None):
        n = x.shape[0] - row0 if n is None else n
        key = (x.data_ptr(), x._version, tuple(x.shape), str(x.device), row0, n)
        with self._lock:
            e = self._d.get(key)
            if e is not None:
                self._d.move_to_end(key)
        if e is None:
            o = spatial_order(x[row0:row0 + n])
            with self._lock:
                self._d[key] = (x, o)
                while len(self._d) > self.maxsize:
                    self._d.popitem(last=False)
            return o
        return e[1]


# rows per workgroup of the matrix-core forward: at or below it the order cannot matter
_ORDER_MIN_ROWS = 256


def row_order_for(orders, q0, eta, split, M):
    """The row visit order(s) a shooting of q0 uses: (order of all rows, order of this rank's
    row slice), either None (no order cache, eta != 0, or too few rows to matter)."""
    order = order_l = None
    if orders is not None and eta == 0:
        if split is not None:
            r0_, n_, _ = split.rows(M)
            if n_ > _ORDER_MIN_ROWS:
                order_l = orders.get(q0, r0_, n_)
        elif M > _ORDER_MIN_ROWS:
            order = orders.get(q0)
    return order, order_l


def _nbytes(ts):
    seen, n = set(), 0
    for t in ts:
        if isinstance(t, torch.Tensor):
            k = (t.untyped_storage().data_ptr(), t.device)
            if k not in seen:
                seen.add(k)
                n += t.untyped_storage().nbytes()
    return n


class ShootCache:
    """Recent forward trajectories keyed by the support-point tensor q0, reused when the same
    shooting (q0, p0[, x0] and the same model parameters) is asked for again.

    Why: DiffPSR.Reg_opt starts every L-BFGS run at the momenta the previous run returned
    (PSR.py:521-569 passes a0[k]); its first closure shoots exactly the trajectory the
    previous run's final shoot computed -- only the data loss changed (new GMM targets), and
    the trajectory does not depend on it.  The kernels are deterministic (no atomics, fixed
    summation order), so a hit returns bitwise the tensors a recomputation would produce;
    the backward runs the adjoint on them as usual.

    Safety: the key is (storage pointer, version counter, shape, device) of q0, and each
    entry holds a strong reference to that q0, so its storage cannot be freed and reused by a
    different tensor while the entry lives; before reuse q0, p0 and x0 are compared bitwise
    (torch.equal) with the cache's own copies of the inputs.  The cache never shares storage
    with tensors handed to callers (ShootFn returns clones on hits AND misses).  Bounded:
    least-recently-used eviction beyond `max_entries` entries or `max_bytes` of device memory
    (one entry per frame is what the Reg_opt reuse needs)."""

    def __init__(self, max_entries=64, max_bytes=8 << 30):
        self._d = OrderedDict()
        self._lock = threading.Lock()
        self.max_entries = max_entries
        self.max_bytes = max_bytes
        self._bytes = 0
        self.hits = 0
        self.misses = 0

    def __getstate__(self):
        return {"max_entries": self.max_entries, "max_bytes": self.max_bytes}

    def __setstate__(self, state):
        self.__init__(state.get("max_entries", 64), state.get("max_bytes", 8 << 30))

    def __deepcopy__(self, memo):
        return ShootCache(self.max_entries, self.max_bytes)

    def __len__(self):
        return len(self._d)

    @property
    def nbytes(self):
        return self._bytes

    @staticmethod
    def _key(q0):
        return (q0.data_ptr(), q0._version, tuple(q0.shape), str(q0.device))

    def lookup(self, q0, p0, x0, params):
        key = self._key(q0)
        with self._lock:
            e = self._d.get(key)
            if e is not None:
                self._d.move_to_end(key)
        # p0 first: it is what differs between the closures of one L-BFGS run (each
        # torch.equal is a device round trip).  The L-BFGS parameter is updated in place, so
        # the same tensor at a newer version is a miss without comparing.  Same tensor OBJECT
        # (weak reference), not just the same address: a new tensor that the allocator put at
        # the old one's address starts a version count of its own, and taking it for an
        # in-place update would make hits depend on allocation order (a false miss -- a
        # recomputation -- never a stale hit, but not a reproducible one)
        if (e is not None and e["p0src"][0]() is p0 and p0.data_ptr() == e["p0src"][1]
                and p0._version != e["p0src"][2]):
            self.misses += 1
            return None
        if (e is None or e["params"] != params or (e["x0"] is None) != (x0 is None)
                or not torch.equal(e["p0"], p0)
                or (x0 is not None and not torch.equal(e["x0"], x0))
                or not torch.equal(e["q0c"], q0)):
            self.misses += 1
            return None
        self.hits += 1
        # the cached tensors may have been produced on another stream (concurrent frames: a
        # new stream per Reg_opt call); keep their memory from being reused while this stream
        # still reads them
        if p0.is_cuda:
            st = torch.cuda.current_stream(p0.device)
            for t in list(e["saved"]) + [t for t in e["outs"] if isinstance(t, torch.Tensor)]:
                t.record_stream(st)
        return e

    def store(self, q0, p0, x0, params, outs, saved):
        e = {"q0": q0, "q0c": outs[0][0], "p0": p0.detach().clone(), "p0src": (weakref.ref(p0), p0.data_ptr(), p0._version),
             "x0": None if x0 is None else x0.detach().clone(),
             "params": params, "outs": outs, "saved": saved}
        e["nbytes"] = _nbytes(list(outs) + list(saved) + [e["p0"], e["x0"]])
        key = self._key(q0)
        with self._lock:
            old = self._d.pop(key, None)
            if old is not None:
                self._bytes -= old["nbytes"]
            self._d[key] = e
            self._bytes += e["nbytes"]
            while len(self._d) > 1 and (len(self._d) > self.max_entries or self._bytes > self.max_bytes):
                _, ev = self._d.popitem(last=False)
                self._bytes -= ev["nbytes"]

    def clear(self):
        with self._lock:
            self._d.clear()
            self._bytes = 0


def _h_rows(p, v):
    """Rows of the Hamiltonian at eta = 0, h_i = p_i.v_i / 2 (LDDMM.py:150-155), from the
    forward's v (when its h slot carried the divergence rows)."""
    return 0.5 * (p * v).sum(1)


def _f_self(q, p, sigma, eta, want_div, want_h=False, order=None):
    """ODE right-hand side at the support points: (v, mG, div[1]) [+ per-row h]."""
    v, mG, g, h = _lib.ode_self_fwd(q, p, sigma, eta, want_div, want_h=want_h, order=order)
    div = g.sum().reshape(1) if want_div else None
    return (v, mG, div, h) if want_h else (v, mG, div)


def _f_ext(q, p, x, sigma, eta, want_div, want_h=False, order=None):
    """ODE with external points: (vq, mGq, div over x [1], vx) [+ per-row h]."""
    v, mG, _, h = _lib.ode_self_fwd(q, p, sigma, eta, False, want_h=want_h, order=order)
    vx, gx = _lib.ode_ext_fwd(x, q, p, sigma, eta, want_div)
    div = gx.sum().reshape(1) if want_div else None
    return (v, mG, div, vx, h) if want_h else (v, mG, div, vx)


def _vjp(q, p, x, lq, lp, lc, lx, sigma, eta, want_div):
    """Vector-Jacobian product of the ODE right-hand side at (q, p[, x]) for cotangents
    (lq on v, lp on mG, lc on div, lx on vx).  Returns (gq, gp, gx)."""
    if x is None:
        gq, gp = _lib.ode_self_bwd(q, p, lq, lp, lc if want_div else None, sigma, eta)
        return gq, gp, None
    gq, gp = _lib.ode_self_bwd(q, p, lq, lp, None, sigma, eta)
    gx = _lib.ode_ext_bwd(x, q, p, lx, lc if want_div else None, sigma, eta, gq, gp)
    return gq, gp, gx


def skip_p1(need_p1, scheme, has_x, eta, split, nt):
    """Whether ShootFn leaves the final momenta P[nt] unformed: only on request, and only on
    the paths whose last step is a fused Euler step (no external points, nt >= 2; single
    device or row split).  `eta` is accepted for the callers' symmetry: both models have the
    mG-less pass."""
    return (not need_p1) and scheme == "Euler" and not has_x and nt >= 2


def phased_split(split, M, order=None):
    """Whether a row-split shooting runs its fused steps t >= 1 in column phases
    (split_step_phased): W | M (the direct path), RowSplit.overlap, natural row order."""
    return (split is not None and split.world > 1 and M % split.world == 0
            and getattr(split, "overlap", False) and order is None)


def split_step_phased(split, Qt, Pt, q_loc, p_loc, sigma, eta, dt, want_div, q_out, p_out=None,
                      zs_out=None, before_remote=None):
    """This rank's rows of the Euler step from (Qt, Pt) in two column phases
    (dicp_lddmm_euler_step_phase_f32): the rows against their own slice (q_loc, p_loc: the
    rows' values, which the rank holds before the all-gather of the step's input has landed),
    then before_remote() (wait for that all-gather, unpack into Qt, Pt), then against the other
    points and one merge.  Every step of a phased shooting and its completion (complete_p1) go
    through here, so a step's bits do not depend on which of the two formed it.  Returns the
    slice's divergence rows g (or None)."""
    M, D = Qt.shape
    r0, n, _ = split.rows(M)
    want_g = bool(want_div) or eta != 0
    g_out = torch.empty(n, device=Qt.device, dtype=Qt.dtype) if want_g else None
    ws = _lib.euler_step_phase_ws(n, M, D, Qt.device)
    outs = (q_out, p_out, g_out, zs_out)
    _lib.euler_step_phase(0, q_loc, p_loc, Qt, Pt, r0, n, sigma, eta, dt, *outs, ws=ws)
    if before_remote is not None:
        before_remote()
    _lib.euler_step_phase(1, q_loc, p_loc, Qt, Pt, r0, n, sigma, eta, dt, *outs, ws=ws)
    return g_out


def last_cost_step(C, Gd, nt, dt):
    """C[nt] = C[nt-1] + dt sum_i g_i(nt-1) of a fused Euler shooting: the last step's
    increment as its own reduction (of row nt-1 of the (nt, M) divergence rows Gd), so a
    completion (complete_p1) that re-runs the last step forms it with the same bits."""
    inc = Gd[nt - 1:nt].sum(1, keepdim=True).mul_(dt)
    torch.add(C[nt - 1], inc[0], out=C[nt])


def complete_p1(Q, P, sigma, eta, want_div, nt, order=None, split=None, C=None):
    """Form P[nt] of a trajectory shot with need_p1=False: the last Euler step again, by the
    same fused pass a full shooting uses (bitwise the P[nt] it would have produced; row split:
    each rank's slice, one all-gather).  Single device: Q[nt] and (with C) the cost C[nt] are
    rewritten from that pass too -- the mG-less pass of the need_p1=False step may run another
    kernel (the ordered rows where a full pass takes the symmetric 4-row forward, other column
    splits), so the completed trajectory is bitwise a fresh full shooting's."""
    with torch.no_grad():
        if split is not None:
            M = Q.shape[1]
            r0, n, _ = split.rows(M)
            if phased_split(split, M, order):   # the phased shooting's own step
                D = Q.shape[2]
                pn_l = torch.empty((n, D), device=Q.device, dtype=Q.dtype)
                split_step_phased(split, Q[nt - 1], P[nt - 1], Q[nt - 1][r0:r0 + n],
                                  P[nt - 1][r0:r0 + n], sigma, eta, 1.0 / nt, want_div,
                                  torch.empty_like(pn_l), pn_l)
                split.gather_into(P[nt], pn_l)
                return
            _, pn_l, _ = _lib.euler_step_rows(Q[nt - 1], P[nt - 1], r0, n, sigma, eta, 1.0 / nt,
                                              want_div, order=order)
            (pn,), _ = split.gather_rows([pn_l], M)
            P[nt].copy_(pn)
            return
        M, D = Q.shape[1], Q.shape[2]
        # the full step exactly as ShootFn's fused loop issues it: divergence rows into row
        # nt-1 of an (nt, M) buffer (same alignment as the forward's Gd), zs rows when the
        # forward keeps them (the zs variant is another kernel)
        use_zs = bool(want_div) and nt >= 2 and _lib.zs_ok(eta)
        Gd = torch.empty((nt, M), device=Q.device, dtype=Q.dtype) if want_div else None
        zs = torch.empty((M, D), device=Q.device, dtype=Q.dtype) if use_zs else None
        _lib.euler_step(Q[nt - 1], P[nt - 1], sigma, eta, 1.0 / nt, want_div, q_out=Q[nt],
                        p_out=P[nt], g_out=Gd[nt - 1] if want_div else None, order=order,
                        zs_out=zs)
        if C is not None and want_div:
            last_cost_step(C, Gd, nt, 1.0 / nt)


class ShootFn(torch.autograd.Function):
    """(q0, p0[, x0]) -> stacked trajectory Q, P (nt+1, M, D), C (nt+1, 1)[, X (nt+1, N, D)],
    H0 = H(q0, p0).

    scheme: "Euler" (x += dt f(x)) or "Ralston" (k1 = f(x), k2 = f(x + 2dt/3 k1),
    x += dt/4 (k1 + 3 k2)), as integrators.py:20-51.  The Hamiltonian at the start point,
    which trajloss needs (LDDMM.py:318-334), comes for free from the first ODE evaluation
    (same fused pass, one extra per-row store): dH0/dp0 = v(q0, p0), dH0/dq0 = -mG(q0, p0).
    """

    @staticmethod
    def forward(ctx, q0, p0, x0, sigma, eta, nt, scheme, want_div, split=None, orders=None,
                cache=None, need_p1=True, raw=False):
        """orders: optional RowOrderCache; the forward passes then visit the support rows in
        the spatial order of q0 (kept for every step: the flow moves neighbours together).
        cache: optional ShootCache (bitwise reuse of a repeated shooting, see there).
        need_p1=False: the final momenta P[nt] are not formed when skip_p1(...) holds (the last
        fused Euler step skips its Gs' sums) and P[nt] is filled with NaN; the caller must not
        read it (LDDMMModel.Optimize's closures do not) or complete it (complete_p1).
        raw: the packed shooting kernels in original-unit coordinates (library option
        coord_raw, per host thread: set here around the forward's launches and again in the
        backward, which autograd may run on another thread)."""
        ctx.raw = bool(raw)
        # the per-thread geometry hint (batch_share) of the forward applies to the backward
        # too, which autograd may run on another thread
        ctx.share = _lib.get_option("batch_share")
        with _lib.coord_mode(ctx.raw):
            return ShootFn._forward(ctx, q0, p0, x0, sigma, eta, nt, scheme, want_div, split, orders,
                                    cache, need_p1)

    @staticmethod
    def _forward(ctx, q0, p0, x0, sigma, eta, nt, scheme, want_div, split, orders, cache, need_p1):
        ctx.set_materialize_grads(False)   # unused outputs (cost, H0, ...) get None, not zeros
        has_x = x0 is not None
        skip = skip_p1(need_p1, scheme, has_x, eta, split, nt)
        # divergence rows (dicp_lddmm_*_zs_f32): the fused Euler steps t >= 1 keep the forward's
        # per-row sums zs = sum_j K z, which their adjoint steps reuse for the divergence
        # cotangent's dL/dp term instead of re-summing it pair by pair (saved, nt x M x D floats)
        use_zs = bool(want_div) and scheme == "Euler" and not has_x and nt >= 2 and _lib.zs_ok(eta)
        ctx.has_zs = use_zs
        # option_epoch: a set_option of a kernel variant between two shootings is a miss (the
        # cached trajectory would not be bitwise what the new variant computes)
        params = (float(sigma), float(eta), int(nt), scheme, bool(want_div),
                  None if split is None else (split.rank, split.world, getattr(split, "overlap", False)),
                  skip, use_zs, ctx.raw,
                  _lib.option_epoch(), _lib.get_option("batch_share"))
        hit = cache.lookup(q0, p0, x0, params) if cache is not None else None
        if hit is not None:
            ctx.split = split if (split is not None and not has_x and scheme == "Euler"
                                  and split.world > 1) else None
            ctx.sigma, ctx.eta, ctx.nt, ctx.scheme, ctx.want_div, ctx.has_x = \
                sigma, eta, nt, scheme, want_div, has_x
            ctx.save_for_backward(*hit["saved"])
            # fresh output tensors (autograd owns them); the saved ones are only read
            return _fresh(hit["outs"])
        # row-split over ranks (core/rowsplit.py): dense Euler shooting only; other schemes
        # run replicated on every rank
        if split is not None and (has_x or scheme != "Euler" or split.world == 1):
            split = None
        ctx.split = split
        if split is None and not has_x and scheme == "Euler" and _graph_eligible(q0, nt):
            # small supports: the whole fused shooting replayed as one captured HIP graph
            order, _ = row_order_for(orders, q0, eta, None, q0.shape[0])
            r = _graph_forward(ctx, q0, p0, order, sigma, eta, nt, want_div, need_p1, params)
            if r is not None:
                outs, saved = r
                ctx.sigma, ctx.eta, ctx.nt, ctx.scheme, ctx.want_div, ctx.has_x = \
                    sigma, eta, nt, scheme, want_div, has_x
                ctx.save_for_backward(*saved)
                if cache is not None:
                    kept = tuple(t.detach() for t in outs)
                    cache.store(q0, p0, x0, params, kept, [t.detach() for t in saved])
                    return _fresh(kept)
                return outs
        M, D = q0.shape
        dev = q0.device
        dt = 1.0 / nt
        Q = torch.empty((nt + 1, M, D), device=dev, dtype=q0.dtype)
        P = torch.empty_like(Q)
        C = torch.zeros((nt + 1, 1), device=dev, dtype=q0.dtype)
        X = torch.empty((nt + 1,) + tuple(x0.shape), device=dev, dtype=q0.dtype) if has_x else None
        Q[0].copy_(q0)
        P[0].copy_(p0)
        if has_x:
            X[0].copy_(x0)
        mids = []  # Ralston intermediate states (needed by the adjoint)
        H0 = v0 = mG0 = None
        order, order_l = row_order_for(orders, q0, eta, split, M)
        Gd, fused_from = None, None  # fused Euler steps: per-step divergence rows, first step
        Zs = None
        if use_zs:
            zrows = split.rows(M)[1] if split is not None else M
            Zs = torch.empty((nt, zrows, D), device=dev, dtype=q0.dtype)
        # row split with W | M: the fused steps write this rank's rows into send buffers and
        # the all-gathers land straight in Q[t+1] / P[t+1]; the divergence partials are kept
        # per step and exchanged once after the loop (rank-ordered, as the staged path)
        direct = split is not None and M % split.world == 0
        if direct:
            # the step writes this rank's new q and p rows side by side, ONE all-gather moves
            # both (W x (2, n_l, D), rank order) and two copies unpack them into Q[t+1], P[t+1]
            # -- one collective per forward step instead of two (latency-bound at large W)
            n_l = M // split.world
            qp_l = torch.empty((2, n_l, D), device=dev, dtype=q0.dtype)
            qs_l, ps_l = qp_l[0], qp_l[1]
            qp_all = torch.empty((split.world, 2, n_l, D), device=dev, dtype=q0.dtype)
            dloc = torch.zeros(nt, device=dev, dtype=q0.dtype)
        # column phases (split_step_phased): the all-gather of step t's rows stays in flight
        # while step t+1 runs the rank's rows against its own slice; `pend` = that gather
        phased = direct and phased_split(split, M, order_l)
        pend = None

        def land(t_in):
            # the all-gather of the rows of Q[t_in], P[t_in] has landed: unpack (rank order)
            nonlocal pend
            if pend is not None:
                pend.wait()
                pend = None
                Q[t_in].view(split.world, n_l, D).copy_(qp_all[:, 0])
                P[t_in].view(split.world, n_l, D).copy_(qp_all[:, 1])

        # per-step views formed once (unbind: one op, against ~6 indexing selects per step --
        # host floor, tools/host_floor.py); the views write into Q, P, Gd, Zs
        Qv, Pv = Q.unbind(0), P.unbind(0)
        Zv = None if Zs is None else Zs.unbind(0)
        Gv = None
        for t in range(nt):
            q, p = Qv[t], Pv[t]
            x = X[t] if has_x else None
            first = t == 0
            if phased and not first:
                r0, n, _ = split.rows(M)
                last_skip = skip and t == nt - 1
                # the rank's own rows of (Q[t], P[t]): the send buffer until the gather lands
                q_loc, p_loc = (qs_l, ps_l) if pend is not None else (q[r0:r0 + n], p[r0:r0 + n])
                g_l = split_step_phased(split, q, p, q_loc, p_loc, sigma, eta, dt, want_div, qs_l,
                                        None if last_skip else ps_l,
                                        None if Zs is None else Zs[t],
                                        before_remote=lambda t=t: land(t))
                if last_skip:
                    split.gather_into(Q[t + 1], qs_l)
                    P[t + 1].fill_(float("nan"))   # not formed: make any read loud
                else:
                    pend = split.gather_into_async(qp_all, qp_l)
                if g_l is not None:
                    torch.sum(g_l, 0, keepdim=True, out=dloc[t:t + 1])
                continue
            if split is not None and direct and not first:
                r0, n, _ = split.rows(M)
                last_skip = skip and t == nt - 1
                _, _, g_l = _lib.euler_step_rows(q, p, r0, n, sigma, eta, dt, want_div, q_out=qs_l,
                                                 p_out=None if last_skip else ps_l, order=order_l,
                                                 want_p=not last_skip,
                                                 zs_out=None if Zs is None else Zs[t])
                if last_skip:
                    split.gather_into(Q[t + 1], qs_l)
                    P[t + 1].fill_(float("nan"))   # not formed: make any read loud
                else:
                    split.gather_into(qp_all, qp_l)
                    Q[t + 1].view(split.world, n_l, D).copy_(qp_all[:, 0])
                    P[t + 1].view(split.world, n_l, D).copy_(qp_all[:, 1])
                if g_l is not None:
                    torch.sum(g_l, 0, keepdim=True, out=dloc[t:t + 1])
                continue
            if split is not None:
                r0, n, _ = split.rows(M)
                if first:
                    if Zs is not None:   # zs in h's slot: H's rows as p.v / 2 (the kernel's h)
                        v_l, mG_l, g_l, _ = _lib.ode_self_fwd_rows(q, p, r0, n, sigma, eta, want_div,
                                                                   order=order_l, zs_out=Zs[0])
                        h_l = _h_rows(p[r0:r0 + n], v_l)
                    else:
                        v_l, mG_l, g_l, h_l = _lib.ode_self_fwd_rows(q, p, r0, n, sigma, eta, want_div,
                                                                     want_h=True, order=order_l)
                    loc = torch.stack([h_l.sum(), g_l.sum() if g_l is not None else h_l.sum() * 0])
                    (v0, mG0), _ = split.gather_rows([v_l, mG_l], M)
                    sums = split.sum_ordered(loc)   # (H0, div): rank-ordered, same bits everywhere
                    H0 = sums[0]
                    torch.add(q, v0, alpha=dt, out=Q[t + 1])
                    torch.add(p, mG0, alpha=dt, out=P[t + 1])
                    div = sums[1:2]
                elif skip and t == nt - 1:
                    # final momenta not wanted: mG-less pass, half the all-gather
                    qn_l, _, g_l = _lib.euler_step_rows(q, p, r0, n, sigma, eta, dt, want_div,
                                                        order=order_l, want_p=False,
                                                        zs_out=None if Zs is None else Zs[t])
                    gs = g_l.sum().reshape(1) if g_l is not None else None
                    (qn,), div = split.gather_rows([qn_l], M, scalar=gs)
                    Q[t + 1].copy_(qn)
                    P[t + 1].fill_(float("nan"))   # not formed: make any read loud
                else:
                    qn_l, pn_l, g_l = _lib.euler_step_rows(q, p, r0, n, sigma, eta, dt, want_div,
                                                           order=order_l,
                                                           zs_out=None if Zs is None else Zs[t])
                    gs = g_l.sum().reshape(1) if g_l is not None else None
                    (qn, pn), div = split.gather_rows([qn_l, pn_l], M, scalar=gs)
                    Q[t + 1].copy_(qn)
                    P[t + 1].copy_(pn)
                if want_div:
                    torch.add(C[t], div, alpha=dt, out=C[t + 1])
                else:
                    C[t + 1].copy_(C[t])
                continue
            if scheme == "Euler" and not has_x and not first:
                # fused pass: Q[t+1], P[t+1] written by the reduction's epilogue; the per-row
                # divergence terms go to Gd[t] and the cost is accumulated once after the loop
                if Gd is None:
                    Gd = torch.empty((nt, M), device=dev, dtype=q0.dtype) if want_div else False
                    Gv = Gd.unbind(0) if want_div else None
                last_skip = skip and t == nt - 1
                _lib.euler_step(q, p, sigma, eta, dt, want_div, q_out=Qv[t + 1], p_out=Pv[t + 1],
                                g_out=Gv[t] if want_div else None, order=order, want_p=not last_skip,
                                zs_out=None if Zv is None else Zv[t])
                if last_skip:
                    Pv[t + 1].fill_(float("nan"))   # not formed: make any read loud
                fused_from = t if fused_from is None else fused_from
                continue
            if has_x:
                out = _f_ext(q, p, x, sigma, eta, want_div, want_h=first, order=order)
                v, mG, div, vx = out[:4]
            elif first and Zs is not None:
                v, mG, g, _ = _lib.ode_self_fwd(q, p, sigma, eta, want_div, order=order, zs_out=Zs[0])
                div = g.sum().reshape(1)
                out = (v, mG, div, _h_rows(p, v))
                vx = None
            else:
                out = _f_self(q, p, sigma, eta, want_div, want_h=first, order=order)
                v, mG, div = out[:3]
                vx = None
            if first:
                H0, v0, mG0 = out[-1].sum(), v, mG
            if scheme == "Euler":
                torch.add(q, v, alpha=dt, out=Q[t + 1])
                torch.add(p, mG, alpha=dt, out=P[t + 1])
                if want_div:
                    torch.add(C[t], div, alpha=dt, out=C[t + 1])
                else:
                    C[t + 1].copy_(C[t])
                if has_x:
                    torch.add(x, vx, alpha=dt, out=X[t + 1])
            else:  # Ralston
                a = 2.0 * dt / 3.0
                qi = torch.add(q, v, alpha=a)
                pi = torch.add(p, mG, alpha=a)
                xi = torch.add(x, vx, alpha=a) if has_x else None
                if has_x:
                    v2, mG2, div2, vx2 = _f_ext(qi, pi, xi, sigma, eta, want_div, order=order)
                else:
                    v2, mG2, div2 = _f_self(qi, pi, sigma, eta, want_div, order=order)
                    vx2 = None
                Q[t + 1].copy_(q + (0.25 * dt) * (v + 3.0 * v2))
                P[t + 1].copy_(p + (0.25 * dt) * (mG + 3.0 * mG2))
                if want_div:
                    C[t + 1].copy_(C[t] + (0.25 * dt) * (div + 3.0 * div2))
                else:
                    C[t + 1].copy_(C[t])
                if has_x:
                    X[t + 1].copy_(x + (0.25 * dt) * (vx + 3.0 * vx2))
                mids.append((qi, pi, xi))
        if phased:
            land(nt)
        if direct and nt > 1:
            # cost of the steps t >= 1: their divergence partials summed in rank order (one
            # all-gather), then C[t+1] = C[t] + dt div_t as the staged path
            if want_div:
                divs = split.sum_ordered(dloc[1:])
                for t in range(1, nt):
                    torch.add(C[t], divs[t - 1:t], alpha=dt, out=C[t + 1])
            else:
                C[2:].copy_(C[1].expand(nt - 1, 1))
        if fused_from is not None:
            # cost of the fused steps: C[t+1] = C[t] + dt sum_i g_i(t), one reduction + scan
            # over the steps before the last, the last step's increment on its own
            # (last_cost_step: complete_p1 re-forms it from the full pass bit for bit)
            if want_div:
                if fused_from < nt - 1:
                    inc = Gd[fused_from:nt - 1].sum(1, keepdim=True).mul_(dt)
                    torch.cumsum(inc, 0, out=C[fused_from + 1:nt])
                    C[fused_from + 1:nt].add_(C[fused_from])
                last_cost_step(C, Gd, nt, dt)
            else:
                C[fused_from + 1:].copy_(C[fused_from].expand(nt - fused_from, 1))
        ctx.sigma, ctx.eta, ctx.nt, ctx.scheme, ctx.want_div, ctx.has_x = \
            sigma, eta, nt, scheme, want_div, has_x
        if H0 is None:  # nt == 0
            v0, mG0, _, h = _lib.ode_self_fwd(q0, p0, sigma, eta, False, want_h=True)
            H0 = h.sum()
        saved = [Q, P, v0, mG0] + ([X] if has_x else [])
        for (qi, pi, xi) in mids:
            saved += [qi, pi] + ([xi] if has_x else [])
        if Zs is not None:
            saved.append(Zs)   # last (ctx.has_zs)
        ctx.save_for_backward(*saved)
        outs = (Q, P, C, X, H0) if has_x else (Q, P, C, H0)
        if cache is not None:
            H0d = H0 if isinstance(H0, torch.Tensor) else torch.as_tensor(H0)
            kept = tuple(t.detach() for t in ((Q, P, C, X, H0d) if has_x else (Q, P, C, H0d)))
            cache.store(q0, p0, x0, params, kept, [t.detach() for t in saved])
            # the cache keeps Q, P, ... (and autograd saved them): the caller gets its own
            # copies, so an in-place write by the caller (complete_shoot) cannot reach them
            return _fresh(kept)
        return outs

    @staticmethod
    def backward(ctx, gQ, gP, gC, *rest):
        with _lib.coord_mode(ctx.raw), _lib.thread_option(getattr(ctx, "share", 1), "batch_share"):
            return ShootFn._backward(ctx, gQ, gP, gC, *rest)

    @staticmethod
    def _backward(ctx, gQ, gP, gC, *rest):
        gX, gH = rest if len(rest) == 2 else (None, rest[0])
        sigma, eta, nt, scheme, want_div, has_x = \
            ctx.sigma, ctx.eta, ctx.nt, ctx.scheme, ctx.want_div, ctx.has_x
        split = ctx.split
        saved = ctx.saved_tensors
        Zs = saved[-1] if ctx.has_zs else None
        if Zs is not None and not _lib.zs_ok(eta):
            Zs = None   # the VJP variant changed since the forward: re-sum the divergence terms
        Q, P, v0, mG0 = saved[:4]
        X = saved[4] if has_x else None
        k = 5 if has_x else 4
        mids = []
        if scheme != "Euler":
            step = 3 if has_x else 2
            for t in range(nt):
                e = saved[k + step * t: k + step * (t + 1)]
                mids.append((e[0], e[1], e[2] if has_x else None))
        dt = 1.0 / nt
        M, D = Q.shape[1], Q.shape[2]
        dev = Q.device
        if split is None and scheme == "Euler" and not has_x and _graph_eligible(Q[0], nt):
            r = _graph_backward(ctx, gQ, gP, gC, gH, saved, Zs)
            if r is not None:
                return r

        def g_or_zero(G, t, shape):
            if G is None:
                return torch.zeros(shape, device=dev, dtype=Q.dtype)
            return G[t]

        lq = g_or_zero(gQ, nt, (M, D)).clone()
        # no cotangent on the final momenta (the usual loss: trajloss + data term on q1 / x1):
        # lp stays None for the first fused adjoint step, whose VJP then skips the b terms
        fused = split is None and scheme == "Euler" and not has_x
        lp = gP[nt].clone() if gP is not None else (
            None if (fused or split is not None) else torch.zeros((M, D), device=dev, dtype=Q.dtype))
        lc = g_or_zero(gC, nt, (1,)).clone()
        lx = g_or_zero(gX, nt, tuple(X.shape[1:])).clone() if has_x else None

        lc_suffix = None
        Qv, Pv = Q.unbind(0), P.unbind(0)    # per-step views formed once (as the forward)
        Zv = None if Zs is None else Zs.unbind(0)
        gQv = None if gQ is None else gQ.unbind(0)
        gPv = None if gP is None else gP.unbind(0)
        lcv = None
        for t in range(nt - 1, -1, -1):
            q, p = Qv[t], Pv[t]
            x = X[t] if has_x else None
            if split is not None:
                # this rank's part of the pair-once VJP, summed over ranks (one all-reduce);
                # the last step needs gp only when q0 needs no gradient (half the bytes too)
                want_lq = t > 0 or ctx.needs_input_grad[0]
                zs_t = None if Zs is None else Zs[t]
                g2 = torch.empty((2, M, D), device=dev, dtype=Q.dtype) if want_lq else None
                gq_l, gp_l = _lib.ode_self_bwd_part(q, p, lq, lp, lc if want_div else None, sigma,
                                                    eta, split.rank, split.world, want_gq=want_lq,
                                                    zs=zs_t, zrow0=split.rows(M)[0],
                                                    gq_out=None if g2 is None else g2[0],
                                                    gp_out=None if g2 is None else g2[1])
                if want_lq:
                    g = split.all_reduce_(g2)   # (gq, gp) parts written side by side: no cat
                    lq = torch.add(lq, g[0], alpha=dt)
                    lp = g[1].mul(dt) if lp is None else torch.add(lp, g[1], alpha=dt)
                else:
                    gp_r = split.all_reduce_(gp_l)
                    lp = gp_r.mul_(dt) if lp is None else torch.add(lp, gp_r, alpha=dt)
                    lq = None
                if gQ is not None and lq is not None:
                    lq = lq + gQ[t]
                if gP is not None:
                    lp = lp + gP[t]
                if gC is not None:
                    lc = lc + gC[t]
                continue
            if scheme == "Euler" and not has_x:
                # fused pass: lambda_t = lambda_{t+1} + dt VJP + the loss's own cotangent at t;
                # the cost cotangent at t is the suffix sum of gC (precomputed, no per-step op)
                if gC is not None and lc_suffix is None:
                    lc_suffix = torch.flip(torch.cumsum(torch.flip(gC, (0,)), 0), (0,))
                    lcv = lc_suffix.unbind(0)
                lct = lc if gC is None else lcv[t + 1]
                # last step: the cotangent of q0 is only needed if q0 requires a gradient (the
                # support points of Reg_opt do not) -- then the gq half is skipped
                want_lq = t > 0 or ctx.needs_input_grad[0]
                lq, lp = _lib.euler_adjoint_step(q, p, lq, lp, lct if want_div else None, sigma, eta,
                                                 dt, None if gQv is None else gQv[t],
                                                 None if gPv is None else gPv[t], want_lq=want_lq,
                                                 zs=None if Zv is None else Zv[t])
                if gC is not None:
                    lc = lcv[t]
                continue
            if scheme == "Euler":
                gq, gp, gx = _vjp(q, p, x, lq, lp, lc, lx, sigma, eta, want_div)
                lq = torch.add(lq, gq, alpha=dt)
                lp = torch.add(lp, gp, alpha=dt)
                if has_x:
                    lx = torch.add(lx, gx, alpha=dt)
            else:
                qi, pi, xi = mids[t]
                # k2 = f(s_i) with cotangent 3dt/4 * lambda'
                gqi, gpi, gxi = _vjp(qi, pi, xi, lq, lp, lc, lx, sigma, eta, want_div)
                c2 = 0.75 * dt
                lqi, lpi = c2 * gqi, c2 * gpi
                lxi = c2 * gxi if has_x else None
                # k1 = f(s) with cotangent dt/4 * lambda' + 2dt/3 * lambda_i (cost: dt/4 lc)
                a = 2.0 * dt / 3.0
                kq = 0.25 * dt * lq + a * lqi
                kp = 0.25 * dt * lp + a * lpi
                kc = 0.25 * dt * lc
                kx = (0.25 * dt * lx + a * lxi) if has_x else None
                gq1, gp1, gx1 = _vjp(q, p, x, kq, kp, kc, kx, sigma, eta, want_div)
                lq = lq + lqi + gq1
                lp = lp + lpi + gp1
                if has_x:
                    lx = lx + lxi + gx1
            if gQ is not None:
                lq = lq + gQ[t]
            if gP is not None:
                lp = lp + gP[t]
            if gC is not None:
                lc = lc + gC[t]
            if has_x and gX is not None:
                lx = lx + gX[t]
        if gH is not None:
            if lq is not None:
                lq = lq - gH * mG0
            lp = lp + gH * v0
        if not ctx.needs_input_grad[0]:
            lq = None
        return lq, lp, (lx if has_x else None), None, None, None, None, None, None, None, None, None, None


class ManualCtx:
    """Stand-in for the autograd context when ShootFn's forward and backward are called
    directly on the calling host thread (shoot_loss_grad) -- what autograd would do, minus
    the engine's device thread, on which every frame's backward would otherwise run in turn."""

    def __init__(self, needs_input_grad):
        self.needs_input_grad = tuple(needs_input_grad)
        self._saved = ()

    def set_materialize_grads(self, value):
        pass

    def save_for_backward(self, *ts):
        self._saved = ts

    @property
    def saved_tensors(self):
        return self._saved


# ---- HIP-graph replay of the fused Euler shooting and its adjoint (small supports) ---------
# At a few thousand support points every pass of a shooting is a ~10-20 us kernel and the
# host's per-call work (wrapper checks, views, ctypes) is most of a closure (tools/host_floor.py:
# the strong-scaling floor).  There the fused Euler forward (nt passes,
# the cost scan) and its adjoint (nt VJP passes) are captured once per configuration -- the
# very same launches, with their workspaces in the graph's private pool -- and replayed: copy
# the inputs into the graph's static tensors, one replay, copy the outputs out (fresh tensors,
# as the direct path returns).  Bitwise the direct path (same kernels, same order: only the
# host's way of issuing them changes; tests/test_gpu_shoot_graph.py).  Keyed per host thread
# and stream (autograd runs the adjoint on its device thread), captured at a key's second
# use (a one-off stream, e.g. a concurrent frame's, is never captured), LRU-bounded.  Off for
# row splits, external points, Ralston, launch batches, the bench's per-launch accounting,
# and DICP_SHOOT_GRAPH=0.
_GRAPH_ON = os.environ.get("DICP_SHOOT_GRAPH", "1") != "0"
_GRAPH_MAX_M = 32768
_GRAPH_MAX = 8
_graphs = OrderedDict()
_graph_seen = OrderedDict()
_graph_lock = threading.Lock()
_graph_tl = threading.local()
graph_stats = {"captures": 0, "replays": 0}


# host threads driving GPU work concurrently (PSR's concurrent frames, the lockstep batches):
# a capture must not begin while another thread issues work to the device (hipStreamBeginCapture
# fails with hipErrorIllegalState, measured in the 4-rank atlas rehearsal), so those sections
# switch the graphs off for their duration
_graph_block = [0]


@contextlib.contextmanager
def graphs_blocked():
    """No HIP-graph capture or replay of shootings while this is active (any thread)."""
    with _graph_lock:
        _graph_block[0] += 1
    try:
        yield
    finally:
        with _graph_lock:
            _graph_block[0] -= 1


def _graph_eligible(q0, nt):
    return (_GRAPH_ON and _graph_block[0] == 0 and nt >= 2 and q0.is_cuda and q0.shape[0] <= _GRAPH_MAX_M
            and not getattr(_graph_tl, "inside", False) and _lib._prof is None
            and getattr(_lib._tl, "batcher", None) is None
            and getattr(_lib._tl, "batch_keep", None) is None
            and not torch.cuda.is_current_stream_capturing())


class _FixedOrder:
    """RowOrderCache stand-in inside a capture: the order computed outside it."""

    def __init__(self, order):
        self.order = order

    def get(self, x, row0=0, n=None):
        return self.order


class _CaptureFailed(Exception):
    pass


_graph_failed = []


def _graph_entry(key, capture):
    """The captured graph of `key`, capturing it at the key's second use (None before)."""
    with _graph_lock:
        ent = _graphs.get(key)
        if ent is not None:
            _graphs.move_to_end(key)
            return ent
        n = _graph_seen.get(key, 0) + 1
        _graph_seen[key] = n
        while len(_graph_seen) > 4 * _GRAPH_MAX:
            _graph_seen.popitem(last=False)
    if n < 2:
        return None
    try:
        ent = capture()
    except _CaptureFailed:
        return None
    with _graph_lock:
        graph_stats["captures"] += 1
        _graphs[key] = ent
        while len(_graphs) > _GRAPH_MAX:
            _graphs.popitem(last=False)
    return ent


def _capture(run, dev):
    """(graph, run's outputs): run() once on a side stream (first-call host queries, lazy
    state), then captured; the tensors run() allocates live in the graph's private pool."""
    _graph_tl.inside = True
    try:
        cur = torch.cuda.current_stream(dev)
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            run()
        cur.wait_stream(side)
        g = torch.cuda.CUDAGraph()
        try:
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                out = run()
        except Exception:
            # a capture that could not begin or complete: the direct path from now on in this
            # process; the graph object is kept (torch's destructor of a half-registered graph
            # aborts the process)
            global _GRAPH_ON
            _GRAPH_ON = False
            _graph_failed.append(g)
            raise _CaptureFailed()
        return g, out
    finally:
        _graph_tl.inside = False


def _copy_many(dsts, srcs):
    """dst.copy_(src) for every pair, as one multi-tensor launch where torch can (same device
    and dtype, dense): the graph replays' input and output copies were ~18 separate buffer
    copies per L-BFGS closure, a tenth of the 2k-point iteration's kernels
    (tools/host_floor_timeline.py).  Copies are exact, so results are bitwise unchanged."""
    if not dsts:
        return
    if len(dsts) == 1:
        dsts[0].copy_(srcs[0])
        return
    torch._foreach_copy_(list(dsts), list(srcs))


def _fresh(ts):
    """tuple(t.clone() for t in ts), the copies in one launch (_copy_many)."""
    out = tuple(torch.empty_like(t) for t in ts)
    _copy_many(out, ts)
    return out


def _clone_all(ts):
    """Fresh copies of a list of tensors (None kept), each distinct tensor copied once."""
    memo = {}
    out, dsts, srcs = [], [], []
    for t in ts:
        if t is None:
            out.append(None)
            continue
        c = memo.get(id(t))
        if c is None:
            c = memo[id(t)] = torch.empty_like(t)
            dsts.append(c)
            srcs.append(t)
        out.append(c)
    _copy_many(dsts, srcs)
    return out


def _graph_forward(ctx, q0, p0, order, sigma, eta, nt, want_div, need_p1, params):
    dev = q0.device
    key = ("fwd", threading.get_ident(), _lib._stream(dev), dev.index, tuple(q0.shape), q0.dtype,
           params, bool(need_p1), None if order is None else (order.data_ptr(), order._version))

    def capture():
        sq0, sp0 = q0.detach().clone(), p0.detach().clone()
        fixed = None if order is None else _FixedOrder(order)

        def run():
            ictx = ManualCtx((False, True) + (False,) * 11)
            ictx.raw, ictx.share = ctx.raw, ctx.share
            outs = ShootFn._forward(ictx, sq0, sp0, None, sigma, eta, nt, "Euler", want_div, None,
                                    fixed, None, need_p1)
            return outs, ictx.saved_tensors, ictx.has_zs
        g, (outs, saved, has_zs) = _capture(run, dev)
        return {"g": g, "in": (sq0, sp0), "outs": outs, "saved": saved, "has_zs": has_zs,
                "order": order}

    ent = _graph_entry(key, capture)
    if ent is None:
        return None
    sq0, sp0 = ent["in"]
    _copy_many([sq0, sp0], [q0, p0])
    ent["g"].replay()
    graph_stats["replays"] += 1
    n_out = len(ent["outs"])
    fresh = _clone_all(list(ent["outs"]) + list(ent["saved"]))
    ctx.has_zs = ent["has_zs"]
    return tuple(fresh[:n_out]), fresh[n_out:]


def _graph_backward(ctx, gQ, gP, gC, gH, saved, Zs):
    dev = saved[0].device
    ins = list(saved[:4]) + [Zs, gQ, gP, gC, gH]
    key = ("bwd", threading.get_ident(), _lib._stream(dev), dev.index,
           tuple(None if t is None else (tuple(t.shape), t.dtype) for t in ins),
           float(ctx.sigma), float(ctx.eta), int(ctx.nt), bool(ctx.want_div),
           tuple(ctx.needs_input_grad[:1]), bool(getattr(ctx, "raw", False)), int(getattr(ctx, "share", 1)),
           _lib.option_epoch())

    def capture():
        st = [None if t is None else t.detach().clone() for t in ins]

        def run():
            ictx = ManualCtx(ctx.needs_input_grad)
            ictx.save_for_backward(*([t for t in st[:4]] + ([st[4]] if st[4] is not None else [])))
            ictx.sigma, ictx.eta, ictx.nt, ictx.scheme, ictx.want_div, ictx.has_x = \
                ctx.sigma, ctx.eta, ctx.nt, "Euler", ctx.want_div, False
            ictx.split, ictx.has_zs = None, st[4] is not None
            ictx.raw, ictx.share = getattr(ctx, "raw", False), getattr(ctx, "share", 1)
            return ShootFn._backward(ictx, st[5], st[6], st[7], st[8])
        g, out = _capture(run, dev)
        return {"g": g, "in": st, "out": out}

    ent = _graph_entry(key, capture)
    if ent is None:
        return None
    pairs = [(s_, t) for s_, t in zip(ent["in"], ins) if t is not None]
    _copy_many([s_ for s_, _ in pairs], [t for _, t in pairs])
    ent["g"].replay()
    graph_stats["replays"] += 1
    out = ent["out"]
    lq, lp = _clone_all([out[0], out[1]])
    return (lq, lp) + tuple(out[2:])


def shoot_loss_grad(LM, dataloss, q0, p0):
    """Optimize's loss at p0 -- trajloss + dataloss(q1) of a need_p1=False Euler shooting
    (LDDMM.py:318-334, optim.py:41-47) -- and its gradient w.r.t. p0, with ShootFn's forward and
    exact adjoint run on THIS thread instead of through autograd (whose CUDA backward runs on
    the engine's device thread): the lockstep frame batches (core/batching.py) need every
    frame's adjoint launches on the frame's own thread.  The cotangents handed to the adjoint
    are exactly those autograd would hand it -- zeros but for dL/dq1 in gQ[nt], 1 in gC[nt], lam
    for H0, none for P -- so loss and gradient are bitwise those of lossfunc(p0).backward().
    Dense support, Euler, no row split.  Returns (loss (1,), grad_p0, shoot)."""
    from .LDDMM import Shoot
    nt = int(LM.nt)
    ctx = ManualCtx((False, True, False) + (False,) * 10)
    raw = LM._raw_for(q0)
    outs = ShootFn.forward(ctx, q0.contiguous(), p0.detach().contiguous(), None, LM.Kernel.sigma,
                           float(LM.eta), nt, LM.scheme, bool(LM.withlogdet), None,
                           getattr(LM, "row_orders", None), getattr(LM, "shoot_cache", None), False, raw)
    Q, P, C, H0 = outs
    sh = Shoot(Q, P, C, None, H0)
    sh.p1_missing = skip_p1(False, LM.scheme, False, float(LM.eta), None, nt)
    if sh.p1_missing:
        sh.raw, sh.q0_key = raw, q0.contiguous()
    vg = getattr(dataloss, "value_and_grad", None)
    r = vg(Q[nt]) if (vg is not None and isinstance(LM.lam, (int, float))) else None
    if r is not None:
        # a data loss that forms its own gradient (PSR's quadratic loss): the cotangents
        # autograd would hand the adjoint, without its engine (~0.1 ms of host time per
        # closure at 2k points, the host floor): 1 on C[nt], lam on H0 (MulBackward's
        # grad * lam), dL/dq1 in gQ[nt]
        dl, gq1 = r
        L = LM.lam * H0 + C[nt] + dl
        gQ = torch.zeros_like(Q)
        gQ[nt].copy_(gq1)
        gH = torch.full_like(H0, LM.lam)
        gC = torch.zeros_like(C)
        gC[nt] = 1.0
        with _lib.coord_mode(raw), _lib.thread_option(ctx.share, "batch_share"):
            grads = ShootFn._backward(ctx, gQ, None, gC, gH)
        return L, grads[1], sh
    with torch.enable_grad():
        q1 = Q[nt].detach().requires_grad_(True)
        H0r = H0.detach().requires_grad_(True)
        C1 = C.detach().requires_grad_(True)
        L = LM.lam * H0r + C1[nt] + dataloss(q1)
        # backward() rather than autograd.grad: the gradient also accumulates into any other
        # leaf the data loss reads (as the reference's L.backward(), optim.py:46, would), and a
        # data loss that does not depend on q1 (a frame without data points) gives no gq1
        L.backward(torch.ones_like(L))
    gq1, gH, gC = q1.grad, H0r.grad, C1.grad
    gQ = torch.zeros_like(Q)
    if gq1 is not None:
        gQ[nt].copy_(gq1)
    if gH is None:
        gH = torch.zeros_like(H0)
    if gC is None:
        gC = torch.zeros_like(C)
    with _lib.coord_mode(raw), _lib.thread_option(ctx.share, "batch_share"):
        grads = ShootFn._backward(ctx, gQ, None, gC, gH)
    return L.detach(), grads[1], sh


class HamiltonianFn(torch.autograd.Function):
    """H(q, p) = sum_i h_i from the fused forward pass (LDDMM.py:142-159).
    dH/dp = v (= KRed - eta GradKRed), dH/dq = G = -mG (the ODE's right-hand side)."""

    @staticmethod
    def forward(ctx, q, p, sigma, eta):
        v, mG, _, h = _lib.ode_self_fwd(q, p, sigma, eta, False, want_h=True)
        ctx.save_for_backward(v, mG)
        return h.sum()

    @staticmethod
    def backward(ctx, gH):
        v, mG = ctx.saved_tensors
        return -gH * mG, gH * v, None, None


class OdeFn(torch.autograd.Function):
    """One differentiable evaluation of LDDMMModel.ODE at the support points
    (returns v, -G, dcost) -- the per-step API used by LDDMMModel.ODE."""

    @staticmethod
    def forward(ctx, q, p, sigma, eta, want_div):
        v, mG, div = _f_self(q, p, sigma, eta, want_div)
        if div is None:
            div = torch.zeros(1, device=q.device, dtype=q.dtype)
        ctx.save_for_backward(q, p)
        ctx.sigma, ctx.eta, ctx.want_div = sigma, eta, want_div
        return v, mG, div

    @staticmethod
    def backward(ctx, gv, gmG, gdiv):
        q, p = ctx.saved_tensors
        gv = torch.zeros_like(q) if gv is None else gv
        gmG = torch.zeros_like(q) if gmG is None else gmG
        gq, gp, _ = _vjp(q, p, None, gv, gmG, gdiv, None, ctx.sigma, ctx.eta, ctx.want_div)
        return gq, gp, None, None, None


class OdeExtFn(torch.autograd.Function):
    """LDDMMModel.ODE with an external point set x: (vq, -Gq, dcost, vx)."""

    @staticmethod
    def forward(ctx, q, p, x, sigma, eta, want_div):
        v, mG, div, vx = _f_ext(q, p, x, sigma, eta, want_div)
        if div is None:
            div = torch.zeros(1, device=q.device, dtype=q.dtype)
        ctx.save_for_backward(q, p, x)
        ctx.sigma, ctx.eta, ctx.want_div = sigma, eta, want_div
        return v, mG, div, vx

    @staticmethod
    def backward(ctx, gv, gmG, gdiv, gvx):
        q, p, x = ctx.saved_tensors
        gv = torch.zeros_like(q) if gv is None else gv
        gmG = torch.zeros_like(q) if gmG is None else gmG
        gvx = torch.zeros_like(x) if gvx is None else gvx
        gq, gp, gx = _vjp(q, p, x, gv, gmG, gdiv, gvx, ctx.sigma, ctx.eta, ctx.want_div)
        return gq, gp, gx, None, None, None
