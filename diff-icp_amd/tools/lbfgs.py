"""L-BFGS with the inverse-Hessian product in compact form (device-friendly).

The reference optimises with torch.optim.LBFGS (diffICP/tools/optim.py:26, strong-Wolfe line
search, history 100, max_iter 20).  Its two-loop recursion costs ~5 tiny device kernels per
stored pair per iteration (dot, scalar mul, axpy, ...): with 10-20 stored pairs that is
~2000 launches per PSR iteration, more than the shooting itself, and they leave the GPU idle
between launches (profiles/r01_timeline_summary.json).

`CompactLBFGS` keeps torch's LBFGS.step control flow line for line (same memory update rule
`ys > 1e-10`, same initial step, same strong-Wolfe line search `torch.optim.lbfgs._strong_wolfe`,
same stopping tests) and replaces only the two-loop recursion by the algebraically identical
compact representation (Byrd, Nocedal & Schnabel 1994, eq. 2.6; H0 = gamma I):

    H v = gamma v + S t - gamma Y u,   u = R^{-1} (S^T v),
    t = R^{-T} ((D + gamma Y^T Y) u - gamma Y^T v)

with S, Y the (m, n) histories kept in preallocated device buffers, R = triu(S^T Y),
D = diag(S^T Y).  Per iteration: one stacked GEMV [S; Y] v on the device, the m x m products
S^T Y, Y^T Y (updated incrementally: two GEMVs per new pair) and the two triangular solves
(float64) on the host, one transfer of the GEMVs' 3m+2 values and one GEMV back.  Results equal torch's two-loop up to floating-point rounding.  The "GEMVs" are torch
elementwise products + reductions, not BLAS calls: rocBLAS allows atomics by default, and the
row-split multi-GPU mode needs bitwise-identical iterates on every rank.

Host round trips.  torch's step and `_strong_wolfe` keep the line-search scalars (gtd, the
step t after an interpolation, the gradient / step norms) as 0-d device tensors, so every
comparison is a device-to-host synchronisation -- ~9-10 per L-BFGS iteration, each leaving
the GPU idle while the host decides (profiles/r03_timeline_summary.json).  Here the same
control flow runs on host scalars: the values torch keeps as 0-d tensors are numpy scalars
of the parameters' dtype (numpy's weak-Python-scalar promotion, NEP 50, is torch's), the
loss values Python floats as in torch, so every decision and step length is bit-identical to
torch.optim.LBFGS's.  Each function evaluation reads (loss, g.d, max|g|) in ONE transfer, an
iteration adds one read of (y.s, y.y) and one of (g.d, max|d| [, sum|g|]) -- 3 round trips per
iteration.  The loss of every evaluation is passed to `on_loss(loss)` (if set) while the
parameters still hold the evaluated point (tools/optim.py tracks the best point with it).
"""
from __future__ import annotations

import math

import numpy as np
import torch

# the host-scalar line search reaches torch's decisions through NEP 50 promotion (a numpy
# float32 scalar combined with a Python float stays float32), which numpy 1.x does not do --
# checked when an optimizer is built (not at import: the rest of the package does not need it)
_NUMPY_NEP50 = int(np.__version__.split(".")[0]) >= 2


def _require_nep50():
    if not _NUMPY_NEP50:
        raise ImportError(f"CompactLBFGS needs numpy >= 2 (NEP 50 scalar promotion), found {np.__version__}")


def _rowdots(A, v):
    """A @ v as a deterministic elementwise product + row reduction, accumulated in float64
    (the m x m algebra is float64 already; an fp32 sum over n ~ 1e5-1e6 entries would make the
    fp32 trajectory depend on the reduction order)."""
    return (A * v[None, :]).sum(1, dtype=torch.float64)


def _absmax(v):
    """max|v| in one reduction launch (torch's abs().max() takes two); a maximum of magnitudes
    involves no rounding, so the value (NaN included) is bitwise the same."""
    return torch.linalg.vector_norm(v, ord=math.inf)


class CompactLBFGS(torch.optim.LBFGS):
    """Drop-in for torch.optim.LBFGS (same constructor and step semantics)."""

    def __init__(self, *args, **kwargs):
        _require_nep50()
        super().__init__(*args, **kwargs)

    # ------------------------------------------------------------------------------
    def _hist_init(self, n, like):
        h = self.param_groups[0]["history_size"]
        st = self.state[self._params[0]]
        st["S"] = torch.empty((h, n), device=like.device, dtype=like.dtype)
        st["Y"] = torch.empty((h, n), device=like.device, dtype=like.dtype)
        # the m x m algebra runs on the host (float64 CPU tensors): on the device it was ~20
        # launches per iteration (triangle, two rocBLAS triangular solves with their index
        # kernels, a dozen scalar ops, the slice writes) -- the largest share of the 2k-point
        # host floor after the shootings (tools/host_floor_timeline.py); on CPU parameters the
        # ops are the same torch CPU ops as before, bit for bit
        st["SY"] = torch.zeros((h, h), dtype=torch.float64)   # s_i . y_j
        st["YY"] = torch.zeros((h, h), dtype=torch.float64)   # y_i . y_j
        st["m"] = 0
        st["pend"] = None

    def _hist_push(self, s, y):
        st = self.state[self._params[0]]
        h = self.param_groups[0]["history_size"]
        S, Y = st["S"], st["Y"]
        m = st["m"]
        if m == h:  # drop the oldest pair (torch: old_dirs.pop(0))
            S[:-1] = S[1:].clone()
            Y[:-1] = Y[1:].clone()
            SY, YY = st["SY"], st["YY"]
            SY[:-1, :-1] = SY[1:, 1:].clone()
            YY[:-1, :-1] = YY[1:, 1:].clone()
            m -= 1
        torch._foreach_copy_([S[m], Y[m]], [s, y])    # one launch for both rows
        # new column of S^T Y / Y^T Y and new row s_m^T Y: two stacked GEMVs on the device,
        # read together with the next _hist_apply's GEMV (one transfer)
        a = _rowdots(torch.cat([S[:m + 1], Y[:m + 1]], 0), y)    # [S^T y; Y^T y]
        b = _rowdots(Y[:m + 1], s)                                 # y_j . s_m
        st["pend"] = (m, a, b)
        st["m"] = m + 1

    def _hist_commit(self, pend, a, b):
        st = self.state[self._params[0]]
        m = pend
        SY, YY = st["SY"], st["YY"]
        SY[:m + 1, m] = a[:m + 1]
        SY[m, :m + 1] = b
        YY[:m + 1, m] = a[m + 1:]
        YY[m, :m + 1] = a[m + 1:]

    def _hist_apply(self, v, gamma):
        """H v (compact form)."""
        st = self.state[self._params[0]]
        m = st["m"]
        pend, st["pend"] = st["pend"], None
        if m == 0:
            return v * gamma
        S, Y = st["S"][:m], st["Y"][:m]
        SY_ = torch.cat([S, Y], 0)
        ab = _rowdots(SY_, v)
        if pend is not None:
            pm, pa, pb = pend
            n_a, n_b = pa.numel(), pb.numel()
            host = torch.cat([pa, pb, ab]).cpu()      # one transfer (a no-op on CPU)
            self._hist_commit(pm, host[:n_a], host[n_a:n_a + n_b])
            ab = host[n_a + n_b:]
        else:
            ab = ab.cpu()
        SY, YY = st["SY"][:m, :m], st["YY"][:m, :m]
        a, b = ab[:m], ab[m:]
        g = gamma if isinstance(gamma, float) else gamma.double()
        R = torch.triu(SY)
        u = torch.linalg.solve_triangular(R, a[:, None], upper=True)[:, 0]
        w = torch.diagonal(SY) * u + g * _rowdots(YY, u) - g * b
        t = torch.linalg.solve_triangular(R.t(), w[:, None], upper=False)[:, 0]
        coef = torch.cat([t, -g * u]).to(dtype=v.dtype).to(v.device)
        return v * gamma + (SY_ * coef[:, None]).sum(0)

    # ------------------------------------------------------------------------------
    on_loss = None   # callback(loss: float) after every function evaluation

    def _read(self, *ts):
        """Device scalars -> host floats in one transfer (float64: exact for either dtype; scalars
        of one dtype are stacked as they are -- the float32 -> Python float conversion is exact
        too -- which saves a conversion launch per scalar)."""
        ts = [t.detach().reshape(()) for t in ts]
        if any(t.dtype != ts[0].dtype for t in ts):
            ts = [t if t.dtype == torch.float64 else t.to(torch.float64) for t in ts]
        return torch.stack(ts).tolist()

    def _dt(self, *vals):
        """Host stand-ins of torch's 0-d tensors: numpy scalars of the parameters' dtype."""
        dt = np.float32 if self._params[0].dtype == torch.float32 else np.float64
        return [dt(v) for v in vals]

    def _evaluate(self, closure, d=None):
        """One function evaluation at the current parameters: (loss, flat_grad, g.d, max|g|);
        g.d is None without d."""
        L = closure()
        flat_grad = self._gather_flat_grad()
        if d is None:
            loss, gmax = self._read(L, _absmax(flat_grad))
            gtd = None
            (gmax,) = self._dt(gmax)
        else:
            loss, gtd, gmax = self._read(L, flat_grad.dot(d), _absmax(flat_grad))
            gtd, gmax = self._dt(gtd, gmax)
        if self.on_loss is not None:
            self.on_loss(loss)
        return loss, flat_grad, gtd, gmax

    def _directional_eval(self, closure, x, t, d):
        self._add_grad(float(t), d)
        out = self._evaluate(closure, d)
        self._set_param(x)
        return out

    @staticmethod
    def _cubic_interpolate(x1, f1, g1, x2, f2, g2, bounds=None):
        """torch.optim.lbfgs._cubic_interpolate on host scalars: the same expression, with
        numpy scalars where torch has 0-d tensors (and Python floats where it has them)."""
        if bounds is not None:
            xmin_bound, xmax_bound = bounds
        else:
            xmin_bound, xmax_bound = (x1, x2) if x1 <= x2 else (x2, x1)
        with np.errstate(all="ignore"):
            d1 = g1 + g2 - 3 * (f1 - f2) / (x1 - x2)
            d2_square = d1 ** 2 - g1 * g2
            if d2_square >= 0:
                d2 = np.sqrt(d2_square)
                if x1 <= x2:
                    min_pos = x2 - (x2 - x1) * ((g2 + d2 - d1) / (g2 - g1 + 2 * d2))
                else:
                    min_pos = x1 - (x1 - x2) * ((g1 + d2 - d1) / (g1 - g2 + 2 * d2))
                return min(max(min_pos, xmin_bound), xmax_bound)
            return (xmin_bound + xmax_bound) / 2.0

    def _strong_wolfe(self, closure, x, t, d, f, g, gtd, gmax, d_norm, c1=1e-4, c2=0.9,
                      tolerance_change=1e-9, max_ls=25):
        """torch.optim.lbfgs._strong_wolfe (same bracketing / zoom control flow) on host
        scalars; returns (f, g, t, evaluations, max|g|) of the accepted point."""
        interp = self._cubic_interpolate
        g = g.clone(memory_format=torch.contiguous_format)
        f_new, g_new, gtd_new, gmax_new = self._directional_eval(closure, x, t, d)
        ls_func_evals = 1
        t_prev, f_prev, g_prev, gtd_prev, gmax_prev = 0, f, g, gtd, gmax
        done = False
        ls_iter = 0
        while ls_iter < max_ls:
            if f_new > (f + c1 * t * gtd) or (ls_iter > 1 and f_new >= f_prev):
                bracket, bracket_f = [t_prev, t], [f_prev, f_new]
                bracket_g = [g_prev, g_new.clone(memory_format=torch.contiguous_format)]
                bracket_gtd, bracket_gmax = [gtd_prev, gtd_new], [gmax_prev, gmax_new]
                break
            if abs(gtd_new) <= -c2 * gtd:
                bracket, bracket_f, bracket_g, bracket_gmax = [t], [f_new], [g_new], [gmax_new]
                done = True
                break
            if gtd_new >= 0:
                bracket, bracket_f = [t_prev, t], [f_prev, f_new]
                bracket_g = [g_prev, g_new.clone(memory_format=torch.contiguous_format)]
                bracket_gtd, bracket_gmax = [gtd_prev, gtd_new], [gmax_prev, gmax_new]
                break
            min_step = t + 0.01 * (t - t_prev)
            max_step = t * 10
            tmp = t
            t = interp(t_prev, f_prev, gtd_prev, t, f_new, gtd_new, bounds=(min_step, max_step))
            t_prev, f_prev, gtd_prev, gmax_prev = tmp, f_new, gtd_new, gmax_new
            g_prev = g_new.clone(memory_format=torch.contiguous_format)
            f_new, g_new, gtd_new, gmax_new = self._directional_eval(closure, x, t, d)
            ls_func_evals += 1
            ls_iter += 1
        if ls_iter == max_ls:
            bracket, bracket_f, bracket_g, bracket_gmax = [0, t], [f, f_new], [g, g_new], [gmax, gmax_new]
        insuf_progress = False
        low_pos, high_pos = (0, 1) if bracket_f[0] <= bracket_f[-1] else (1, 0)
        while not done and ls_iter < max_ls:
            if abs(bracket[1] - bracket[0]) * d_norm < tolerance_change:
                break
            t = interp(bracket[0], bracket_f[0], bracket_gtd[0], bracket[1], bracket_f[1], bracket_gtd[1])
            eps = 0.1 * (max(bracket) - min(bracket))
            if min(max(bracket) - t, t - min(bracket)) < eps:
                if insuf_progress or t >= max(bracket) or t <= min(bracket):
                    t = max(bracket) - eps if abs(t - max(bracket)) < abs(t - min(bracket)) else min(bracket) + eps
                    insuf_progress = False
                else:
                    insuf_progress = True
            else:
                insuf_progress = False
            f_new, g_new, gtd_new, gmax_new = self._directional_eval(closure, x, t, d)
            ls_func_evals += 1
            ls_iter += 1
            if f_new > (f + c1 * t * gtd) or f_new >= bracket_f[low_pos]:
                bracket[high_pos], bracket_f[high_pos] = t, f_new
                bracket_g[high_pos] = g_new.clone(memory_format=torch.contiguous_format)
                bracket_gtd[high_pos], bracket_gmax[high_pos] = gtd_new, gmax_new
                low_pos, high_pos = (0, 1) if bracket_f[0] <= bracket_f[1] else (1, 0)
            else:
                if abs(gtd_new) <= -c2 * gtd:
                    done = True
                elif gtd_new * (bracket[high_pos] - bracket[low_pos]) >= 0:
                    bracket[high_pos], bracket_f[high_pos] = bracket[low_pos], bracket_f[low_pos]
                    bracket_g[high_pos], bracket_gtd[high_pos] = bracket_g[low_pos], bracket_gtd[low_pos]
                    bracket_gmax[high_pos] = bracket_gmax[low_pos]
                bracket[low_pos], bracket_f[low_pos] = t, f_new
                bracket_g[low_pos] = g_new.clone(memory_format=torch.contiguous_format)
                bracket_gtd[low_pos], bracket_gmax[low_pos] = gtd_new, gmax_new
        return (bracket_f[low_pos], bracket_g[low_pos], bracket[low_pos], ls_func_evals,
                bracket_gmax[low_pos])

    @torch.no_grad()
    def step(self, closure):  # noqa: C901 -- mirrors torch.optim.LBFGS.step
        if len(self.param_groups) != 1:
            raise AssertionError("Expected exactly one param_group")
        closure = torch.enable_grad()(closure)
        group = self.param_groups[0]
        lr = float(group["lr"])
        max_iter = group["max_iter"]
        max_eval = group["max_eval"]
        tolerance_grad = group["tolerance_grad"]
        tolerance_change = group["tolerance_change"]
        line_search_fn = group["line_search_fn"]
        if line_search_fn not in (None, "strong_wolfe"):
            raise RuntimeError("only 'strong_wolfe' is supported")

        state = self.state[self._params[0]]
        state.setdefault("func_evals", 0)
        state.setdefault("n_iter", 0)

        loss, flat_grad, _, gmax = self._evaluate(closure)
        orig_loss = loss
        current_evals = 1
        state["func_evals"] += 1
        if gmax <= tolerance_grad:
            return orig_loss

        d = state.get("d")
        t = state.get("t")
        H_diag = state.get("H_diag")
        prev_flat_grad = state.get("prev_flat_grad")
        prev_loss = state.get("prev_loss")

        n_iter = 0
        while n_iter < max_iter:
            n_iter += 1
            state["n_iter"] += 1

            if state["n_iter"] == 1:
                d = flat_grad.neg()
                self._hist_init(flat_grad.numel(), flat_grad)
                H_diag = 1
            else:
                y = flat_grad.sub(prev_flat_grad)
                s = d.mul(t)
                ys, yy = self._dt(*self._read(y.dot(s), y.dot(y)))
                if ys > 1e-10:
                    self._hist_push(s, y)
                    H_diag = ys / yy
                d = self._hist_apply(flat_grad.neg(), H_diag if isinstance(H_diag, int) else float(H_diag))

            if prev_flat_grad is None:
                prev_flat_grad = flat_grad.clone(memory_format=torch.contiguous_format)
            else:
                prev_flat_grad.copy_(flat_grad)
            prev_loss = loss

            first = state["n_iter"] == 1
            if first:
                gtd, d_norm, gsum = self._dt(*self._read(flat_grad.dot(d), _absmax(d),
                                                         flat_grad.abs().sum()))
                t = min(1.0, 1.0 / gsum) * lr
            else:
                gtd, d_norm = self._dt(*self._read(flat_grad.dot(d), _absmax(d)))
                t = lr
            if gtd > -tolerance_change:
                break

            ls_func_evals = 0
            if line_search_fn is not None:
                x_init = self._clone_param()
                loss, flat_grad, t, ls_func_evals, gmax = self._strong_wolfe(
                    closure, x_init, t, d, loss, flat_grad, gtd, gmax, d_norm, max_ls=max_eval - current_evals)
                self._add_grad(float(t), d)
                opt_cond = gmax <= tolerance_grad
            else:
                self._add_grad(float(t), d)
                opt_cond = False
                if n_iter != max_iter:
                    loss, flat_grad, _, gmax = self._evaluate(closure)
                    opt_cond = gmax <= tolerance_grad
                    ls_func_evals = 1

            current_evals += ls_func_evals
            state["func_evals"] += ls_func_evals

            if n_iter == max_iter:
                break
            if current_evals >= max_eval:
                break
            if opt_cond:
                break
            # max|t d| = |t| max|d| in the parameters' dtype (rounding is monotone)
            if abs(self._dt(t)[0]) * d_norm <= tolerance_change:
                break
            if abs(loss - prev_loss) < tolerance_change:
                break

        state["d"] = d
        state["t"] = t
        state["H_diag"] = H_diag
        state["prev_flat_grad"] = prev_flat_grad
        state["prev_loss"] = prev_loss
        return orig_loss
