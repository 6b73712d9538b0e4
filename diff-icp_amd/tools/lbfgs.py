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
D = diag(S^T Y).  Per iteration: one stacked GEMV [S; Y] v, two m x m triangular solves
(float64) and one GEMV back; the m x m products are updated incrementally (two GEMVs per new
pair).  Results equal torch's two-loop up to floating-point rounding.  The "GEMVs" are torch
elementwise products + reductions, not BLAS calls: rocBLAS allows atomics by default, and the
row-split multi-GPU mode needs bitwise-identical iterates on every rank.
"""
from __future__ import annotations

import torch
from torch.optim.lbfgs import _strong_wolfe


def _rowdots(A, v):
    """A @ v as a deterministic elementwise product + row reduction, accumulated in float64
    (the m x m algebra is float64 already; an fp32 sum over n ~ 1e5-1e6 entries would make the
    fp32 trajectory depend on the reduction order)."""
    return (A * v[None, :]).sum(1, dtype=torch.float64)


class CompactLBFGS(torch.optim.LBFGS):
    """Drop-in for torch.optim.LBFGS (same constructor and step semantics)."""

    # ------------------------------------------------------------------------------
    def _hist_init(self, n, like):
        h = self.param_groups[0]["history_size"]
        st = self.state[self._params[0]]
        st["S"] = torch.empty((h, n), device=like.device, dtype=like.dtype)
        st["Y"] = torch.empty((h, n), device=like.device, dtype=like.dtype)
        st["SY"] = torch.zeros((h, h), device=like.device, dtype=torch.float64)  # s_i . y_j
        st["YY"] = torch.zeros((h, h), device=like.device, dtype=torch.float64)  # y_i . y_j
        st["m"] = 0

    def _hist_push(self, s, y):
        st = self.state[self._params[0]]
        h = self.param_groups[0]["history_size"]
        S, Y, SY, YY = st["S"], st["Y"], st["SY"], st["YY"]
        m = st["m"]
        if m == h:  # drop the oldest pair (torch: old_dirs.pop(0))
            S[:-1] = S[1:].clone()
            Y[:-1] = Y[1:].clone()
            SY[:-1, :-1] = SY[1:, 1:].clone()
            YY[:-1, :-1] = YY[1:, 1:].clone()
            m -= 1
        S[m].copy_(s)
        Y[m].copy_(y)
        # new column of S^T Y / Y^T Y and new row s_m^T Y: two stacked GEMVs
        a = _rowdots(torch.cat([S[:m + 1], Y[:m + 1]], 0), y)    # [S^T y; Y^T y]
        b = _rowdots(Y[:m + 1], s)                                 # y_j . s_m
        SY[:m + 1, m] = a[:m + 1].double()
        SY[m, :m + 1] = b.double()
        YY[:m + 1, m] = a[m + 1:].double()
        YY[m, :m + 1] = a[m + 1:].double()
        st["m"] = m + 1

    def _hist_apply(self, v, gamma):
        """H v (compact form)."""
        st = self.state[self._params[0]]
        m = st["m"]
        if m == 0:
            return v * gamma
        S, Y = st["S"][:m], st["Y"][:m]
        SY, YY = st["SY"][:m, :m], st["YY"][:m, :m]
        SY_ = torch.cat([S, Y], 0)
        ab = _rowdots(SY_, v).double()
        a, b = ab[:m], ab[m:]
        g = gamma if isinstance(gamma, float) else gamma.double()
        R = torch.triu(SY)
        u = torch.linalg.solve_triangular(R, a[:, None], upper=True)[:, 0]
        w = torch.diagonal(SY) * u + g * _rowdots(YY, u) - g * b
        t = torch.linalg.solve_triangular(R.t(), w[:, None], upper=False)[:, 0]
        coef = torch.cat([t, -g * u]).to(v.dtype)
        return v * gamma + (SY_ * coef[:, None]).sum(0)

    # ------------------------------------------------------------------------------
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

        state = self.state[self._params[0]]
        state.setdefault("func_evals", 0)
        state.setdefault("n_iter", 0)

        orig_loss = closure()
        loss = float(orig_loss)
        current_evals = 1
        state["func_evals"] += 1

        flat_grad = self._gather_flat_grad()
        opt_cond = flat_grad.abs().max() <= tolerance_grad
        if opt_cond:
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
                ys = y.dot(s)
                if ys > 1e-10:
                    self._hist_push(s, y)
                    H_diag = ys / y.dot(y)
                d = self._hist_apply(flat_grad.neg(), H_diag)

            if prev_flat_grad is None:
                prev_flat_grad = flat_grad.clone(memory_format=torch.contiguous_format)
            else:
                prev_flat_grad.copy_(flat_grad)
            prev_loss = loss

            if state["n_iter"] == 1:
                t = min(1.0, 1.0 / flat_grad.abs().sum()) * lr
            else:
                t = lr

            gtd = flat_grad.dot(d)
            if gtd > -tolerance_change:
                break

            ls_func_evals = 0
            if line_search_fn is not None:
                if line_search_fn != "strong_wolfe":
                    raise RuntimeError("only 'strong_wolfe' is supported")
                x_init = self._clone_param()

                def obj_func(x, t, d):
                    return self._directional_evaluate(closure, x, t, d)

                loss, flat_grad, t, ls_func_evals = _strong_wolfe(
                    obj_func, x_init, t, d, loss, flat_grad, gtd, max_ls=max_eval - current_evals)
                self._add_grad(t, d)
                opt_cond = flat_grad.abs().max() <= tolerance_grad
            else:
                self._add_grad(t, d)
                if n_iter != max_iter:
                    with torch.enable_grad():
                        loss = closure()
                    loss = float(loss)
                    flat_grad = self._gather_flat_grad()
                    opt_cond = flat_grad.abs().max() <= tolerance_grad
                    ls_func_evals = 1

            current_evals += ls_func_evals
            state["func_evals"] += ls_func_evals

            if n_iter == max_iter:
                break
            if current_evals >= max_eval:
                break
            if opt_cond:
                break
            if d.mul(t).abs().max() <= tolerance_change:
                break
            if abs(loss - prev_loss) < tolerance_change:
                break

        state["d"] = d
        state["t"] = t
        state["H_diag"] = H_diag
        state["prev_flat_grad"] = prev_flat_grad
        state["prev_loss"] = prev_loss
        return orig_loss
