"""TEST-ONLY executable spec of the C-ABI contract (include/difficp_hip.h), backed by the
CPU oracle.  `install(monkeypatch)` replaces the entry points of difficp_amd._lib so the
host-side logic (shooting adjoint, EM bookkeeping, PSR driver, sharded gloo path) can be
tested on CPU.  Never used by the product: difficp_amd raises without the HIP library.
"""
import math
import os

import torch

from oracle import torch_ref as R

LOG2E = 1.4426950408889634
LN2 = math.log(2.0)


# FAKE_HIP_DTYPE: the arithmetic of the oracle-backed entry points.  float64 (default): an
# executable spec whose only float32 roundings are the outputs'; "float32": the reference's
# own torch path run in float32 (SURVEY 8(c)'s "oracle32"), for the float32 drift that the
# GPU parity tolerances of L-BFGS-driven traces are stated against
_DT = torch.float32 if os.environ.get("FAKE_HIP_DTYPE", "float64") == "float32" else torch.float64


def _d(t):
    return None if t is None else t.detach().to(_DT)


def _out(t, like):
    return t.to(dtype=like.dtype, device=like.device).contiguous()


def gauss_red(op, x, y, sigma, b=None, c=None):
    from difficp_amd import _lib as L
    X, Y, B, Cc = _d(x), _d(y), _d(b), _d(c)
    if op == L.KBASE:
        r = R.KBase(X, Y, sigma)
    elif op == L.KREDSCAL:
        r = R.KRedScal(X, Y, B, sigma)
    elif op == L.KRED:
        r = R.KRed(X, Y, B, sigma)
    elif op == L.GRADK:
        r = R.GradKRed(X, Y, sigma)
    elif op == L.GRADK_REV:          # rows = x here (former columns), cols = (y, b)
        r = R.GradKRed_rev(Y, X, B, sigma)
    elif op == L.DDK:
        r = R.DDKRed(X, Y, B, sigma)
    elif op == L.GENDK:
        r = R.GenDKRed(X, Y, B, Cc, sigma)
    elif op == L.HESSK:
        r = R.HessKRed(X, Y, B, Cc, sigma)
    elif op == L.LAPK:
        r = R.LapKRed(X, Y, sigma)
    elif op == L.GRADLAPK:
        r = R.GradLapKRed(X, Y, sigma)
    elif op == L.GRADKSCAL:
        r = R._rows(lambda xc: torch.sum(R.GradK(xc, Y, sigma) * B[None, :, None], 1), X)
    elif op == L.GRADLAPKSCAL:
        D = X.shape[1]

        def f(xc):
            D2 = torch.sum((xc[:, None, :] - Y[None, :, :]) ** 2, -1)[:, :, None]
            return torch.sum(torch.exp(-D2 / (2 * sigma ** 2)) * (Y[None, :, :] - xc[:, None, :])
                             * (D2 / sigma ** 6 - (D + 2) / sigma ** 4) * B[None, :, None], 1)
        r = R._rows(f, X)
    elif op == L.MIN_SQDIST_OTHER:
        return _out(R.MinSqDistOther(x.detach()), x)
    elif op == L.MIN_SQDIST:
        r = R.MinSqDist(X, Y) if Y.shape[0] else torch.full((X.shape[0],), float("inf"), dtype=_DT)
    else:
        raise NotImplementedError(op)
    return _out(r, x)


def gauss_red_grad(kind, x, y, sigma, r1=None, r2=None, c1=None, c2=None, cw=None):
    """The five pair formulas of dicp_gauss_red_grad_f32 (include/difficp_hip.h), float64."""
    from difficp_amd import _lib as L
    X, Y = _d(x), _d(y)
    M, D = X.shape
    N = Y.shape[0]
    s = 1.0 / sigma ** 2
    z0 = lambda n: torch.zeros(n, D, dtype=_DT)
    R1 = _d(r1) if r1 is not None else z0(M)
    C1 = _d(c1) if c1 is not None else z0(N)
    if kind == L.GRAD_HESSW and r2 is None and c2 is None:
        R2, C2 = z0(M), z0(N)
        R2[:, 0] = 1.0
        C2[:, 0] = 1.0
    else:
        R2 = _d(r2) if r2 is not None else z0(M)
        C2 = _d(c2) if c2 is not None else z0(N)
    W = _d(cw) if cw is not None else torch.ones(N, dtype=_DT)
    z = X[:, None, :] - Y[None, :, :]
    r2v = (z * z).sum(-1)
    K = torch.exp(-0.5 * s * r2v)
    dot = lambda a, b: (a * b).sum(-1)
    if kind in (L.GRAD_HESSW, L.GRAD_HESSWP):
        u = R1[:, None] - C1[None] if kind == L.GRAD_HESSW else R1[:, None] * C1[None]
        w = K * (W[None] * dot(R2[:, None], C2[None]) if kind == L.GRAD_HESSW else 1.0)
        out = (w[..., None] * (s * s * dot(z, u)[..., None] * z - s * u)).sum(1)
    elif kind == L.GRAD_ZDOTV:
        a = R1[:, None] + C1[None]
        out = (-s * (K * dot(z, a))[..., None] * C2[None]).sum(1)
    elif kind == L.GRAD_HESS3:
        u = R1[:, None] - C1[None]
        g = R2[:, None] + C2[None]
        zg, zu, ug = dot(z, g), dot(z, u), dot(u, g)
        t = s * s * (zg[..., None] * u + zu[..., None] * g) - s * z * (s * s * zu * zg - s * ug)[..., None]
        out = (K[..., None] * t).sum(1)
    elif kind == L.GRAD_GRADLAP3:
        g = R1[:, None] + C1[None]
        phi = s ** 3 * r2v - (D + 2) * s * s
        t = phi[..., None] * g + (s ** 3 * (D + 4 - s * r2v) * dot(g, z))[..., None] * z
        out = -(K[..., None] * t).sum(1)
    else:
        raise NotImplementedError(kind)
    return _out(out, x)


def _self_terms(q, p, sigma, eta):
    s = 1.0 / sigma ** 2
    KR = R.KRed(q, q, p, sigma)
    GK = R.GradKRed(q, q, sigma)
    LK = R.LapKRed(q, q, sigma)
    v = KR - eta * GK
    G = R.GenDKRed(q, q, p, p, sigma)
    if eta != 0:
        G = G - eta * R.HessKRed(q, q, p, p, sigma) - eta ** 2 * R.GradLapKRed(q, q, sigma)
    g = (p * GK).sum(-1) + eta * LK
    h = 0.5 * (p * KR).sum(-1) - eta * (p * GK).sum(-1) - 0.5 * eta ** 2 * LK
    return v, -G, g, h


def ode_self_fwd(q, p, sigma, eta, want_div, want_h=False, order=None, zs_out=None):
    if zs_out is not None:
        assert eta == 0 and not want_h
        _zs_rows(q, 0, q.shape[0], sigma, zs_out)
    v, mG, g, h = _self_terms(_d(q), _d(p), sigma, eta)
    return (_out(v, q), _out(mG, q), _out(g, q) if (want_div or eta != 0) else None,
            _out(h, q) if want_h else None)


def ode_self_bwd(q, p, gv, gmG, gdiv, sigma, eta):
    Q = _d(q).requires_grad_(True)
    P = _d(p).requires_grad_(True)
    with torch.enable_grad():
        v, mG, g, _ = _self_terms(Q, P, sigma, eta)
        L = (v * _d(gv)).sum() + (mG * _d(gmG)).sum()
        if gdiv is not None:
            L = L + g.sum() * _d(gdiv).reshape(-1)[0]
        gq, gp = torch.autograd.grad(L, (Q, P))
    return _out(gq, q), _out(gp, q)


def _zs_rows(q, row0, nrows, sigma, zs_out):
    """divergence rows zs_i = sum_j K (q_i - q_j) = -sigma^2 GradKRed(q, q)_i of rows
    [row0, row0 + nrows), into zs_out"""
    Q = _d(q)
    zs_out.copy_(-sigma ** 2 * R.GradKRed(Q[row0:row0 + nrows], Q, sigma))


def euler_step(q, p, sigma, eta, dt, want_div, q_out=None, p_out=None, g_out=None, order=None,
               want_p=True, zs_out=None):
    if zs_out is not None:
        assert eta == 0
        _zs_rows(q, 0, q.shape[0], sigma, zs_out)
    v, mG, g, _ = ode_self_fwd(q, p, sigma, eta, want_div)
    if not want_p:   # like the device pass: p_next is not formed
        p_out = None
    if g_out is not None and g is not None:
        g_out.copy_(g)
        g = g_out
    qn, pn = q + dt * v, p + dt * mG
    if q_out is not None:
        q_out.copy_(qn)
        qn = q_out
    if p_out is not None:
        p_out.copy_(pn)
        pn = p_out
    return qn, (pn if want_p else None), g


def euler_adjoint_step(q, p, lq, lp, gdiv, sigma, eta, dt, addq=None, addp=None, want_lq=True,
                       zs=None):
    if zs is not None:   # the divergence rows must be those of q (the device VJP trusts them)
        ref = torch.empty_like(zs)
        _zs_rows(q, 0, q.shape[0], sigma, ref)
        assert torch.allclose(zs, ref, rtol=1e-5, atol=1e-6)
    if lp is None:   # zero momentum cotangent
        lp = torch.zeros_like(lq)
    gq, gp = ode_self_bwd(q, p, lq, lp, gdiv, sigma, eta)
    lqn, lpn = lq + dt * gq, lp + dt * gp
    if addq is not None:
        lqn = lqn + addq
    if addp is not None:
        lpn = lpn + addp
    return (lqn if want_lq else None), lpn


def _ext_terms(x, q, p, sigma, eta):
    s = 1.0 / sigma ** 2
    D = x.shape[1]
    vx = R.KRed(x, q, p, sigma) - eta * R.GradKRed(x, q, sigma)
    z = x[:, None, :] - q[None, :, :]
    r2 = (z ** 2).sum(-1)
    K = torch.exp(-r2 * s / 2)
    gx = s * (K * (z * p[None, :, :]).sum(-1)).sum(1) + eta * s * (K * (s * r2 - D)).sum(1)
    return vx, gx


def ode_ext_fwd(x, q, p, sigma, eta, want_div):
    vx, gx = _ext_terms(_d(x), _d(q), _d(p), sigma, eta)
    return _out(vx, x), (_out(gx, x) if want_div else None)


def ode_ext_bwd(x, q, p, gvx, gdiv, sigma, eta, gq, gp):
    X = _d(x).requires_grad_(True)
    Q = _d(q).requires_grad_(True)
    P = _d(p).requires_grad_(True)
    with torch.enable_grad():
        vx, gx = _ext_terms(X, Q, P, sigma, eta)
        L = (vx * _d(gvx)).sum()
        if gdiv is not None:
            L = L + gx.sum() * _d(gdiv).reshape(-1)[0]
        ggx, ggq, ggp = torch.autograd.grad(L, (X, Q, P))
    gq += _out(ggq, q)
    gp += _out(ggp, q)
    return _out(ggx, x)


def gmm_estep(X, mu, w2, mu2, sigma, lgn, want_stats, hint=None):   # hint: a shift only (no effect)
    Xd, M, W2 = _d(X), _d(mu), _d(w2)
    D2 = ((Xd[:, None, :] - M[None, :, :]) ** 2).sum(-1)
    t2 = W2[None, :] - D2 * LOG2E / (2 * sigma ** 2)
    T2 = torch.logsumexp(t2 * LN2, 1) / LN2
    T = LN2 * T2 - lgn
    stats = None
    if want_stats:
        g = torch.exp(LN2 * (t2 - T2[:, None]))
        lg = LN2 * (t2 - T2[:, None])
        stats = torch.cat([g @ M, (g * (M ** 2).sum(-1)[None, :]).sum(1, keepdim=True),
                           (g * lg).sum(1, keepdim=True), (g * LN2 * W2[None, :]).sum(1, keepdim=True),
                           (g * D2).sum(1, keepdim=True)], 1)
        stats = _out(stats, X)
    return _out(T, X), _out(T2, X), stats


def gmm_mstep(X, T2, mu, w2, sigma):
    Xd, M, W2 = _d(X), _d(mu), _d(w2)
    D2 = ((Xd[:, None, :] - M[None, :, :]) ** 2).sum(-1)
    lg2 = W2[None, :] - D2 * LOG2E / (2 * sigma ** 2) - _d(T2)[:, None]
    lg = lg2 * LN2
    w_new = torch.logsumexp(lg, 0)
    mu_new = torch.softmax(lg, 0).t() @ Xd
    return _out(torch.cat([w_new[:, None], mu_new], 1), X)


def gmm_targets(X, T2, mu_old, w2_old, sigma_old, mu_new, lpi_new):
    Xd, Mo, W2, Mn, Lp = _d(X), _d(mu_old), _d(w2_old), _d(mu_new), _d(lpi_new)
    D2 = ((Xd[:, None, :] - Mo[None, :, :]) ** 2).sum(-1)
    g = torch.exp(LN2 * (W2[None, :] - D2 * LOG2E / (2 * sigma_old ** 2) - _d(T2)[:, None]))
    D2n = ((Xd[:, None, :] - Mn[None, :, :]) ** 2).sum(-1)
    rows = torch.cat([g @ Mn, (g * (Mn ** 2).sum(-1)[None, :]).sum(1, keepdim=True),
                      (g * Lp[None, :]).sum(1, keepdim=True), g.sum(1, keepdim=True),
                      (g * D2n).sum(1, keepdim=True)], 1)
    return _out(rows, X)


def radius_count(x, y, radius):
    d = R.SqDistF32(x.detach(), y.detach())
    return _out((d <= radius ** 2).sum(1).to(torch.float64), x)


def kernel_ridge_cg(x, v, sigma, alpha, eps=1e-6, maxiter=5000, chunk=32):
    b, k = R.KridgeSolve_cg(_d(x), _d(v), sigma, alpha, eps=eps, maxiter=maxiter)
    st = "converged" if k < maxiter else "maxiter"
    return _out(b, v), {"status": st, "iterations": k, "residual2": 0.0, "threshold": 0.0}


def ode_self_fwd_rows(q, p, row0, nrows, sigma, eta, want_div, want_h=False, order=None, zs_out=None):
    if zs_out is not None:
        assert eta == 0 and not want_h
        _zs_rows(q, row0, nrows, sigma, zs_out)
    v, mG, g, h = ode_self_fwd(q, p, sigma, eta, want_div, want_h)
    sl = slice(row0, row0 + nrows)
    return v[sl].contiguous(), mG[sl].contiguous(), None if g is None else g[sl].contiguous(), \
        None if h is None else h[sl].contiguous()


def euler_step_rows(q, p, row0, nrows, sigma, eta, dt, want_div, q_out=None, p_out=None, order=None,
                    want_p=True, zs_out=None):
    if zs_out is not None:
        assert eta == 0
        _zs_rows(q, row0, nrows, sigma, zs_out)
    v, mG, g, _ = ode_self_fwd_rows(q, p, row0, nrows, sigma, eta, want_div)
    sl = slice(row0, row0 + nrows)
    qn, pn = q[sl] + dt * v, (p[sl] + dt * mG if want_p else None)
    if q_out is not None:
        qn = q_out.copy_(qn)
    if p_out is not None and want_p:
        pn = p_out.copy_(pn)
    return qn, pn, g


def _cross_terms(qr, pr, qc, pc, sigma, eta):
    """(v, mG, g, zs) of the rows (qr, pr) against the columns (qc, pc) only."""
    v = R.KRed(qr, qc, pc, sigma) - eta * R.GradKRed(qr, qc, sigma)
    G = R.GenDKRed(qr, qc, pc, pr, sigma)      # (x, y, column field b, row field c)
    if eta != 0:
        G = G - eta * R.HessKRed(qr, qc, pc, pr, sigma) - eta ** 2 * R.GradLapKRed(qr, qc, sigma)
    g = (pr * R.GradKRed(qr, qc, sigma)).sum(-1) + eta * R.LapKRed(qr, qc, sigma)
    zs = -sigma ** 2 * R.GradKRed(qr, qc, sigma)
    return v, -G, g, zs


def euler_step_phase_ws(nrows, M, D, device):
    return {}


def euler_step_phase(phase, q_loc, p_loc, q, p, row0, nrows, sigma, eta, dt, q_out, p_out=None,
                     g_out=None, zs_out=None, ws=None):
    """dicp_lddmm_euler_step_phase_f32: phase 0 = the rows against their own slice (kept in
    ws), phase 1 = against the other points (wrapping from row0 + nrows), then the step."""
    if phase == 0:
        ws["part"] = _cross_terms(_d(q_loc), _d(p_loc), _d(q_loc), _d(p_loc), sigma, eta)
        return q_out
    M = q.shape[0]
    idx = [(row0 + nrows + j) % M for j in range(M - nrows)]
    Q, P = _d(q), _d(p)
    rq, rp = Q[row0:row0 + nrows], P[row0:row0 + nrows]
    rem = _cross_terms(rq, rp, Q[idx], P[idx], sigma, eta)
    v, mG, g, zs = (a + b for a, b in zip(ws.pop("part"), rem))
    for out, val in ((q_out, rq + dt * v), (p_out, rp + dt * mG), (g_out, g), (zs_out, zs)):
        if out is not None:
            out.copy_(val.to(out.dtype))
    return q_out


def ode_self_bwd_part(q, p, gv, gmG, gdiv, sigma, eta, part, nparts, want_gq=True, zs=None, zrow0=0,
                      gq_out=None, gp_out=None):
    """Row-slice decomposition (the kernels' eta != 0 split): part r holds the full VJP of
    its rows, zeros elsewhere; the sum over parts is the VJP."""
    if zs is not None:   # the rank's own forward slice of the divergence rows
        ref = torch.empty_like(zs)
        _zs_rows(q, zrow0, zs.shape[0], sigma, ref)
        assert torch.allclose(zs, ref, rtol=1e-5, atol=1e-6)
    if gmG is None:   # zero momentum cotangent
        gmG = torch.zeros_like(gv)
    gq, gp = ode_self_bwd(q, p, gv, gmG, gdiv, sigma, eta)
    M = q.shape[0]
    per = -(-M // nparts)
    r0, r1 = min(per * part, M), min(per * part + per, M)
    mask = torch.zeros(M, 1, dtype=gq.dtype)
    mask[r0:r1] = 1
    gq, gp = gq * mask, gp * mask
    if gq_out is not None and want_gq:
        gq = gq_out.copy_(gq)
    if gp_out is not None:
        gp = gp_out.copy_(gp)
    return (gq if want_gq else None), gp


_ENTRIES = ("gauss_red_grad", "ode_self_fwd_rows", "euler_step_rows", "euler_step_phase", "euler_step_phase_ws", "ode_self_bwd_part", "kernel_ridge_cg", "euler_step", "euler_adjoint_step", "radius_count", "gauss_red", "ode_self_fwd", "ode_self_bwd", "ode_ext_fwd", "ode_ext_bwd",
            "gmm_estep", "gmm_mstep", "gmm_targets")


def install(monkeypatch):
    from difficp_amd import _lib
    g = globals()
    for name in _ENTRIES:
        monkeypatch.setattr(_lib, name, g[name])


def install_plain():
    """Without pytest (subprocess workers of the gloo tests)."""
    from difficp_amd import _lib
    g = globals()
    for name in _ENTRIES:
        setattr(_lib, name, g[name])
