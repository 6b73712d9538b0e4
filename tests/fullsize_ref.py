"""TEST-ONLY float64 restatements of the reference operators for row subsets at full size.

Each function evaluates, for a subset of target rows (or of support columns), the exact
formulas of the reference against ALL the other points, in row/column chunks, so a 50k-200k
problem can be checked on a few hundred rows (size-independent parity).  They run
on whatever device their inputs live on (float64 on the GPU box: the checker, never the
product).  Each is checked against the oracle (oracle/torch_ref.py, pinned by the goldens) at
small size in tests/test_oracle_golden.py::test_fullsize_ref_formulas.

    LDDMM.py:100-116 (v), :120-138 (mdivsum), :142-159 (Hamiltonian), :176-227 (ODE, with
    gradcomponent: :198-203); kernel.py:186-207, :284-292 (the reductions they use).
"""
import torch


def self_terms(qr, pr, qc, pc, sigma, eta=0.0, chunk=4096):
    """Rows (qr, pr) against columns (qc, pc) of the fused ODE right-hand side:
    v  = KRed - eta GradKRed                                   (LDDMM.py:114)
    mG = -(GenDKRed - eta HessKRed(q,q,p,p) - eta^2 GradLapKRed) (LDDMM.py:198-203)
    g  = p_i . GradKRed_i + eta LapKRed_i    (row form of mdivsum(q,q,p), LDDMM.py:133-135)
    h  = 1/2 p_i . KRed_i - eta p_i . GradKRed_i - 1/2 eta^2 LapKRed_i  (LDDMM.py:150-155)."""
    D = qr.shape[1]
    s = 1.0 / sigma ** 2
    KR = torch.zeros_like(qr)
    GK = torch.zeros_like(qr)
    GD = torch.zeros_like(qr)
    HK = torch.zeros_like(qr)
    GL = torch.zeros_like(qr)
    LK = torch.zeros(qr.shape[0], dtype=qr.dtype, device=qr.device)
    for j0 in range(0, qc.shape[0], chunk):
        qj, pj = qc[j0:j0 + chunk], pc[j0:j0 + chunk]
        z = qr[:, None, :] - qj[None, :, :]
        r2 = (z * z).sum(-1)
        K = torch.exp(-0.5 * s * r2)
        KR = KR + K @ pj
        GK = GK - s * (K[:, :, None] * z).sum(1)
        pp = pr @ pj.T
        GD = GD - s * ((K * pp)[:, :, None] * z).sum(1)
        if eta != 0:
            u = pr[:, None, :] - pj[None, :, :]
            zu = (z * u).sum(-1)
            HK = HK + ((s * s * zu)[:, :, None] * z - s * u).mul(K[:, :, None]).sum(1)
            GL = GL - (z * (K * (s ** 3 * r2 - (D + 2) * s * s))[:, :, None]).sum(1)
            LK = LK + (K * (s * s * r2 - D * s)).sum(1)
    v = KR - eta * GK
    mG = -(GD - eta * HK - eta ** 2 * GL)
    g = (pr * GK).sum(-1) + eta * LK
    h = 0.5 * (pr * KR).sum(-1) - eta * (pr * GK).sum(-1) - 0.5 * eta ** 2 * LK
    return v, mG, g, h


def self_vjp_subset(q, p, a, b, gam, sub, sigma, eta=0.0, chunk=8192):
    """d/d(q_i, p_i), i in sub, of L = sum_k a_k.v_k + b_k.mG_k + gam g_k over ALL rows k
    (b = None: zero mG cotangent): row-side derivatives of the rows in `sub` (columns
    detached) plus column-side derivatives of all rows against the columns in `sub`."""
    qs = q[sub].clone().requires_grad_(True)
    ps = p[sub].clone().requires_grad_(True)

    def part(qr, pr, qc, pc, ar, br):
        v, mG, g, _ = self_terms(qr, pr, qc, pc, sigma, eta)
        L = (ar * v).sum() + gam * g.sum()
        if br is not None:
            L = L + (br * mG).sum()
        return L

    with torch.enable_grad():
        L = part(qs, ps, q, p, a[sub], None if b is None else b[sub])
        gq, gp = torch.autograd.grad(L, (qs, ps))
        for k0 in range(0, q.shape[0], chunk):
            sl = slice(k0, k0 + chunk)
            L = part(q[sl], p[sl], qs, ps, a[sl], None if b is None else b[sl])
            dq, dp = torch.autograd.grad(L, (qs, ps))
            gq, gp = gq + dq, gp + dp
    return gq, gp


def ext_terms(x, q, p, sigma, eta=0.0, chunk=4096):
    """External points x carried by the flow (LDDMM.py:219-227): vx = v(x, q, p) (:100-116)
    and the per-x-row terms of mdivsum(x, q, p) (:120-138), gx_i = s sum_j K (z.p_j) +
    eta s sum_j K (s r2 - D), z = x_i - q_j."""
    D = x.shape[1]
    s = 1.0 / sigma ** 2
    vx = torch.zeros_like(x)
    gx = torch.zeros(x.shape[0], dtype=x.dtype, device=x.device)
    for j0 in range(0, q.shape[0], chunk):
        qj, pj = q[j0:j0 + chunk], p[j0:j0 + chunk]
        z = x[:, None, :] - qj[None, :, :]
        r2 = (z * z).sum(-1)
        K = torch.exp(-0.5 * s * r2)
        vx = vx + K @ pj + eta * s * (K[:, :, None] * z).sum(1)
        gx = gx + s * (K * (z * pj[None]).sum(-1)).sum(1) + eta * s * (K * (s * r2 - D)).sum(1)
    return vx, gx


def ext_vjp_subset(x, q, p, a, gam, xsub, qsub, sigma, eta=0.0, chunk=8192):
    """Of L = sum_i a_i.vx_i + gam gx_i over ALL external rows i: d/dx_i for i in xsub (each
    row depends only on its own x) and d/d(q_j, p_j) for j in qsub (all rows against the
    support columns in qsub)."""
    with torch.enable_grad():
        xs = x[xsub].clone().requires_grad_(True)
        vx, gx = ext_terms(xs, q, p, sigma, eta)
        gxs, = torch.autograd.grad((a[xsub] * vx).sum() + gam * gx.sum(), (xs,))
        qs = q[qsub].clone().requires_grad_(True)
        ps = p[qsub].clone().requires_grad_(True)
        gq = torch.zeros_like(qs)
        gp = torch.zeros_like(ps)
        for k0 in range(0, x.shape[0], chunk):
            sl = slice(k0, k0 + chunk)
            vx, gx = ext_terms(x[sl], qs, ps, sigma, eta)
            dq, dp = torch.autograd.grad((a[sl] * vx).sum() + gam * gx.sum(), (qs, ps))
            gq, gp = gq + dq, gp + dp
    return gxs, gq, gp


def gmm_rows(X, mu, lpi, sigma, lgn, chunk=65536):
    """E-step rows (GMM.py:260-273, 303): T_n = LSE_c t_nc, gamma, Y_n = sum_c gamma_nc mu_c,
    for the rows of X (all components)."""
    Ts, Ys = [], []
    for a in range(0, X.shape[0], chunk):
        Xc = X[a:a + chunk]
        D2 = ((Xc[:, None, :] - mu[None]) ** 2).sum(-1)
        t = lpi[None] - D2 / (2 * sigma ** 2) - lgn
        T = t.logsumexp(1)
        Ts.append(T)
        Ys.append(torch.exp(t - T[:, None]) @ mu)
    return torch.cat(Ts), torch.cat(Ys)


def gmm_columns(X, mu, lpi, sigma, chunk=16384):
    """M-step column statistics over ALL rows (GMM.py:286-297): log sum_n gamma_nc,
    sum_n gamma_nc x_n / sum_n gamma_nc, sum_nc gamma_nc D2_nc (old mu)."""
    C = mu.shape[0]
    m = torch.full((C,), float("-inf"), dtype=X.dtype, device=X.device)
    acc_w = torch.zeros(C, dtype=X.dtype, device=X.device)
    acc_x = torch.zeros_like(mu)
    sd2 = torch.zeros((), dtype=X.dtype, device=X.device)
    for a in range(0, X.shape[0], chunk):
        Xc = X[a:a + chunk]
        D2 = ((Xc[:, None, :] - mu[None]) ** 2).sum(-1)
        t = lpi[None] - D2 / (2 * sigma ** 2)
        lg = t - t.logsumexp(1, keepdim=True)
        mc = lg.max(0).values
        mn = torch.maximum(m, mc)
        sc_old = torch.exp(m - mn)
        sc_old = torch.where(torch.isfinite(m), sc_old, torch.zeros_like(sc_old))
        e = torch.exp(lg - mn[None])
        acc_w = acc_w * sc_old + e.sum(0)
        acc_x = acc_x * sc_old[:, None] + e.T @ Xc
        sd2 = sd2 + (lg.exp() * D2).sum()
        m = mn
    return m + acc_w.log(), acc_x / acc_w[:, None], sd2


# ---------------------------------------------------------------------------------------
# Whole shootings and their gradients at full size (Euler; LDDMM.py:286-299, :318-334,
# integrators.py:20-33; the gradient of tools/optim.py:46's L.backward()), row-chunked
# ---------------------------------------------------------------------------------------
def ode_full(q, p, sigma, eta=0.0, withlogdet=True, rows=2048):
    """LDDMMModel.ODE (LDDMM.py:176-227) for ALL rows: (v, mG, dcost) with dcost =
    mdivsum(q, q, p) = sum_i g_i (hybrid / logdet) or 0 (classic)."""
    vs, ms, gsum = [], [], torch.zeros((), dtype=q.dtype, device=q.device)
    for r0 in range(0, q.shape[0], rows):
        v, mG, g, _ = self_terms(q[r0:r0 + rows], p[r0:r0 + rows], q, p, sigma, eta)
        vs.append(v)
        ms.append(mG)
        gsum = gsum + g.sum()
    dc = gsum if withlogdet else torch.zeros_like(gsum)
    return torch.cat(vs), torch.cat(ms), dc


def hamiltonian_full(q, p, sigma, eta=0.0, rows=2048):
    """H(q, p) (LDDMM.py:142-159) as the sum of self_terms' per-row h."""
    H = torch.zeros((), dtype=q.dtype, device=q.device)
    for r0 in range(0, q.shape[0], rows):
        H = H + self_terms(q[r0:r0 + rows], p[r0:r0 + rows], q, p, sigma, eta)[3].sum()
    return H


def ode_vjp_full(q, p, a, b, gam, sigma, eta=0.0, withlogdet=True, rows=1024, chunk=4096):
    """d/d(q, p) of L = sum_k a_k.v_k + b_k.mG_k + gam dcost over ALL rows (b None: zero mG
    cotangent), by autograd of row chunks of the ODE against all columns."""
    gq = torch.zeros_like(q)
    gp = torch.zeros_like(p)
    with torch.enable_grad():
        qq = q.detach().clone().requires_grad_(True)
        pp = p.detach().clone().requires_grad_(True)
        for r0 in range(0, q.shape[0], rows):
            sl = slice(r0, r0 + rows)
            v, mG, g, _ = self_terms(qq[sl], pp[sl], qq, pp, sigma, eta, chunk)
            L = (a[sl] * v).sum()
            if b is not None:
                L = L + (b[sl] * mG).sum()
            if withlogdet:
                L = L + gam * g.sum()
            dq, dp = torch.autograd.grad(L, (qq, pp))
            gq += dq
            gp += dp
    return gq, gp


def shoot_full(q0, p0, sigma, nt, eta=0.0, withlogdet=True):
    """Euler shooting (integrators.py:20-33 over LDDMM.py:176-227): lists Q, P (nt+1) and
    the cost at each time (float64 scalars)."""
    dt = 1.0 / nt
    Q, P, C = [q0], [p0], [torch.zeros((), dtype=q0.dtype, device=q0.device)]
    for _ in range(nt):
        v, mG, dc = ode_full(Q[-1], P[-1], sigma, eta, withlogdet)
        Q.append(Q[-1] + dt * v)
        P.append(P[-1] + dt * mG)
        C.append(C[-1] + dt * dc)
    return Q, P, C


def shoot_loss_grad_p0(q0, p0, sigma, nt, lam, y, eta=0.0, withlogdet=True, rows=1024, chunk=4096):
    """Optimize's loss at p0 (LDDMM.py:318-334 trajloss + the quadratic data loss
    1/2 |q1 - y|^2) and its gradient w.r.t. p0 (optim.py:46), by the discrete adjoint of
    the Euler shooting with chunked-autograd VJPs of each step.  Returns
    (q1, cost1, trajloss, loss, grad_p0)."""
    dt = 1.0 / nt
    Q, P, C = shoot_full(q0, p0, sigma, nt, eta, withlogdet)
    H0 = hamiltonian_full(q0, p0, sigma, eta)
    traj = lam * H0 + C[-1]
    loss = traj + 0.5 * ((Q[-1] - y) ** 2).sum()
    lq = Q[-1] - y              # dL/dq1
    lp = None                   # the loss does not read p1
    for t in range(nt - 1, -1, -1):
        gq, gp = ode_vjp_full(Q[t], P[t], lq, lp, 1.0, sigma, eta, withlogdet, rows, chunk)
        lq = lq + dt * gq
        lp = (0 if lp is None else lp) + dt * gp
    # dH0/dp0 = v(q0, p0) (eta = 0) -- by autograd of the chunked Hamiltonian in general
    with torch.enable_grad():
        pp = p0.detach().clone().requires_grad_(True)
        dH, = torch.autograd.grad(hamiltonian_full(q0, pp, sigma, eta), (pp,))
    return Q[-1], C[-1], traj, loss, lp + lam * dH
