"""Where does the eta != 0 (logdet, exact ICP_two_set model) cost integral lose accuracy?
(VERDICT r05 "Next round" 1.)  On the failing case of tests/test_gpu_e2e_fullsize.py
(M points, small displacement around the ridge zero-speed a0), compares step by step:

* the per-step cost increments C[t+1] - C[t] of the HIP shooting, the float32 restatement and
  the float64 restatement (tests/fullsize_ref.py) -- trajectory + evaluation error;
* at the float64 trajectory's own states (cast to float32): the HIP forward's divergence rows g
  and Hamiltonian rows h against float64 rows, summed in float32 (as the shooting does) and in
  float64 -- evaluation error alone, split into the per-row error and the row-sum error;
* the magnitudes of the two cancelling terms of g (-s/alpha p.Z' and eta s L).

Usage (GPU box): python tools/probes/logdet_cost_diag.py [--M 20000] [--disp small] > out.jsonl
                 python tools/probes/logdet_cost_diag.py mixed [--M 20000]   (mixed_shoot)
"""
import argparse
import json
import math
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import fullsize_ref as F  # noqa: E402  (test-only checker)

SIG, LAM, NT = 0.1, 1e3, 10


def rel(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    n = float(b.norm())
    return float((a - b).norm()) / n if n > 0 else float((a - b).norm())


def rows_all(q, p, eta, rows=2048):
    """g, h, eta L, mG and GradKRed rows of every point (float64 or float32 as the inputs)."""
    out = [[], [], [], [], []]
    s = 1.0 / SIG ** 2
    for r0 in range(0, q.shape[0], rows):
        v, mG, g, h = F.self_terms(q[r0:r0 + rows], p[r0:r0 + rows], q, p, SIG, eta)
        out[0].append(g)
        out[1].append(h)
        out[3].append(mG)
        # the two cancelling parts of g: p_i.GradKRed_i and eta LapKRed_i
        qr = q[r0:r0 + rows]
        lk = torch.zeros(qr.shape[0], dtype=q.dtype, device=q.device)
        gk = torch.zeros_like(qr)
        for j0 in range(0, q.shape[0], 4096):
            z = qr[:, None, :] - q[None, j0:j0 + 4096, :]
            r2 = (z * z).sum(-1)
            K = torch.exp(-0.5 * s * r2)
            lk = lk + (K * (s * s * r2 - 3 * s)).sum(1)
            gk = gk - s * (K[:, :, None] * z).sum(1)
        out[2].append(eta * lk)
        out[4].append(gk)
    return [torch.cat(o) for o in out]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=20000)
    ap.add_argument("--disp", default="small")
    ap.add_argument("--steps", default="0,5,9")
    ap.add_argument("--coord", default="auto", help="LDDMMModel.coord_mode of the HIP shooting")
    args = ap.parse_args()
    from difficp_amd import _lib, workloads
    from difficp_amd.core.LDDMM import LDDMMModel
    dev = torch.device("cuda:0")
    M = args.M
    _, xB = workloads.two_set_points(M, seed=3)
    q0 = xB.double().to(dev)
    g = torch.Generator().manual_seed(M)
    ph = torch.rand(3, generator=g, dtype=torch.float64).to(dev)
    amp = 2e-6
    if args.disp != "small":
        pr = 1e-6 * torch.sin(2 * math.pi * (q0[:, [1, 2, 0]] + ph))
        v, _, _ = F.ode_full(q0, pr, SIG, 0.0, True)
        amp = 1e-6 * float(args.disp) * SIG / float(v.norm(dim=1).max())
    p0 = amp * torch.sin(2 * math.pi * (q0[:, [1, 2, 0]] + ph))
    eta = 1.0 / LAM
    LM0 = LDDMMModel(sigma=SIG, D=3, lambd=LAM, version="logdet", scheme="Euler", nt=NT,
                     spec={"device": dev, "dtype": torch.float32})
    q32 = q0.float().contiguous()
    a0 = LM0.v2p(q32, torch.zeros_like(q32), version="ridge_keops", alpha=1e-3)
    p0 = p0 + a0.double()

    Q64, P64, C64 = F.shoot_full(q0, p0, SIG, NT, eta, True)
    Q32, P32, C32 = F.shoot_full(q0.float(), p0.float(), SIG, NT, eta, True)
    LM = LDDMMModel(sigma=SIG, D=3, lambd=LAM, version="logdet", scheme="Euler", nt=NT,
                    spec={"device": dev, "dtype": torch.float32})
    LM.shoot_cache = None
    LM.coord_mode = args.coord
    with torch.no_grad():
        sh = LM.Shoot(q0.float().contiguous(), p0.float().contiguous(), need_p1=False)
    Ch = [float(sh[t][2].reshape(())) for t in range(NT + 1)]
    c64 = [float(c) for c in C64]
    c32 = [float(c) for c in C32]
    print(json.dumps({"what": "cost", "M": M, "disp": args.disp, "coord": args.coord, "C64": c64, "C32": c32, "Chip": Ch,
                      "rel_C32": abs(c32[-1] - c64[-1]) / abs(c64[-1]),
                      "rel_Chip": abs(Ch[-1] - c64[-1]) / abs(c64[-1])}), flush=True)
    for t in range(NT):
        d64 = c64[t + 1] - c64[t]
        print(json.dumps({"what": "inc", "t": t, "d64": d64, "d32": c32[t + 1] - c32[t],
                          "dhip": Ch[t + 1] - Ch[t],
                          "q_rel_hip": rel(sh[t][0], Q64[t]), "q_rel_32": rel(Q32[t], Q64[t]),
                          "p_rel_hip": rel(sh[t][1], P64[t]) if t < NT else None,
                          "p_rel_32": rel(P32[t], P64[t])}), flush=True)

    for t in [int(s) for s in args.steps.split(",")]:
        q, p = Q64[t], P64[t]
        g64, h64, el, m64, gk64 = rows_all(q, p, eta)
        gq, hq, _, mq, _ = rows_all(q.float(), p.float(), eta)
        with _lib.coord_mode(args.coord == "raw"):
            _, mh, gh, hh = _lib.ode_self_fwd(q.float().contiguous(), p.float().contiguous(), SIG, eta, True,
                                             want_h=True)
        torch.cuda.synchronize()
        S64 = float(g64.sum())
        rec = {"what": "eval", "t": t, "sum_g64": S64, "sum_abs_g64": float(g64.abs().sum()),
               "sum_abs_etaL": float(el.abs().sum()), "max_abs_etaL": float(el.abs().max()),
               "rows_rel_hip": rel(gh, g64), "rows_rel_32": rel(gq, g64),
               "sum_hip_f32": float(gh.sum()), "sum_hip_f64": float(gh.double().sum()),
               "sum_32_f32": float(gq.sum()), "sum_32_f64": float(gq.double().sum())}
        for k in ("sum_hip_f32", "sum_hip_f64", "sum_32_f32", "sum_32_f64"):
            rec["rel_" + k] = abs(rec[k] - S64) / abs(S64)
        # per-row error statistics: is it a few bad rows or all of them?
        eh = (gh.double() - g64)
        e3 = (gq.double() - g64)
        rec["row_err_hip_mean"] = float(eh.mean())
        rec["row_err_32_mean"] = float(e3.mean())
        rec["row_err_hip_rms"] = float(eh.pow(2).mean().sqrt())
        rec["row_err_32_rms"] = float(e3.pow(2).mean().sqrt())
        # mG: norm error and its projection on GradKRed (the direction in which a momentum
        # error moves sum g = sum_i p_i.GradKRed_i + eta sum LapKRed)
        rec["mG_rel_hip"] = rel(mh, m64)
        rec["mG_rel_32"] = rel(mq, m64)
        rec["mG_proj_hip"] = float(((mh.double() - m64) * gk64).sum())
        rec["mG_proj_32"] = float(((mq.double() - m64) * gk64).sum())
        rec["mG_proj_scale"] = float((m64.abs() * gk64.abs()).sum())
        H64 = float(h64.sum())
        rec.update({"H64": H64, "rel_H_hip_f32": abs(float(hh.sum()) - H64) / abs(H64),
                    "rel_H_hip_f64": abs(float(hh.double().sum()) - H64) / abs(H64),
                    "rel_H_32_f32": abs(float(hq.sum()) - H64) / abs(H64),
                    "rel_H_32_f64": abs(float(hq.double().sum()) - H64) / abs(H64),
                    "h_rows_rel_hip": rel(hh, h64), "h_rows_rel_32": rel(hq, h64),
                    "h_row_err_hip_mean": float((hh.double() - h64).mean()),
                    "h_row_err_32_mean": float((hq.double() - h64).mean())})
        print(json.dumps(rec), flush=True)




def mixed_shoot(q0, p0, eta, src_v, src_m, src_g, coord="auto"):
    """Euler shooting in float64 whose v / mG / g (divergence rows) come, each, from one of
    'f64' (the float64 restatement), 'f32' (the float32 restatement at the float32-cast state)
    or 'hip' (the HIP forward at the float32-cast state): which output's evaluation error
    drives the cost drift.  Returns the cost after each step."""
    from difficp_amd import _lib
    dt = 1.0 / NT
    q, p, C, Cs = q0, p0, 0.0, []
    for _ in range(NT):
        outs = {}
        need = {src_v, src_m, src_g}
        if "f64" in need:
            outs["f64"] = F.ode_full(q, p, SIG, eta, True)
        if "f32" in need:
            v, m, d = F.ode_full(q.float(), p.float(), SIG, eta, True)
            outs["f32"] = (v.double(), m.double(), d.double())
        if "hip" in need:
            with _lib.coord_mode(coord == "raw"):
                v, m, g, _ = _lib.ode_self_fwd(q.float().contiguous(), p.float().contiguous(), SIG, eta, True)
            outs["hip"] = (v.double(), m.double(), g.double().sum())
        v, m, d = outs[src_v][0], outs[src_m][1], outs[src_g][2]
        q, p, C = q + dt * v, p + dt * m, C + dt * float(d)
        Cs.append(C)
    return Cs


def mixed_main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=20000)
    ap.add_argument("--coord", default="auto")
    args = ap.parse_args(sys.argv[2:])
    from difficp_amd import workloads
    from difficp_amd.core.LDDMM import LDDMMModel
    dev = torch.device("cuda:0")
    M = args.M
    _, xB = workloads.two_set_points(M, seed=3)
    q0 = xB.double().to(dev)
    g = torch.Generator().manual_seed(M)
    ph = torch.rand(3, generator=g, dtype=torch.float64).to(dev)
    p0 = 2e-6 * torch.sin(2 * math.pi * (q0[:, [1, 2, 0]] + ph))
    eta = 1.0 / LAM
    LM0 = LDDMMModel(sigma=SIG, D=3, lambd=LAM, version="logdet", scheme="Euler", nt=NT,
                     spec={"device": dev, "dtype": torch.float32})
    q32 = q0.float().contiguous()
    a0 = LM0.v2p(q32, torch.zeros_like(q32), version="ridge_keops", alpha=1e-3)
    p0 = p0 + a0.double()
    ref = mixed_shoot(q0, p0, eta, "f64", "f64", "f64")
    for combo in [("f32", "f64", "f64"), ("f64", "f32", "f64"), ("f64", "f64", "f32"),
                  ("hip", "f64", "f64"), ("f64", "hip", "f64"), ("f64", "f64", "hip"),
                  ("f32", "f32", "f32"), ("hip", "hip", "hip")]:
        Cs = mixed_shoot(q0, p0, eta, *combo, coord=args.coord)
        print(json.dumps({"what": "mixed", "M": M, "coord": args.coord, "v": combo[0], "mG": combo[1],
                          "g": combo[2], "rel_C1": abs(Cs[-1] - ref[-1]) / abs(ref[-1]),
                          "err": [c - r for c, r in zip(Cs, ref)]}), flush=True)


def vsrc_main():
    """Where does the velocity's evaluation error come from (the output whose error drives the
    cost drift, mixed_main)?  At the start state: the first-order effect of each variant's v
    error on the next step's sum g, dt * sum_i (v_i - v64_i) . d(sum g)/dq_i, against float64."""
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=20000)
    args = ap.parse_args(sys.argv[2:])
    from difficp_amd import _lib, workloads
    from difficp_amd.core.LDDMM import LDDMMModel
    dev = torch.device("cuda:0")
    M = args.M
    _, xB = workloads.two_set_points(M, seed=3)
    q0 = xB.double().to(dev)
    g = torch.Generator().manual_seed(M)
    ph = torch.rand(3, generator=g, dtype=torch.float64).to(dev)
    p0 = 2e-6 * torch.sin(2 * math.pi * (q0[:, [1, 2, 0]] + ph))
    eta = 1.0 / LAM
    LM0 = LDDMMModel(sigma=SIG, D=3, lambd=LAM, version="logdet", scheme="Euler", nt=NT,
                     spec={"device": dev, "dtype": torch.float32})
    q32 = q0.float().contiguous()
    a0 = LM0.v2p(q32, torch.zeros_like(q32), version="ridge_keops", alpha=1e-3)
    p0 = p0 + a0.double()
    s = 1.0 / SIG ** 2
    q, p = q0, p0
    qf, pf = q.float(), p.float()
    gq, _ = F.ode_vjp_full(q, p, torch.zeros_like(q), None, 1.0, SIG, eta, True)
    v64 = F.ode_full(q, p, SIG, eta, True)[0]
    dt = 1.0 / NT

    def v_variant(kind, rows=2048, chunk=4096):
        out = []
        for r0 in range(0, M, rows):
            if kind == "in64":          # float64 arithmetic on the float32-rounded inputs
                qr, qc, pc = qf[r0:r0 + rows].double(), qf.double(), pf.double()
            else:
                qr, qc, pc = qf[r0:r0 + rows], qf, pf
            V = torch.zeros(qr.shape, dtype=torch.float64, device=dev)
            Z = torch.zeros(qr.shape, dtype=torch.float64, device=dev)
            for j0 in range(0, M, chunk):
                qj, pj = qc[j0:j0 + chunk], pc[j0:j0 + chunk]
                z = qr[:, None, :] - qj[None]
                K = torch.exp(-0.5 * s * (z * z).sum(-1))
                if kind == "k32acc64":    # K (and z) in float32, products and sums in float64
                    V += K.double() @ pj.double()
                    Z += (K.double()[:, :, None] * z.double()).sum(1)
                elif kind == "k32p64":    # K in float32, p exact (float64), sums float64
                    V += K.double() @ p[j0:j0 + chunk]
                    Z += (K.double()[:, :, None] * z.double()).sum(1)
                else:
                    V += K @ pj if kind == "in64" else (K @ pj).double()
                    Z += (K[:, :, None] * z).sum(1).double()
            out.append(V + eta * s * Z)
        return torch.cat(out)

    res = {}
    for kind in ("in64", "k32acc64", "k32p64", "f32"):
        res[kind] = v_variant(kind)
    for mode in ("auto", "raw"):
        with _lib.coord_mode(mode == "raw"):
            res["hip_" + mode] = _lib.ode_self_fwd(qf.contiguous(), pf.contiguous(), SIG, eta, True)[0].double()
    for k, v in res.items():
        e = v - v64
        print(json.dumps({"what": "vsrc", "M": M, "variant": k, "rel": rel(v, v64),
                          "proj": float(dt * (e * gq).sum()),
                          "proj_abs_scale": float(dt * (e.abs() * gq.abs()).sum())}), flush=True)


def accum_main():
    """Which accumulation scheme of the velocity sums V = sum K p, Z = sum K z (float32 pair
    terms as the kernels form them) removes the systematic v error (vsrc_main): sequential
    float32 sums over sub-tiles of T columns, sub-tile totals in float32 or float64 -- the
    first-order effect on the next step's sum g, as vsrc_main."""
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=20000)
    args = ap.parse_args(sys.argv[2:])
    from difficp_amd import workloads
    from difficp_amd.core.LDDMM import LDDMMModel
    dev = torch.device("cuda:0")
    M = args.M
    _, xB = workloads.two_set_points(M, seed=3)
    q0 = xB.double().to(dev)
    g = torch.Generator().manual_seed(M)
    ph = torch.rand(3, generator=g, dtype=torch.float64).to(dev)
    p0 = 2e-6 * torch.sin(2 * math.pi * (q0[:, [1, 2, 0]] + ph))
    eta = 1.0 / LAM
    LM0 = LDDMMModel(sigma=SIG, D=3, lambd=LAM, version="logdet", scheme="Euler", nt=NT,
                     spec={"device": dev, "dtype": torch.float32})
    q32 = q0.float().contiguous()
    a0 = LM0.v2p(q32, torch.zeros_like(q32), version="ridge_keops", alpha=1e-3)
    p = p0 + a0.double()
    q = q0
    s = 1.0 / SIG ** 2
    qf, pf = q.float(), p.float()
    gq, _ = F.ode_vjp_full(q, p, torch.zeros_like(q), None, 1.0, SIG, eta, True)
    v64 = F.ode_full(q, p, SIG, eta, True)[0]
    dt = 1.0 / NT
    schemes = [(256, "f32"), (256, "f64"), (64, "f64"), (32, "f64"), (16, "f64"), (8, "f64"),
               (1, "f64")]
    B = 256
    accs = {sc: (torch.zeros(M, 6, dtype=torch.float32, device=dev),
                 torch.zeros(M, 6, dtype=torch.float64 if sc[1] == "f64" else torch.float32, device=dev))
            for sc in schemes}
    for j0 in range(0, M, B):
        qj, pj = qf[j0:j0 + B], pf[j0:j0 + B]
        z = qf[:, None, :] - qj[None]                       # (M, B, 3) float32
        K = torch.exp(-0.5 * s * (z * z).sum(-1))           # float32
        terms = torch.cat([K[:, :, None] * pj[None], K[:, :, None] * z], 2)   # (M, B, 6) float32
        for c in range(terms.shape[1]):
            t = terms[:, c]
            for (T, tot) in schemes:
                part, total = accs[(T, tot)]
                part += t
                if (c + 1) % T == 0 or c == terms.shape[1] - 1:
                    total += part.to(total.dtype)
                    part.zero_()
    for sc in schemes:
        tot = accs[sc][1].double()
        v = tot[:, :3] + eta * s * tot[:, 3:]
        e = v - v64
        print(json.dumps({"what": "accum", "M": M, "subtile": sc[0], "total": sc[1], "rel": rel(v, v64),
                          "proj": float(dt * (e * gq).sum())}), flush=True)


def const_main():
    """Do the float32 roundings of the kernels' launch constants drive the systematic v error?
    Float64 sums over the float32-rounded points, with (a) the exact exponent and coefficient,
    (b) the exponent of the float32 coordinate scale alpha32 (K = 2^(-alpha32^2 |z|^2), i.e. a
    sigma off by alpha's rounding), (c) the coefficient of Z' as the kernel forms it
    (eta32 * (s / alpha64)_32, applied to sum K alpha32 z), (d) both -- each as vsrc_main's
    first-order effect on the next step's sum g."""
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=20000)
    args = ap.parse_args(sys.argv[2:])
    import numpy as np
    from difficp_amd import workloads
    from difficp_amd.core.LDDMM import LDDMMModel
    dev = torch.device("cuda:0")
    M = args.M
    _, xB = workloads.two_set_points(M, seed=3)
    q0 = xB.double().to(dev)
    g = torch.Generator().manual_seed(M)
    ph = torch.rand(3, generator=g, dtype=torch.float64).to(dev)
    p0 = 2e-6 * torch.sin(2 * math.pi * (q0[:, [1, 2, 0]] + ph))
    eta = 1.0 / LAM
    LM0 = LDDMMModel(sigma=SIG, D=3, lambd=LAM, version="logdet", scheme="Euler", nt=NT,
                     spec={"device": dev, "dtype": torch.float32})
    q32 = q0.float().contiguous()
    a0 = LM0.v2p(q32, torch.zeros_like(q32), version="ridge_keops", alpha=1e-3)
    p = p0 + a0.double()
    q = q0
    s = 1.0 / SIG ** 2
    gq, _ = F.ode_vjp_full(q, p, torch.zeros_like(q), None, 1.0, SIG, eta, True)
    v64 = F.ode_full(q, p, SIG, eta, True)[0]
    dt = 1.0 / NT
    qd, pd = q.float().double(), p.float().double()
    a64 = math.sqrt(1.4426950408889634 / (2.0 * SIG * SIG))
    a32 = float(np.float32(a64))
    sa32 = float(np.float32(s / a64))
    c_kernel = float(np.float32(np.float32(eta) * np.float32(sa32)))   # eta * sa in the store

    def v_of(alpha_exp, coef, rows=2048, chunk=4096):
        out = []
        for r0 in range(0, M, rows):
            qr = qd[r0:r0 + rows]
            V = torch.zeros_like(qr)
            Z = torch.zeros_like(qr)
            for j0 in range(0, M, chunk):
                z = qr[:, None, :] - qd[None, j0:j0 + chunk]
                K = torch.exp2(-(alpha_exp ** 2) * (z * z).sum(-1))
                V += K @ pd[j0:j0 + chunk]
                Z += (K[:, :, None] * z).sum(1)
            out.append(V + coef * Z)
        return torch.cat(out)

    for name, ae, co in (("exact", a64, eta * s), ("alpha32_exponent", a32, eta * s),
                         ("kernel_coef", a64, c_kernel * a32), ("both", a32, c_kernel * a32)):
        v = v_of(ae, co)
        e = v - v64
        print(json.dumps({"what": "const", "M": M, "variant": name, "rel": rel(v, v64),
                          "proj": float(dt * (e * gq).sum()), "alpha_rel": a32 / a64 - 1,
                          "coef_rel": c_kernel * a32 / (eta * s) - 1}), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "mixed":
        mixed_main()
    elif len(sys.argv) > 1 and sys.argv[1] == "vsrc":
        vsrc_main()
    elif len(sys.argv) > 1 and sys.argv[1] == "accum":
        accum_main()
    elif len(sys.argv) > 1 and sys.argv[1] == "const":
        const_main()
    else:
        main()
