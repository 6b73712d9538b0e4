"""Generate the golden fixtures of tests/golden/*.npz by IMPORTING THE REFERENCE ITSELF
(AdrienWohrer/diff-icp at /root/reference, torch path) -- build container only; the GPU
box never runs this (the reference does not exist there).  No reference source is copied:
the script imports the package and records inputs/outputs of its public functions.

pykeops is absent, and diffICP/tools/point_sets.py:8 imports it unconditionally, so a stub
module is placed in sys.modules AFTER importing kernel/LDDMM (which guard their import), and
GMM.use_keops is forced False: every computversion then resolves to the reference's own
torch implementation.

    python tests/golden/make_golden.py [--only c1|decim|psr_std|chui]
"""
import importlib.machinery
import os
import sys
import types
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def import_reference():
    import matplotlib
    matplotlib.use("Agg")
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    import diffICP.tools.kernel as K  # noqa: F401  (guarded keops import -> torch path)
    import diffICP.core.LDDMM as L  # noqa: F401
    pk = types.ModuleType("pykeops")
    pk.__spec__ = importlib.machinery.ModuleSpec("pykeops", None)
    pkt = types.ModuleType("pykeops.torch")
    pkt.__spec__ = importlib.machinery.ModuleSpec("pykeops.torch", None)

    def _nope(*a, **k):
        raise RuntimeError("keops unavailable")
    pkt.LazyTensor = pkt.Vi = pkt.Vj = pkt.Pm = _nope
    pk.torch = pkt
    sys.modules["pykeops"] = pk
    sys.modules["pykeops.torch"] = pkt
    import diffICP.core.GMM as G
    G.use_keops = False
    import diffICP.core.PSR as P

    # kernel.py:328's torch branch compares a (values, indices) namedtuple with a float and
    # raises; patch in the intended boolean for non-dense supports.
    def check_coverage(self, X, Y, Rthreshold):
        return ((X[:, None, :] - Y[None, :, :]) ** 2).sum(-1).min(dim=1).values > (Rthreshold * self.sigma) ** 2
    K.GaussKernel.check_coverage = check_coverage
    return K, L, G, P


def main():
    import torch
    K, L, G, P = import_reference()
    torch.manual_seed(20261015)
    f64 = torch.float64

    # ---------------- 1. the ten reductions (kernel.py:177-292) ----------------
    red = {}
    for (M, N, D, sig) in [(64, 96, 2, 0.05), (64, 96, 3, 0.2), (64, 96, 2, 1.0), (300, 300, 3, 0.2)]:
        key = f"M{M}_N{N}_D{D}_s{sig}"
        g = torch.Generator().manual_seed(M * 7 + N + D)
        x = torch.rand(M, D, generator=g, dtype=f64)
        y = torch.rand(N, D, generator=g, dtype=f64)
        b = torch.randn(N, D, generator=g, dtype=f64)
        c = torch.randn(M, D, generator=g, dtype=f64)
        d = torch.randn(N, generator=g, dtype=f64)
        dm = torch.randn(M, D, generator=g, dtype=f64)
        GK = K.GaussKernel(sig, D, computversion="torch", spec={"device": "cpu", "dtype": f64})
        for nm, t in dict(x=x, y=y, b=b, c=c, d=d, dm=dm).items():
            red[f"{key}/in_{nm}"] = t.numpy()
        red[f"{key}/sigma"] = np.array(sig)
        red[f"{key}/KBase"] = GK.KBase(x, y).numpy()
        red[f"{key}/KRedScal"] = GK.KRedScal(x, y, d).numpy()
        red[f"{key}/KRed"] = GK.KRed(x, y, b).numpy()
        red[f"{key}/GradKRed"] = GK.GradKRed(x, y).numpy()
        red[f"{key}/GradKRed_rev"] = GK.GradKRed_rev(x, y, dm).numpy()
        red[f"{key}/DDKRed"] = GK.DDKRed(x, y, b).numpy()
        red[f"{key}/GenDKRed"] = GK.GenDKRed(x, y, b, c).numpy()
        red[f"{key}/HessKRed"] = GK.HessKRed(x, y, b, c).numpy()
        red[f"{key}/LapKRed"] = GK.LapKRed(x, y).numpy()
        red[f"{key}/GradLapKRed"] = GK.GradLapKRed(x, y).numpy()
    np.savez_compressed(os.path.join(HERE, "reductions.npz"), **red)

    # ---------------- 2. LDDMM shooting + gradients (LDDMM.py:100-334) ----------------
    sh = {}
    for version in ("classic", "hybrid", "logdet"):
        for scheme in ("Euler", "Ralston"):
            for ext in (0, 30):
                for D in (2, 3):
                    key = f"{version}_{scheme}_x{ext}_D{D}"
                    g = torch.Generator().manual_seed(zlib.crc32(key.encode()))
                    M, lam, sig, nt = 40, 50.0, 0.3, 6
                    q0 = torch.rand(M, D, generator=g, dtype=f64)
                    p0 = 0.05 * torch.randn(M, D, generator=g, dtype=f64)
                    x0 = torch.rand(ext, D, generator=g, dtype=f64) if ext else None
                    tgt = torch.randn(ext if ext else M, D, generator=g, dtype=f64)
                    LM = L.LDDMMModel(sigma=sig, D=D, lambd=lam, version=version, scheme=scheme, nt=nt,
                                      computversion="torch", spec={"device": "cpu", "dtype": f64})
                    pr = p0.clone().requires_grad_(True)
                    s = LM.Shoot(q0, pr, x0)
                    last = s[-1][-1] if ext else s[-1][0]
                    traj = LM.trajloss(s)
                    Lt = traj + ((last - tgt) ** 2).sum()
                    (gp,) = torch.autograd.grad(Lt, (pr,))
                    sh[f"{key}/q0"] = q0.numpy()
                    sh[f"{key}/p0"] = p0.numpy()
                    if ext:
                        sh[f"{key}/x0"] = x0.numpy()
                    sh[f"{key}/tgt"] = tgt.numpy()
                    sh[f"{key}/params"] = np.array([sig, lam, nt])
                    sh[f"{key}/q1"] = s[-1][0].detach().numpy()
                    sh[f"{key}/p1"] = s[-1][1].detach().numpy()
                    sh[f"{key}/cost1"] = s[-1][2].detach().numpy()
                    if ext:
                        sh[f"{key}/x1"] = s[-1][3].detach().numpy()
                    sh[f"{key}/trajloss"] = np.array(traj.item())
                    sh[f"{key}/loss"] = np.array(Lt.item())
                    sh[f"{key}/grad_p0"] = gp.numpy()
                    sh[f"{key}/H0"] = np.array(LM.Hamiltonian(q0, p0).item())
    np.savez_compressed(os.path.join(HERE, "shoot.npz"), **sh)

    # ---------------- 3. EM step (GMM.py:236-325) + log-likelihoods (:714-721) ----------------
    em = {}
    opts = {"all": dict(mu=True, w=True, sigma=True, eta0=True),
            "sigma": dict(mu=False, w=False, sigma=True, eta0=True),
            "mu": dict(mu=True, w=False, sigma=False, eta0=False),
            "mu_w": dict(mu=True, w=True, sigma=False, eta0=True)}
    for D in (2, 3):
        for outl in (False, True):
            for oname, opt in opts.items():
                key = f"D{D}_out{int(outl)}_{oname}"
                g = torch.Generator().manual_seed(zlib.crc32(key.encode()))
                N, C = 200, 12
                X = torch.rand(N, D, generator=g, dtype=f64)
                mu = torch.rand(C, D, generator=g, dtype=f64)
                w = 0.3 * torch.randn(C, generator=g, dtype=f64)
                GM = G.GaussianMixtureUnif(mu, sigma=0.15, use_outliers=outl, computversion="torch",
                                           spec={"device": "cpu", "dtype": f64})
                GM.w = w.clone()
                GM.to_optimize = dict(opt)
                em[f"{key}/X"] = X.numpy()
                em[f"{key}/mu0"] = mu.numpy()
                em[f"{key}/w0"] = w.numpy()
                em[f"{key}/sigma0"] = np.array(0.15)
                for it in range(2):
                    Y, Cfe, FE = GM.EM_step(X)
                    em[f"{key}/it{it}/Y"] = Y.numpy()
                    em[f"{key}/it{it}/Cfe"] = np.array(float(Cfe))
                    em[f"{key}/it{it}/FE"] = np.array(float(FE))
                    em[f"{key}/it{it}/mu"] = GM.mu.numpy()
                    em[f"{key}/it{it}/w"] = GM.w.numpy()
                    em[f"{key}/it{it}/sigma"] = np.array(GM.sigma)
                    if outl:
                        em[f"{key}/it{it}/eta0"] = np.array(GM.outliers["eta0"])
                        em[f"{key}/it{it}/vol0"] = np.array(GM.outliers["vol0"])
                em[f"{key}/loglik"] = GM.log_likelihoods(X).numpy()
                Ys, Cs, Fs = GM.EM_step(X, skip_M=True)
                em[f"{key}/skipM/Y"] = Ys.numpy()
                em[f"{key}/skipM/FE"] = np.array(float(Fs))
    np.savez_compressed(os.path.join(HERE, "em.npz"), **em)

    # ---------------- 4. PSR traces (PSR.py:242-569) ----------------
    tr = {}
    # (a) two-set style, 3D, hybrid dense, GMM on y fixed mu/w, sigma optimised
    #     (ICP_two_set.py:179-187 GMM; LDDMM hybrid as ICP_atlas's default model)
    g = torch.Generator().manual_seed(7)
    N = 150
    xB = torch.rand(N, 3, generator=g, dtype=f64)
    xA = xB + 0.03 * torch.sin(2 * np.pi * xB[:, [1, 2, 0]]) + 0.005 * torch.randn(N, 3, generator=g, dtype=f64)
    spec64 = {"device": "cpu", "dtype": f64}
    GMMi = G.GaussianMixtureUnif(xB, sigma=0.05, computversion="torch", spec=spec64)
    GMMi.to_optimize = {"mu": False, "sigma": True, "w": False, "eta0": False}
    LMi = L.LDDMMModel(sigma=0.1, D=3, lambd=1e3, version="hybrid", scheme="Euler", nt=10,
                       computversion="torch", spec=spec64)
    PS = P.DiffPSR([[xA]], GMMi, LMi, dataspec=spec64, compspec=spec64)
    PS.printstuff = False
    tr["twoset/xA"] = xA.numpy()
    tr["twoset/xB"] = xB.numpy()
    tr["twoset/FE_init"] = np.array(float(PS.FE))
    for it in range(3):
        PS.GMM_opt(max_iterations=10, tol=1e-3)
        tr[f"twoset/it{it}/FE_gmm"] = np.array(float(PS.FE))
        tr[f"twoset/it{it}/sigma"] = np.array(PS.GMMi[0].sigma)
        PS.Reg_opt(tol=1e-3, nmax=1)
        tr[f"twoset/it{it}/FE_reg"] = np.array(float(PS.FE))
        tr[f"twoset/it{it}/x1"] = PS.x1[0, 0].numpy()
        tr[f"twoset/it{it}/a0"] = PS.a0[0].numpy()
    # (b) atlas style, 2D, 3 frames, GMM fully optimised (ICP_atlas.py:170-298), classic,
    #     grid support (2D only, PSR.py:472-482)
    frames = []
    for k in range(3):
        gk = torch.Generator().manual_seed(100 + k)
        base = torch.rand(60, 2, generator=gk, dtype=f64)
        frames.append([base + 0.02 * torch.sin(2 * np.pi * base[:, [1, 0]]) * (1 + k)])
    GMMa = G.GaussianMixtureUnif(torch.zeros(8, 2, dtype=f64), computversion="torch", spec=spec64)
    LMa = L.LDDMMModel(sigma=0.2, D=2, lambd=500.0, version="classic", scheme="Euler", nt=10,
                       computversion="torch", spec=spec64)
    PA = P.DiffPSR(frames, GMMa, LMa, dataspec=spec64, compspec=spec64)
    PA.printstuff = False
    torch.manual_seed(3)
    PA.reinitialize_GMM()
    PA.set_support_scheme("grid", rho=np.sqrt(2))
    for k in range(3):
        tr[f"atlas/x0_{k}"] = frames[k][0].numpy()
    tr["atlas/mu_init"] = PA.GMMi[0].mu.numpy()
    tr["atlas/sigma_init"] = np.array(PA.GMMi[0].sigma)
    tr["atlas/q0"] = PA.q0[0].numpy()
    tr["atlas/FE_init"] = np.array(float(PA.FE))
    for it in range(2):
        PA.GMM_opt(max_iterations=10, tol=1e-3)
        tr[f"atlas/it{it}/FE_gmm"] = np.array(float(PA.FE))
        tr[f"atlas/it{it}/mu"] = PA.GMMi[0].mu.numpy()
        tr[f"atlas/it{it}/sigma"] = np.array(PA.GMMi[0].sigma)
        PA.Reg_opt(tol=1e-3, nmax=1)
        tr[f"atlas/it{it}/FE_reg"] = np.array(float(PA.FE))
        for k in range(3):
            tr[f"atlas/it{it}/x1_{k}"] = PA.x1[k, 0].numpy()
    np.savez_compressed(os.path.join(HERE, "psr_traces.npz"), **tr)
    for fn in ("reductions", "shoot", "em", "psr_traces"):
        print(fn, os.path.getsize(os.path.join(HERE, fn + ".npz")), "bytes")


def c1_trace():
    """BASELINE configs[0] (diffICP/examples/diffICP_basic.py): one 2D spiral point set of
    500 points (generate_spiral_point_sets, seed 1234 set by that module at import) registered
    to the FIXED generating GMM (mu, w frozen, sigma optimised from 0.1), classic LDDMM
    sigma 0.2 lambda 500 Euler, grid support rho = sqrt(2) (diffICP_basic.py:58-93);
    iteration = GMM_opt() + Reg_opt(tol=1e-5) with the reference defaults
    (diffICP_basic.py:116-119).  The inputs are generated in the reference's float32, the
    trace is recorded in float64."""
    import torch
    K, L, G, P = import_reference()
    from diffICP.examples.generate_spiral_point_sets import generate_spiral_point_sets
    torch.manual_seed(1234)
    x0, GMMg, _ = generate_spiral_point_sets(K=1, Nkbounds=(500, 501), sigma_GMM=0.025,
                                             sigma_LDDMM=0.1, lambda_LDDMM=1e2)
    f64 = torch.float64
    spec64 = {"device": "cpu", "dtype": f64}
    x = x0[0].to(f64)
    tr = {"x0": x.numpy(), "mu": GMMg.mu.to(f64).numpy(), "w": GMMg.w.to(f64).numpy()}
    GM = G.GaussianMixtureUnif(GMMg.mu.to(f64), computversion="torch", spec=spec64)
    GM.w = GMMg.w.to(f64)
    GM.sigma = 0.1
    GM.to_optimize = {"mu": False, "sigma": True, "w": False, "eta0": False}
    LM = L.LDDMMModel(sigma=0.2, D=2, lambd=5e2, version="classic", computversion="torch",
                      scheme="Euler", spec=spec64)
    PS = P.DiffPSR([[x]], GM, LM, dataspec=spec64, compspec=spec64)
    PS.printstuff = False
    PS.set_support_scheme("grid", rho=np.sqrt(2))
    tr["q0"] = PS.q0[0].numpy()
    tr["FE_init"] = np.array(float(PS.FE))
    for it in range(3):
        PS.GMM_opt()
        tr[f"it{it}/FE_gmm"] = np.array(float(PS.FE))
        tr[f"it{it}/sigma"] = np.array(PS.GMMi[0].sigma)
        PS.Reg_opt(tol=1e-5)
        tr[f"it{it}/FE_reg"] = np.array(float(PS.FE))
        tr[f"it{it}/x1"] = PS.x1[0, 0].numpy()
        tr[f"it{it}/a0"] = PS.a0[0].numpy()
        print("C1 it", it, float(PS.FE), PS.GMMi[0].sigma)
    np.savez_compressed(os.path.join(HERE, "c1_trace.npz"), **tr)
    print("c1_trace", os.path.getsize(os.path.join(HERE, "c1_trace.npz")), "bytes")


def decim_cases():
    """decimate (point_sets.py:102-133) on random 2D/3D sets and on a regular grid (many ties
    and near-threshold distances), plus a 2-iteration 3D PSR trace with the "decim" support
    scheme (PSR.py:458-470; custom support -> external-point shooting)."""
    import torch
    K, L, G, P = import_reference()
    import diffICP.tools.point_sets as PS_
    out = {}
    g = torch.Generator().manual_seed(11)
    cases = {"rand2d": (torch.rand(400, 2, generator=g), 0.1),
             "rand3d": (torch.rand(600, 3, generator=g), 0.15),
             "grid2d": (torch.stack(torch.meshgrid(torch.arange(20) * 0.05, torch.arange(20) * 0.05,
                                                   indexing="ij"), -1).reshape(-1, 2).float(), 0.05),
             "dup3d": (torch.rand(50, 3, generator=g).repeat(3, 1), 0.2)}
    for name, (x, R) in cases.items():
        kept, rej = PS_.decimate(x, R)
        out[f"{name}/x"] = x.numpy()
        out[f"{name}/R"] = np.array(R)
        out[f"{name}/kept"] = np.array(kept, dtype=np.int64)
        print("decim", name, len(kept))
    f64 = torch.float64
    spec64 = {"device": "cpu", "dtype": f64}
    gx = torch.Generator().manual_seed(12)
    xB = torch.rand(200, 3, generator=gx, dtype=f64)
    xA = xB + 0.03 * torch.sin(2 * np.pi * xB[:, [2, 0, 1]]) + 0.005 * torch.randn(200, 3, generator=gx, dtype=f64)
    GM = G.GaussianMixtureUnif(xB, sigma=0.05, computversion="torch", spec=spec64)
    GM.to_optimize = {"mu": False, "sigma": True, "w": False, "eta0": False}
    LM = L.LDDMMModel(sigma=0.15, D=3, lambd=1e3, version="hybrid", scheme="Euler", nt=10,
                      computversion="torch", spec=spec64)
    PSR = P.DiffPSR([[xA]], GM, LM, dataspec=spec64, compspec=spec64)
    PSR.printstuff = False
    PSR.set_support_scheme("decim", rho=1.0)
    out["psr/xA"] = xA.numpy()
    out["psr/xB"] = xB.numpy()
    out["psr/q0"] = PSR.q0[0].numpy()
    out["psr/FE_init"] = np.array(float(PSR.FE))
    for it in range(2):
        PSR.GMM_opt(max_iterations=10, tol=1e-3)
        out[f"psr/it{it}/FE_gmm"] = np.array(float(PSR.FE))
        PSR.Reg_opt(tol=1e-3, nmax=1)
        out[f"psr/it{it}/FE_reg"] = np.array(float(PSR.FE))
        out[f"psr/it{it}/x1"] = PSR.x1[0, 0].numpy()
        print("decim psr it", it, float(PSR.FE), PSR.q0[0].shape)
    np.savez_compressed(os.path.join(HERE, "decim.npz"), **out)
    print("decim", os.path.getsize(os.path.join(HERE, "decim.npz")), "bytes")


def psr_std_cases():
    """PSR_standard: data_distance (PSR_standard.py:37-58) with and without
    template weights, and a DiffPSR_std trace (2 frames, 2D, classic LDDMM lambda=2 as
    standard_atlas.py, dense support): E at init, after Reg_opt(nmax=2), after
    Template_opt(nmax=2) -- y0, a0, y1 recorded (float64, torch path)."""
    import torch
    K, L, G, P = import_reference()
    import diffICP.core.PSR_standard as PS
    f64 = torch.float64
    spec64 = {"device": "cpu", "dtype": f64}
    out = {}
    g = torch.Generator().manual_seed(31)
    for D in (2, 3):
        x = torch.rand(70, D, generator=g, dtype=f64)
        y = torch.rand(50, D, generator=g, dtype=f64)
        w = torch.rand(50, generator=g, dtype=f64) / 50
        DK = K.GaussKernel(0.15, D, computversion="torch", spec=spec64)
        out[f"dd{D}/x"], out[f"dd{D}/y"], out[f"dd{D}/w"] = x.numpy(), y.numpy(), w.numpy()
        out[f"dd{D}/L"] = np.array(float(PS.data_distance(DK, x, y)))
        out[f"dd{D}/Lw"] = np.array(float(PS.data_distance(DK, x, y, w)))
    t = torch.linspace(0, 2 * np.pi, 41, dtype=f64)[:-1]
    y0 = torch.stack([0.5 + 0.3 * torch.cos(t), 0.5 + 0.2 * torch.sin(t)], 1)
    xs = []
    for k in range(2):
        tk = torch.rand(60, generator=g, dtype=f64) * 2 * np.pi
        xs.append(torch.stack([0.5 + (0.3 + 0.04 * k) * torch.cos(tk) + 0.03 * torch.sin(3 * tk),
                               0.5 + (0.2 - 0.03 * k) * torch.sin(tk)], 1)
                  + 0.01 * torch.randn(60, 2, generator=g, dtype=f64))
    DK = K.GaussKernel(0.1, 2, computversion="torch", spec=spec64)
    LM = L.LDDMMModel(sigma=0.2, D=2, lambd=2.0, version="classic", scheme="Euler", nt=10,
                      computversion="torch", spec=spec64)
    PSR = PS.DiffPSR_std([[xk] for xk in xs], y0, 0.05, LM, DK, dataspec=spec64, compspec=spec64)
    PSR.printstuff = False
    out["std/y0_init"] = y0.numpy()
    for k in range(2):
        out[f"std/x{k}"] = xs[k].numpy()
    out["std/E_init"] = np.array(float(PSR.E))
    PSR.Reg_opt(nmax=2, tol=1e-3)
    out["std/E_reg"] = np.array(float(PSR.E))
    for k in range(2):
        out[f"std/a0_reg{k}"] = PSR.a0[k].detach().numpy()
        out[f"std/y1_reg{k}"] = PSR.y1[k, 0].detach().numpy()
    PSR.Template_opt(nmax=2, tol=1e-3)
    out["std/E_tpl"] = np.array(float(PSR.E))
    out["std/y0_tpl"] = PSR.y0[0].detach().numpy()
    print("psr_std E", out["std/E_init"], out["std/E_reg"], out["std/E_tpl"])
    np.savez_compressed(os.path.join(HERE, "psr_std.npz"), **out)
    print("psr_std", os.path.getsize(os.path.join(HERE, "psr_std.npz")), "bytes")


def reductions_large():
    """The (M, N) = (1000, 700) per-operator fixtures of SURVEY 8c (D = 3 / sigma 0.05 and
    D = 2 / sigma 1.0), same layout as reductions.npz."""
    import torch
    K, L, G, P = import_reference()
    f64 = torch.float64
    red = {}
    for (M, N, D, sig) in [(1000, 700, 3, 0.05), (1000, 700, 2, 1.0)]:
        key = f"M{M}_N{N}_D{D}_s{sig}"
        g = torch.Generator().manual_seed(M * 7 + N + D)
        x = torch.rand(M, D, generator=g, dtype=f64)
        y = torch.rand(N, D, generator=g, dtype=f64)
        b = torch.randn(N, D, generator=g, dtype=f64)
        c = torch.randn(M, D, generator=g, dtype=f64)
        d = torch.randn(N, generator=g, dtype=f64)
        dm = torch.randn(M, D, generator=g, dtype=f64)
        GK = K.GaussKernel(sig, D, computversion="torch", spec={"device": "cpu", "dtype": f64})
        for nm, t in dict(x=x, y=y, b=b, c=c, d=d, dm=dm).items():
            red[f"{key}/in_{nm}"] = t.numpy()
        red[f"{key}/sigma"] = np.array(sig)
        red[f"{key}/KBase"] = GK.KBase(x, y).numpy()
        red[f"{key}/KRedScal"] = GK.KRedScal(x, y, d).numpy()
        red[f"{key}/KRed"] = GK.KRed(x, y, b).numpy()
        red[f"{key}/GradKRed"] = GK.GradKRed(x, y).numpy()
        red[f"{key}/GradKRed_rev"] = GK.GradKRed_rev(x, y, dm).numpy()
        red[f"{key}/DDKRed"] = GK.DDKRed(x, y, b).numpy()
        red[f"{key}/GenDKRed"] = GK.GenDKRed(x, y, b, c).numpy()
        red[f"{key}/HessKRed"] = GK.HessKRed(x, y, b, c).numpy()
        red[f"{key}/LapKRed"] = GK.LapKRed(x, y).numpy()
        red[f"{key}/GradLapKRed"] = GK.GradLapKRed(x, y).numpy()
    np.savez_compressed(os.path.join(HERE, "reductions_large.npz"), **red)
    print("reductions_large", os.path.getsize(os.path.join(HERE, "reductions_large.npz")), "bytes")


def chui_case():
    """SURVEY 8c fixture "one Chui dataset (ex3) two-set trace": the reference's own data file
    (diffICP/examples/chui-data/demodata_ex3.mat, read as data), DiffPSR with the ICP_two_set
    defaults (ICP_two_set.py:140-207: GMM on xB, sigma 0.1 optimised, mu / w fixed; LDDMM
    sigma 0.2, hybrid (withlogdet, gradcomponent False), Euler nt=10, grid support rho=1;
    lambda fixed at 1e2 since "auto" needs the affine calibration); 4 iterations of
    GMM_opt(10, tol 1e-3) + Reg_opt(nmax=1, tol 1e-3) (ICP_two_set.py:254-282), float64."""
    import scipy.io
    import torch
    K, L, G, P = import_reference()
    f64 = torch.float64
    spec64 = {"device": "cpu", "dtype": f64}
    yo = scipy.io.loadmat(os.path.join(REF, "diffICP/examples/chui-data/demodata_ex3.mat"))
    xA = torch.tensor(yo["x3"], dtype=f64).contiguous()
    xB = torch.tensor(yo["y3"], dtype=f64).contiguous()
    GM = G.GaussianMixtureUnif(xB, sigma=0.1, computversion="torch", spec=spec64)
    GM.to_optimize = {"mu": False, "sigma": True, "w": False, "eta0": False}
    LM = L.LDDMMModel(sigma=0.2, D=2, lambd=1e2, withlogdet=True, gradcomponent=False,
                      computversion="torch", scheme="Euler", nt=10, spec=spec64)
    PSR = P.DiffPSR([[xA]], GM, LM, dataspec=spec64, compspec=spec64)
    PSR.printstuff = False
    PSR.set_support_scheme("grid", rho=1.0)
    out = {"xA": xA.numpy(), "xB": xB.numpy(), "q0": PSR.q0[0].numpy(), "FE_init": np.array(float(PSR.FE))}
    for it in range(4):
        PSR.GMM_opt(max_iterations=10, tol=1e-3)
        out[f"it{it}/FE_gmm"] = np.array(float(PSR.FE))
        out[f"it{it}/sigma"] = np.array(float(PSR.GMMi[0].sigma))
        PSR.Reg_opt(tol=1e-3, nmax=1)
        out[f"it{it}/FE_reg"] = np.array(float(PSR.FE))
        out[f"it{it}/x1"] = PSR.x1[0, 0].numpy()
        out[f"it{it}/a0"] = PSR.a0[0].detach().numpy()
        print("chui it", it, float(PSR.FE), float(PSR.GMMi[0].sigma))
    np.savez_compressed(os.path.join(HERE, "chui_ex3.npz"), **out)
    print("chui", os.path.getsize(os.path.join(HERE, "chui_ex3.npz")), "bytes")


def multi_inputs(case):
    """Inputs of the multi-structure traces (diffICP_full.py:37-97 style): K = 3 frames x S = 3
    structures, each structure a noisy sample of its own curve of C centres, warped per frame
    by a smooth field, one structure of one frame EMPTY (the case diffICP_full.py:94-97 leaves
    commented out).  Seeded, float64; also used by tests/multi_case.py (via the stored arrays)."""
    import torch
    f64 = torch.float64
    D = 2 if case == "m2d" else 3
    g = torch.Generator().manual_seed(41 if D == 2 else 43)
    t = torch.linspace(0, 2 * np.pi, 13, dtype=f64)[:-1]
    curves = [torch.stack((0.5 + 0.4 * (t / 7) * t.cos(), 0.5 + 0.3 * t.sin()), 1),
              torch.stack((1 + 0.4 * t.cos(), 0.5 + 0.4 * t.sin()), 1),
              torch.stack((0.8 + 0.1 * (t - np.pi), -0.06 * (t - np.pi)), 1)]
    if D == 3:
        curves = [torch.cat((c, (0.2 * s + 0.1 * torch.sin(t + s))[:, None]), 1) for s, c in enumerate(curves)]
    sig = [0.025, 0.04, 0.06]
    empty = (1, 2) if D == 2 else (2, 0)
    x = []
    for k in range(3):
        fr = []
        amp = 0.02 * (1 + k)
        for s in range(3):
            if (k, s) == empty:
                fr.append(torch.empty(0, D, dtype=f64))
                continue
            n = int(torch.randint(25, 40, (1,), generator=g))
            lab = torch.randint(0, 12, (n,), generator=g)
            pts = curves[s][lab] + sig[s] * torch.randn(n, D, generator=g, dtype=f64)
            perm = [(d + 1) % D for d in range(D)]
            fr.append((pts + amp * torch.sin(2 * np.pi * pts[:, perm])).contiguous())
        x.append(fr)
    return x


def multi_case():
    """Multi-structure diff-ICP traces (MultiPSR with S > 1: one GMM per structure, targets
    concatenated per frame across structures, per-structure sigma in the quadratic loss,
    PSR.py:197-271, 498-516, 521-569), float64, torch path, dense support, 2 iterations of
    GMM_opt(10, tol 1e-3) + Reg_opt(nmax=1, tol 1e-3):
      m2d: 2D, hybrid LDDMM sigma 0.2 lambda 5e2 (diffICP_full.py:131-134), ONE GMM (C = 12,
           mu / sigma / w optimised) copied per structure, reinitialize_GMM (seed 5);
      m3d: 3D, classic LDDMM sigma 0.25 lambda 1e2, a LIST of GMMs with C = 6 / 10 / 8:
           structure 1 with sigma fixed, structure 2 with the outlier component.
    The randn draws of reinitialize_GMM are recorded (mu_init / sigma_init per structure)."""
    import torch
    K, L, G, P = import_reference()
    f64 = torch.float64
    spec64 = {"device": "cpu", "dtype": f64}
    out = {}
    for case in ("m2d", "m3d"):
        x = multi_inputs(case)
        D = x[0][0].shape[1] if x[0][0].shape[0] else x[0][1].shape[1]
        if case == "m2d":
            GMMi = G.GaussianMixtureUnif(torch.zeros(12, D, dtype=f64), computversion="torch", spec=spec64)
            GMMi.to_optimize = {"mu": True, "sigma": True, "w": True, "eta0": False}
            LM = L.LDDMMModel(sigma=0.2, D=D, lambd=5e2, version="hybrid", scheme="Euler", nt=10,
                              computversion="torch", spec=spec64)
        else:
            GMMi = []
            for s, C in enumerate((6, 10, 8)):
                gm = G.GaussianMixtureUnif(torch.zeros(C, D, dtype=f64), use_outliers=(s == 2),
                                           computversion="torch", spec=spec64)
                gm.to_optimize = {"mu": True, "sigma": s != 1, "w": True, "eta0": True}
                if s == 1:
                    gm.sigma = 0.05
                GMMi.append(gm)
            LM = L.LDDMMModel(sigma=0.25, D=D, lambd=1e2, version="classic", scheme="Euler", nt=10,
                              computversion="torch", spec=spec64)
        PS = P.DiffPSR(x, GMMi, LM, dataspec=spec64, compspec=spec64)
        PS.printstuff = False
        torch.manual_seed(5)
        PS.reinitialize_GMM()
        for k in range(3):
            for s in range(3):
                out[f"{case}/x0_{k}_{s}"] = x[k][s].numpy()
        for s in range(3):
            out[f"{case}/mu_init_{s}"] = PS.GMMi[s].mu.numpy()
            out[f"{case}/sigma_init_{s}"] = np.array(float(PS.GMMi[s].sigma))
        out[f"{case}/FE_init"] = np.array(float(PS.FE))
        for it in range(2):
            PS.GMM_opt(max_iterations=10, tol=1e-3)
            out[f"{case}/it{it}/FE_gmm"] = np.array(float(PS.FE))
            for s in range(3):
                gm = PS.GMMi[s]
                out[f"{case}/it{it}/mu_{s}"] = gm.mu.numpy()
                out[f"{case}/it{it}/w_{s}"] = gm.w.numpy()
                out[f"{case}/it{it}/sigma_{s}"] = np.array(float(gm.sigma))
                out[f"{case}/it{it}/Cfe_{s}"] = np.array(float(PS.Cfe[s]))
                if gm.outliers:
                    out[f"{case}/it{it}/eta0_{s}"] = np.array(float(gm.outliers["eta0"]))
            PS.Reg_opt(tol=1e-3, nmax=1)
            out[f"{case}/it{it}/FE_reg"] = np.array(float(PS.FE))
            out[f"{case}/it{it}/quadloss"] = np.array(PS.quadloss, dtype=np.float64)
            out[f"{case}/it{it}/regloss"] = np.array([float(r) for r in PS.regloss])
            for k in range(3):
                out[f"{case}/it{it}/a0_{k}"] = PS.a0[k].detach().numpy()
                for s in range(3):
                    out[f"{case}/it{it}/x1_{k}_{s}"] = PS.x1[k, s].detach().numpy()
            print("multi", case, "it", it, float(PS.FE), [float(g.sigma) for g in PS.GMMi])
    np.savez_compressed(os.path.join(HERE, "multi.npz"), **out)
    print("multi", os.path.getsize(os.path.join(HERE, "multi.npz")), "bytes")


def psr_std_support_cases():
    """DiffPSR_std with a non-dense support (PSR_standard.py:445-505 set_support_scheme "decim"
    / "grid", rho 1) and with / without template weights (:159-166): 3 frames of 200 2D points
    around a 120-point ellipse template, classic LDDMM sigma 0.2 lambda 2, data kernel 0.1,
    noise 0.05; energies after init and after 2 x (Reg_opt(nmax=2, tol 1e-4) +
    Template_opt(nmax=2, tol 1e-4)).  The inputs are drawn in float32 exactly as
    tests/test_gpu_support.py::test_psr_std_support_schemes draws them; the reference runs in
    float64.  Also records whether the reference itself warns of an energy increase (its
    PSR_standard.py:311-315 check)."""
    import warnings as W
    import torch
    K, L, G, P = import_reference()
    import diffICP.core.PSR_standard as PS
    f64 = torch.float64
    spec64 = {"device": "cpu", "dtype": f64}
    out = {}
    for scheme in ("decim", "grid"):
        for weights in (False, True):
            g = torch.Generator().manual_seed(13)
            t = torch.linspace(0, 2 * np.pi, 121)[:-1]
            y0 = torch.stack([0.5 + 0.3 * torch.cos(t), 0.5 + 0.2 * torch.sin(t)], 1)
            xs = []
            for k in range(3):
                tk = torch.rand(200, generator=g) * 2 * np.pi
                xs.append(torch.stack([0.5 + (0.3 + 0.03 * k) * torch.cos(tk), 0.5 + (0.2 - 0.02 * k) * torch.sin(tk)], 1)
                          + 0.01 * torch.randn(200, 2, generator=g))
            key = f"{scheme}_w{int(weights)}"
            DK = K.GaussKernel(0.1, 2, computversion="torch", spec=spec64)
            LM = L.LDDMMModel(sigma=0.2, D=2, lambd=2.0, version="classic", scheme="Euler", nt=10,
                              computversion="torch", spec=spec64)
            with W.catch_warnings(record=True) as caught:
                W.simplefilter("always")
                PSR = PS.DiffPSR_std([[xk.to(f64)] for xk in xs], y0.to(f64), 0.05, LM, DK,
                                     template_weights=weights, dataspec=spec64, compspec=spec64)
                PSR.printstuff = False
                PSR.set_support_scheme(scheme, rho=1.0)
                Es = [float(PSR.E)]
                for _ in range(2):
                    PSR.Reg_opt(nmax=2, tol=1e-4)
                    Es.append(float(PSR.E))
                    PSR.Template_opt(nmax=2, tol=1e-4)
                    Es.append(float(PSR.E))
            incr = sum("increase in optimization energy" in str(c.message) for c in caught)
            out[f"{key}/E"] = np.array(Es)
            out[f"{key}/n_increase_warnings"] = np.array(incr)
            out[f"{key}/nq0"] = np.array(PSR.q0.shape[0] if hasattr(PSR.q0, "shape") else PSR.q0[0].shape[0])
            print("psr_std_support", key, Es, "increase warnings:", incr)
    np.savez_compressed(os.path.join(HERE, "psr_std_support.npz"), **out)
    print("psr_std_support", os.path.getsize(os.path.join(HERE, "psr_std_support.npz")), "bytes")


if __name__ == "__main__":
    only = sys.argv[2] if sys.argv[1:2] == ["--only"] else None
    if only is None:
        main()
    if only in (None, "c1"):
        c1_trace()
    if only in (None, "decim"):
        decim_cases()
    if only in (None, "psr_std"):
        psr_std_cases()
    if only in (None, "chui"):
        chui_case()
    if only in (None, "red_large"):
        reductions_large()
    if only in (None, "multi"):
        multi_case()
    if only in (None, "psr_std_support"):
        psr_std_support_cases()
