"""Cross-timing of the CPU baseline restatement against the reference's own CPU path (build
container only: imports the reference from /root/reference with the SURVEY App. C recipe of
tests/golden/make_golden.py; the GPU box never runs this).

SURVEY 8(d): the CPU baseline that bench.py reports on the GPU box is the chunked torch
restatement (oracle/torch_ref.py, the reference's torch arithmetic) -- the reference itself
cannot travel.  This script times both on the same operators and sizes (N <= 4000, float32,
all host threads) and records the ratio restatement / reference, which must stay within
1.5x for the restatement to stand in for the reference's CPU path:

  * KRed, GenDKRed (kernel.py:186-187, :202-203, torch versions);
  * one hybrid ODE evaluation (LDDMM.py:176-227: KRed + GenDKRed + GradKRed) and its
    torch-autograd backward (the L.backward() of optim.py:46, per ODE evaluation);
  * one EM step (GMM.py:236-325, torch path) at N points x C = N/4 components.

    python tools/cpu_crosstime.py [--out profiles/r03_cpu_crosstime.json]
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def best_of(f, reps=3):
    f()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    return min(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r03_cpu_crosstime.json"))
    ap.add_argument("--sizes", default="1000,2000,4000")
    args = ap.parse_args()
    import torch
    from make_golden import import_reference
    from oracle import torch_ref as R
    K, L, G, _ = import_reference()
    threads = os.cpu_count() or 1
    torch.set_num_threads(threads)
    spec = {"device": "cpu", "dtype": torch.float32}
    sig = 0.1
    rows = []
    for N in (int(s) for s in args.sizes.split(",")):
        g = torch.Generator().manual_seed(N)
        q = torch.rand(N, 3, generator=g)
        p = 0.01 * torch.randn(N, 3, generator=g)
        a = torch.randn(N, 3, generator=g)
        b = torch.randn(N, 3, generator=g)
        GK = K.GaussKernel(sig, 3, computversion="torch", spec=spec)
        LM = L.LDDMMModel(sigma=sig, D=3, lambd=1e3, spec=spec, version="hybrid", computversion="torch",
                          scheme="Euler", nt=10)
        m = R.LDDMM(sig, 3, 1e3, False, True)
        c0 = torch.zeros(1)

        def ode_bwd(fode):
            qq = q.clone().requires_grad_(True)
            pp = p.clone().requires_grad_(True)
            v, mG, dc = fode(qq, pp, c0)
            torch.autograd.grad((a * v).sum() + (b * mG).sum() + dc.sum(), (qq, pp))

        C = N // 4
        X = torch.rand(N, 3, generator=g)
        mu = torch.rand(C, 3, generator=g)
        GM = G.GaussianMixtureUnif(mu, sigma=0.05, spec=spec, computversion="torch")
        opt = {"mu": True, "w": True, "sigma": True, "eta0": False}
        GM.to_optimize = dict(opt)
        w0 = torch.zeros(C)

        def em_ref():
            GM.mu, GM.w, GM.sigma = mu.clone(), w0.clone(), 0.05
            GM.EM_step(X)

        ops = {
            "KRed": (lambda: GK.KRed(q, q, p), lambda: R.KRed(q, q, p, sig)),
            "GenDKRed": (lambda: GK.GenDKRed(q, q, p, p), lambda: R.GenDKRed(q, q, p, p, sig)),
            "ODE_fwd": (lambda: LM.ODE(q, p, c0), lambda: m.ODE(q, p, c0)),
            "ODE_fwd_bwd": (lambda: ode_bwd(LM.ODE), lambda: ode_bwd(m.ODE)),
            "EM_step": (em_ref, lambda: R.em_step(X, mu, w0, 0.05, opt)),
        }
        for name, (fr, fo) in ops.items():
            tr = best_of(fr)
            to = best_of(fo)
            pairs = N * (C if name == "EM_step" else N)
            rows.append({"op": name, "N": N, "pairs": pairs, "reference_s": round(tr, 5),
                         "restatement_s": round(to, 5), "ratio_restatement_over_reference": round(to / tr, 3),
                         "reference_Gpair_per_s": round(pairs / tr / 1e9, 4)})
            print(json.dumps(rows[-1]), flush=True)
    worst = max(max(r["ratio_restatement_over_reference"], 1 / r["ratio_restatement_over_reference"]) for r in rows)
    out = {"what": "CPU baseline restatement (oracle/torch_ref.py) vs the reference's torch CPU path, "
                   "imported from /root/reference (SURVEY App. C recipe), float32, best of 3",
           "threads": threads, "host": "build container (8-core guest)", "worst_ratio": round(worst, 3),
           "within_1p5x": worst <= 1.5, "rows": rows}
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print(f"worst ratio {worst:.3f} -> {args.out}")


if __name__ == "__main__":
    main()
