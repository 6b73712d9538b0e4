"""A/B of experiment builds of the centred reductions (make -C diff-icp_amd/csrc variant
NAME=... EXTRA=...): KRed / GradKRed at M = N (x = y, the north_star's kernel sum) and the
external-point forward (eta = 0 and eta != 0, with the divergence row), each build in its own
subprocess (DICP_LIB_PATH), builds alternated `--passes` times, minimum per op reported;
outputs of every build are compared bitwise with the first build's.

    python tools/cx_pk_ab.py [--M 100000] [--passes 2] [--set cx|fwd] [--out f.json] base cxpk0 ...
(--set fwd: the fused self forward -- Euler step with divergence rows, without mG, eta != 0,
with the Hamiltonian rows -- instead of the centred reductions)
("base" = the default in-tree library.)
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VAR = os.path.join(ROOT, "diff-icp_amd", "variants")

CHILD = r"""
import hashlib, json, sys, torch
sys.path.insert(0, %r)
from difficp_amd import _lib as L
M = %d
dev = torch.device("cuda:0")
g = torch.Generator().manual_seed(M)
x = torch.rand(M, 3, generator=g).to(dev)
b = (0.01 * torch.randn(M, 3, generator=g)).to(dev)
xe = torch.rand(M, 3, generator=g).to(dev)
zs = torch.empty_like(x)
if %r == "fwd":   # the fused self forward (packed.hpp) in the variants the shooting runs
    fns = {"step_zs": lambda: L.euler_step(x, b, 0.1, 0.0, 0.1, True, zs_out=zs),
           "step_nog": lambda: L.euler_step(x, b, 0.1, 0.0, 0.1, True, want_p=False),
           "fwd_eta": lambda: L.ode_self_fwd(x, b, 0.1, 1e-3, True),
           "fwd_h": lambda: L.ode_self_fwd(x, b, 0.1, 0.0, True, want_h=True)}
else:
    L.set_option("red_alg", 2)
    fns = {"KRed": lambda: L.gauss_red(L.KRED, x, x, 0.1, b=b),
           "GradKRed": lambda: L.gauss_red(L.GRADK, x, x, 0.1),
           "KBase": lambda: L.gauss_red(L.KBASE, x, x, 0.1),
           "ext_fwd_eta0": lambda: L.ode_ext_fwd(xe, x, b, 0.1, 0.0, True),
           "ext_fwd_eta": lambda: L.ode_ext_fwd(xe, x, b, 0.1, 1e-3, True)}
out, digest = {}, {}
for k, fn in fns.items():
    r = fn()
    torch.cuda.synchronize()
    h = hashlib.sha1()
    for t in (r if isinstance(r, (tuple, list)) else (r,)):
        if t is not None:
            h.update(t.detach().cpu().numpy().tobytes())
    digest[k] = h.hexdigest()[:16]
    best = 1e9
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); fn(); fn(); e1.record(); e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / 3)
    out[k] = best
print(json.dumps({"ms": out, "digest": digest}))
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=100000)
    ap.add_argument("--passes", type=int, default=2)
    ap.add_argument("--out", default=None)
    ap.add_argument("--set", default="cx", choices=["cx", "fwd"])
    ap.add_argument("names", nargs="+")
    a = ap.parse_args()
    res, dig = {}, {}
    for _ in range(a.passes):
        for name in a.names:
            env = dict(os.environ)
            if name != "base":
                env["DICP_LIB_PATH"] = os.path.join(VAR, f"libdifficp_hip_{name}.so")
            r = subprocess.run([sys.executable, "-c", CHILD % (ROOT, a.M, a.set)], env=env,
                               capture_output=True, text=True, timeout=300)
            if r.returncode != 0:
                res.setdefault(name, {})["error"] = r.stderr[-800:]
                print(name, r.stderr[-800:], flush=True)
                continue
            t = json.loads(r.stdout.strip().splitlines()[-1])
            d = res.setdefault(name, {})
            for k, v in t["ms"].items():
                d[k] = round(min(d.get(k, 1e9), v), 4)
            dig[name] = t["digest"]
            print(name, json.dumps(t), flush=True)
    ref = dig.get(a.names[0], {})
    same = {n: {k: v == ref.get(k) for k, v in dg.items()} for n, dg in dig.items()}
    line = {"M": a.M, "ms": res, "bitwise_equal_to_" + a.names[0]: same}
    print(json.dumps(line))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(line, f, indent=1)


if __name__ == "__main__":
    main()
