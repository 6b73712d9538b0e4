"""A/B of experiment builds of the native library (make -C diff-icp_amd/csrc variant
NAME=... EXTRA=...): each build is timed in its own subprocess (DICP_LIB_PATH), the
builds are alternated `--passes` times and the per-kernel minimum is reported.

    python tools/ab_libs.py [--M 50000] [--passes 2] base early early_u1 ...
("base" = the default in-tree library.)
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VAR = os.path.join(ROOT, "diff-icp_amd", "variants")

CHILD = r"""
import json, sys, torch
sys.path.insert(0, %r)
from difficp_amd import _lib
import os
for kv in filter(None, os.environ.get("DICP_AB_OPTS", "").split(",")):   # e.g. sym_rp=2
    k, v = kv.split("=")
    _lib.set_option(k, int(v))
M = %d
dev = torch.device("cuda:0")
torch.manual_seed(0)
q = torch.rand(M, 3, device=dev); p = 0.01 * torch.randn(M, 3, device=dev)
ga = torch.randn(M, 3, device=dev); gb = torch.randn(M, 3, device=dev); gd = torch.ones(1, device=dev)
w2 = torch.zeros(M, device=dev); mu2 = (q * q).sum(-1)
zs = torch.empty_like(q)
T2 = _lib.gmm_estep(q, q, w2, mu2, 0.05, 0.0, False)[1]
X4 = torch.rand(640000, 3, device=dev); mu4 = torch.rand(512, 3, device=dev)       # the C4 EM shape
w24 = torch.full((512,), -9.0, device=dev); m24 = (mu4 * mu4).sum(-1)
T24 = _lib.gmm_estep(X4, mu4, w24, m24, 0.05, 0.0, False)[1]
fns = {"fwd": lambda: _lib.ode_self_fwd(q, p, 0.1, 0.0, True),
       "step_zs": lambda: _lib.euler_step(q, p, 0.1, 0.0, 0.1, True, zs_out=zs),
       "adj_zs": lambda: _lib.euler_adjoint_step(q, p, ga, gb, gd, 0.1, 0.0, 0.1, zs=zs),
       "adj_b0": lambda: _lib.euler_adjoint_step(q, p, ga, None, gd, 0.1, 0.0, 0.1, zs=zs),
       "adj_gp": lambda: _lib.euler_adjoint_step(q, p, ga, gb, gd, 0.1, 0.0, 0.1, want_lq=False, zs=zs),
       "bwd": lambda: _lib.ode_self_bwd(q, p, ga, gb, gd, 0.1, 0.0),
       "estep": lambda: _lib.gmm_estep(q, q, w2, mu2, 0.05, 0.0, True),
       "mstep": lambda: _lib.gmm_mstep(q, T2, q, w2, 0.05),
       "estep_c4": lambda: _lib.gmm_estep(X4, mu4, w24, m24, 0.05, 0.0, True),
       "mstep_c4": lambda: _lib.gmm_mstep(X4, T24, mu4, w24, 0.05),
       "kred": lambda: _lib.gauss_red(_lib.KRED, q, q, 0.1, b=p),
       # the exact ICP_two_set model's forward (eta = 1 / lambda != 0, logdet)
       "fwd_eta": lambda: _lib.ode_self_fwd(q, p, 0.1, 0.01, True),
       "step_eta": lambda: _lib.euler_step(q, p, 0.1, 0.01, 0.1, True)}
only = [k for k in os.environ.get("DICP_AB_ONLY", "").split(",") if k]
if only:
    fns = {k: v for k, v in fns.items() if k in only}
out = {}
for k, fn in fns.items():
    fn(); fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); fn(); fn(); e1.record(); e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / 3)
    out[k] = best
print(json.dumps(out))
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=50000)
    ap.add_argument("--passes", type=int, default=2)
    ap.add_argument("names", nargs="+")
    a = ap.parse_args()
    res = {}
    for _ in range(a.passes):
        for name in a.names:
            env = dict(os.environ)
            if name != "base":
                env["DICP_LIB_PATH"] = os.path.join(VAR, f"libdifficp_hip_{name}.so")
            r = subprocess.run([sys.executable, "-c", CHILD % (ROOT, a.M)], env=env,
                               capture_output=True, text=True, timeout=300)
            if r.returncode != 0:
                res.setdefault(name, {})["error"] = r.stderr[-500:]
                continue
            t = json.loads(r.stdout.strip().splitlines()[-1])
            d = res.setdefault(name, {})
            for k, v in t.items():
                d[k] = round(min(d.get(k, 1e9), v), 4)
    print(json.dumps({"M": a.M, "ab_libs": res}))


if __name__ == "__main__":
    main()
