"""Time the hot shooting kernels of libraries built from earlier commits against HEAD's, on one
box (VERDICT r03 "find the VJP regression").

    python tools/bisect_vjp.py build  c092ecc 73d3f8c~1 73d3f8c d93a18f~1 d93a18f HEAD
        (build container: `git archive` of diff-icp_amd/csrc + include at each commit into
        /tmp/dicp_bisect/<name>/, make, copy the library to diff-icp_amd/variants/
        libdifficp_hip_bisect_<name>.so -- the variants travel to the GPU box with the tree)
    python tools/bisect_vjp.py time [--M 100000] [--passes 3] c092ecc 73d3f8c~1 ...
        (GPU box: each library in its own subprocess, alternated `passes` times; per kernel
        the minimum over passes of the best-of-5 mean of 3 launches, HIP events)

The child binds the C-ABI directly with ctypes (the entry points timed here kept their
signatures since round 2), so it does not depend on HEAD's Python binding knowing an old
library's options.  Kernels: the fused Euler step writing divergence rows (step_zs) and the
three adjoint-step variants the shooting's backward launches (adj_zs: full VJP reusing the
divergence rows; adj_b0: zero momentum cotangent; adj_gp: no gq half).
"""
import argparse
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VAR = os.path.join(ROOT, "diff-icp_amd", "variants")


def _tag(rev):
    return rev.replace("~", "m").replace("^", "p")


def build(revs):
    os.makedirs(VAR, exist_ok=True)
    for rev in revs:
        name = _tag(rev)
        d = os.path.join("/tmp/dicp_bisect", name)
        shutil.rmtree(d, ignore_errors=True)
        os.makedirs(d)
        arch = subprocess.run(["git", "-C", ROOT, "archive", rev, "diff-icp_amd/csrc", "include"],
                              check=True, capture_output=True).stdout
        subprocess.run(["tar", "-x", "-C", d], input=arch, check=True)
        csrc = os.path.join(d, "diff-icp_amd", "csrc")
        subprocess.run(["make", "-C", csrc, "-j8", "../libdifficp_hip.so"], check=True,
                       stdout=subprocess.DEVNULL)
        dst = os.path.join(VAR, f"libdifficp_hip_bisect_{name}.so")
        shutil.copy(os.path.join(d, "diff-icp_amd", "libdifficp_hip.so"), dst)
        print(rev, "->", dst)


CHILD = r"""
import ctypes, json, sys, torch
lib = ctypes.CDLL(sys.argv[1])
M = int(sys.argv[2])
P, I64, INT, DBL, SZ = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_double, ctypes.c_size_t
lib.dicp_workspace_bytes.argtypes = [INT, I64, I64, INT]; lib.dicp_workspace_bytes.restype = SZ
lib.dicp_lddmm_euler_step_zs_f32.argtypes = [P, P, I64, I64, I64, INT, DBL, DBL, DBL, P, P, P, P, P, P, SZ, P]
lib.dicp_lddmm_euler_adjoint_step_zs_f32.argtypes = [P, P, P, P, P, I64, INT, DBL, DBL, DBL, P, P, P, P, P, P, SZ, P]
lib.dicp_version.restype = ctypes.c_char_p
dev = torch.device("cuda:0")
torch.manual_seed(0)
D = 3
q = torch.rand(M, D, device=dev); p = 0.01 * torch.randn(M, D, device=dev)
lq = torch.randn(M, D, device=dev); lp = torch.randn(M, D, device=dev); gd = torch.ones(1, device=dev)
qn = torch.empty_like(q); pn = torch.empty_like(q); zs = torch.empty_like(q)
lqn = torch.empty_like(q); lpn = torch.empty_like(q)
def ws(kind):
    nb = lib.dicp_workspace_bytes(kind, M, M, D)
    return torch.empty(max(nb, 16), dtype=torch.uint8, device=dev), nb
wf, nf = ws(1); wb, nb = ws(2)
st = torch.cuda.current_stream(dev).cuda_stream
ptr = lambda t: None if t is None else t.data_ptr()
def chk(rc):
    assert rc == 0, rc
fns = {
  "step_zs": lambda: chk(lib.dicp_lddmm_euler_step_zs_f32(ptr(q), ptr(p), M, 0, M, D, 0.1, 0.0, 0.1, None,
                                                           ptr(qn), ptr(pn), None, ptr(zs), ptr(wf), nf, st)),
  "adj_zs": lambda: chk(lib.dicp_lddmm_euler_adjoint_step_zs_f32(ptr(q), ptr(p), ptr(lq), ptr(lp), ptr(gd), M, D,
                        0.1, 0.0, 0.1, None, None, ptr(zs), ptr(lqn), ptr(lpn), ptr(wb), nb, st)),
  "adj_b0": lambda: chk(lib.dicp_lddmm_euler_adjoint_step_zs_f32(ptr(q), ptr(p), ptr(lq), None, ptr(gd), M, D,
                        0.1, 0.0, 0.1, None, None, ptr(zs), ptr(lqn), ptr(lpn), ptr(wb), nb, st)),
  "adj_gp": lambda: chk(lib.dicp_lddmm_euler_adjoint_step_zs_f32(ptr(q), ptr(p), ptr(lq), ptr(lp), ptr(gd), M, D,
                        0.1, 0.0, 0.1, None, None, ptr(zs), None, ptr(lpn), ptr(wb), nb, st)),
}
out = {"version": lib.dicp_version().decode()}
fns["step_zs"]()
for k, fn in fns.items():
    fn(); fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); fn(); fn(); e1.record(); e1.synchronize()
        best = min(best, e0.elapsed_time(e1) / 3)
    out[k] = best
out["lpn_sum"] = float(lpn.double().sum())
print(json.dumps(out))
"""


def time_libs(revs, M, passes):
    res = {}
    for _ in range(passes):
        for rev in revs:
            path = os.path.join(VAR, f"libdifficp_hip_bisect_{_tag(rev)}.so")
            r = subprocess.run([sys.executable, "-c", CHILD, path, str(M)], capture_output=True,
                               text=True, timeout=300)
            if r.returncode != 0:
                print(rev, "FAILED", r.stderr[-2000:], file=sys.stderr)
                raise SystemExit(1)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            cur = res.setdefault(rev, {})
            for k, v in d.items():
                if isinstance(v, float) and k != "lpn_sum":
                    cur[k] = min(cur.get(k, 1e9), v)
                else:
                    cur[k] = v
            print(json.dumps({"rev": rev, **d}), flush=True)
    print(json.dumps({"M": M, "passes": passes, "min_ms": res}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("mode", choices=["build", "time"])
    ap.add_argument("--M", type=int, default=100000)
    ap.add_argument("--passes", type=int, default=3)
    ap.add_argument("revs", nargs="+")
    a = ap.parse_args()
    if a.mode == "build":
        build(a.revs)
    else:
        time_libs(a.revs, a.M, a.passes)


if __name__ == "__main__":
    main()
