"""A/B of the divergence-row reuse at the bench's size: the adjoint step with and without the
forward's zs rows (and the forward with and without writing them), alternated in one process,
HIP events on the launch stream.  Prints one JSON object.

    python tools/zs_ab.py [--M 100000] [--reps 10]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from difficp_amd import _lib as L  # noqa: E402


def timed(fn, reps):
    st = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        fn()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=100000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    M, sig, dt = a.M, 0.1, 0.1
    q = torch.rand(M, 3, device=dev, generator=g)
    p = 0.01 * torch.randn(M, 3, device=dev, generator=g)
    lq = torch.randn(M, 3, device=dev, generator=g)
    lp = torch.randn(M, 3, device=dev, generator=g)
    gd = torch.full((1,), 0.3, device=dev)
    zs = torch.empty(M, 3, device=dev)
    qo, po, go = torch.empty_like(q), torch.empty_like(q), torch.empty(M, device=dev)
    L.euler_step(q, p, sig, 0.0, dt, True, zs_out=zs)
    cases = {
        "fwd": lambda: L.euler_step(q, p, sig, 0.0, dt, True, q_out=qo, p_out=po, g_out=go),
        "fwd_zs": lambda: L.euler_step(q, p, sig, 0.0, dt, True, q_out=qo, p_out=po, g_out=go, zs_out=zs),
        "bwd": lambda: L.euler_adjoint_step(q, p, lq, lp, gd, sig, 0.0, dt),
        "bwd_zs": lambda: L.euler_adjoint_step(q, p, lq, lp, gd, sig, 0.0, dt, zs=zs),
        "bwd_b0": lambda: L.euler_adjoint_step(q, p, lq, None, gd, sig, 0.0, dt),
        "bwd_b0_zs": lambda: L.euler_adjoint_step(q, p, lq, None, gd, sig, 0.0, dt, zs=zs),
        "bwd_gp": lambda: L.euler_adjoint_step(q, p, lq, lp, gd, sig, 0.0, dt, want_lq=False),
        "bwd_gp_zs": lambda: L.euler_adjoint_step(q, p, lq, lp, gd, sig, 0.0, dt, want_lq=False, zs=zs),
    }
    res = {k: [] for k in cases}
    for _ in range(a.rounds):
        for k, fn in cases.items():
            res[k].append(timed(fn, a.reps))
            print(f"{k}: {res[k][-1]:.3f} ms", file=sys.stderr, flush=True)
    out = {k: min(v) for k, v in res.items()}
    out["M"] = M
    out["speedup_bwd"] = out["bwd"] / out["bwd_zs"]
    out["speedup_bwd_b0"] = out["bwd_b0"] / out["bwd_b0_zs"]
    out["speedup_bwd_gp"] = out["bwd_gp"] / out["bwd_gp_zs"]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
