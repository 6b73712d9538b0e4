"""A/B of the packed eta = 0 symmetric VJP with 4 rows per lane (256-point groups,
dicp_set_option "sym_rp" 2) against 2 rows ("sym_rp" 1): agreement and time per launch of
every variant the shooting's backward runs -- the adjoint step reusing the divergence rows
(adj_zs), its zero-momentum-cotangent first step (adj_b0), the gp-only last step (adj_gp),
the plain VJP with the divergence pair terms (bwd) -- and of the row-split pair-subset parts
(part W: the slowest of the W parts), alternating in one process.

    SIZES=50000,70000,90000,100000,200000 PARTS=2,4,8 python tools/probes/sym_rp_ab.py
One JSON line per size (and per part count).  The automatic rule (sym_rp 0) is reported as
"auto_rows" = which form the library picks at that size.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from difficp_amd import _lib  # noqa: E402

dev = torch.device("cuda:0")
st = torch.cuda.current_stream()


def timeit(fn, reps):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        fn()
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def ab(fns, M, passes=3):
    row = {}
    for name, fn in fns.items():
        outs, best = {}, {}
        for v in (1, 2):
            _lib.set_option("sym_rp", v)
            outs[v] = [t.clone() for t in fn() if isinstance(t, torch.Tensor)]
        err = max(float((a - b).norm() / b.norm()) for a, b in zip(outs[2], outs[1]))
        reps = max(2, int(2e10 / (M * M)))
        for _ in range(passes):
            for v in (1, 2):
                _lib.set_option("sym_rp", v)
                best[v] = min(best.get(v, 1e9), timeit(fn, reps))
        row[name] = {"rows2_ms": round(best[1], 4), "rows4_ms": round(best[2], 4),
                     "speedup": round(best[1] / best[2], 4), "rel_err": err}
    _lib.set_option("sym_rp", 0)
    return row


def main():
    sizes = [int(v) for v in os.environ.get("SIZES", "50000,100000").split(",")]
    parts = [int(v) for v in os.environ.get("PARTS", "").split(",") if v]
    for M in sizes:
        g = torch.Generator().manual_seed(M)
        q = torch.rand(M, 3, generator=g).to(dev)
        p = (0.01 * torch.randn(M, 3, generator=g)).to(dev)
        ga = torch.randn(M, 3, generator=g).to(dev)
        gb = torch.randn(M, 3, generator=g).to(dev)
        gd = torch.ones(1, device=dev)
        zs = torch.empty_like(q)
        _lib.euler_step(q, p, 0.1, 0.0, 0.1, True, zs_out=zs)
        fns = {"adj_zs": lambda: _lib.euler_adjoint_step(q, p, ga, gb, gd, 0.1, 0.0, 0.1, zs=zs),
               "adj_b0": lambda: _lib.euler_adjoint_step(q, p, ga, None, gd, 0.1, 0.0, 0.1, zs=zs),
               "adj_gp": lambda: _lib.euler_adjoint_step(q, p, ga, gb, gd, 0.1, 0.0, 0.1, want_lq=False,
                                                         zs=zs),
               "bwd": lambda: _lib.ode_self_bwd(q, p, ga, gb, gd, 0.1, 0.0)}
        row = {"M": M, **ab(fns, M)}
        print(json.dumps(row), flush=True)
        for W in parts:
            # every part of a W-way split; the row split waits for the slowest one
            def part_fn(k, W=W):
                return lambda: _lib.ode_self_bwd_part(q, p, ga, gb, gd, 0.1, 0.0, k, W, zs=zs[:0])
            fns = {f"part{k}of{W}": part_fn(k) for k in range(W)}
            r = ab(fns, M // max(1, int(W ** 0.5)), passes=2)
            slow2 = max(v["rows2_ms"] for v in r.values())
            slow4 = max(v["rows4_ms"] for v in r.values())
            print(json.dumps({"M": M, "parts": W, "slowest_rows2_ms": slow2, "slowest_rows4_ms": slow4,
                              "speedup": round(slow2 / slow4, 4),
                              "max_rel_err": max(v["rel_err"] for v in r.values())}), flush=True)


if __name__ == "__main__":
    main()
