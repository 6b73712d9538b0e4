"""The column groups per workgroup (dicp_set_option "sym_L") of the 4-row symmetric VJP at the
sizes where it runs: automatic vs forced 2 / 4 / 8, adjoint step with divergence rows and the
gp-only step, alternating in one process (HIP events).

    SIZES=100000,200000 [REPS=10 ROUNDS=5 LS=0,2,4,8 KIND=vjp|fwd|both] python tools/probes/sym_L_rows4.py

(KIND=fwd: the symmetric 4-row forward's Euler step with divergence rows, which the same
option steers; SYM_RP=1/2 forces 2 / 4 rows per lane for the VJP; FWD_ALG=5/6 the symmetric
4-row / the ordered forward.)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from difficp_amd import _lib  # noqa: E402

dev = torch.device("cuda:0")
st = torch.cuda.current_stream()
if os.environ.get("SYM_RP"):     # force 2 (1) or 4 (2) rows per lane
    _lib.set_option("sym_rp", int(os.environ["SYM_RP"]))
if os.environ.get("FWD_ALG"):    # 5 = symmetric 4-row forward, 6 = ordered
    _lib.set_option("fwd_alg", int(os.environ["FWD_ALG"]))


def timeit(fn, reps):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        fn()
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


for M in [int(v) for v in os.environ.get("SIZES", "100000,200000").split(",")]:
    g = torch.Generator().manual_seed(M)
    q = torch.rand(M, 3, generator=g).to(dev)
    p = (0.01 * torch.randn(M, 3, generator=g)).to(dev)
    ga = torch.randn(M, 3, generator=g).to(dev)
    gb = torch.randn(M, 3, generator=g).to(dev)
    gd = torch.ones(1, device=dev)
    zs = torch.empty_like(q)
    _lib.euler_step(q, p, 0.1, 0.0, 0.1, True, zs_out=zs)
    fns = {"adj_zs": lambda: _lib.euler_adjoint_step(q, p, ga, gb, gd, 0.1, 0.0, 0.1, zs=zs),
           "adj_gp": lambda: _lib.euler_adjoint_step(q, p, ga, gb, gd, 0.1, 0.0, 0.1, want_lq=False, zs=zs),
           "adj_b0": lambda: _lib.euler_adjoint_step(q, p, ga, None, gd, 0.1, 0.0, 0.1, zs=zs)}
    qn, pn, zs2 = torch.empty_like(q), torch.empty_like(q), torch.empty_like(q)
    fwd = {"step_zs": lambda: _lib.euler_step(q, p, 0.1, 0.0, 0.1, True, q_out=qn, p_out=pn, zs_out=zs2)}
    kind = os.environ.get("KIND", "vjp")
    fns = {"vjp": fns, "fwd": fwd, "both": {**fns, **fwd}}[kind]
    reps = int(os.environ.get("REPS", "0")) or max(2, int(2e10 / (M * M)))
    rounds = int(os.environ.get("ROUNDS", "3"))
    Ls = [int(v) for v in os.environ.get("LS", "0,2,4,8").split(",")]
    row = {"M": M}
    for name, fn in fns.items():
        best = {}
        for _ in range(rounds):
            for L in Ls:
                _lib.set_option("sym_L", L)
                best[L] = min(best.get(L, 1e9), timeit(fn, reps))
        _lib.set_option("sym_L", 0)
        row[name] = {f"L{L}" if L else "auto": round(v, 4) for L, v in best.items()}
    print(json.dumps(row), flush=True)
