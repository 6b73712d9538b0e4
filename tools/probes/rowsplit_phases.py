"""Per-rank cost of the row split's forward step in column phases (RowSplit.overlap,
core/shooting.split_step_phased: own slice, then the slices before / after) against the
one-pass slice step (dicp_lddmm_euler_step_zs_f32), on one GPU: each rank's slice timed alone
(HIP events, alternating), W = 2, 4, 8 at 100k, and the local phase alone (what the
all-gather of the previous step can hide behind).  The phased step pays when its extra time
is below the all-gather's (~30-100 us for 2.4 MB over xGMI at W = 8).

    SIZES=100000 WORLDS=2,4,8 python tools/probes/rowsplit_phases.py
"""
import json
import os
import sys
import types

import torch

sys.path.insert(0, os.getcwd())
from difficp_amd import _lib  # noqa: E402
from difficp_amd.core.shooting import split_step_phased  # noqa: E402

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


def split_of(rank, world):
    def rows(M):
        p = -(-M // world)
        r0 = min(p * rank, M)
        return r0, min(r0 + p, M) - r0, p
    return types.SimpleNamespace(rank=rank, world=world, rows=rows, overlap=True)


reps = int(os.environ.get("REPS", "20"))
for M in [int(v) for v in os.environ.get("SIZES", "100000").split(",")]:
    g = torch.Generator().manual_seed(M)
    q = torch.rand(M, 3, generator=g).to(dev)
    p = (0.01 * torch.randn(M, 3, generator=g)).to(dev)
    for W in [int(v) for v in os.environ.get("WORLDS", "2,4,8").split(",")]:
        for rank in sorted({0, W // 2, W - 1}):
            sp = split_of(rank, W)
            r0, n, _ = sp.rows(M)
            qo, po, zo = (torch.empty((n, 3), device=dev) for _ in range(3))
            qo2, po2, zo2 = (torch.empty((n, 3), device=dev) for _ in range(3))
            ql, pl = q[r0:r0 + n].clone(), p[r0:r0 + n].clone()
            one = lambda: _lib.euler_step_rows(q, p, r0, n, 0.1, 0.0, 0.1, True, q_out=qo, p_out=po,
                                               zs_out=zo)
            ph = lambda: split_step_phased(sp, q, p, ql, pl, 0.1, 0.0, 0.1, True, qo2, po2, zo2)
            ws = _lib.euler_step_phase_ws(n, M, 3, dev)
            ph0 = lambda: _lib.euler_step_phase(0, ql, pl, q, p, r0, n, 0.1, 0.0, 0.1, qo2, po2,
                                                torch.empty(n, device=dev), zo2, ws=ws)
            a = b = c = 1e9
            for _ in range(3):
                a = min(a, timeit(one, reps))
                b = min(b, timeit(ph, reps))
                c = min(c, timeit(ph0, reps))
            one()
            ph()
            torch.cuda.synchronize()
            err = float(((qo2 - qo).abs().max() / qo.abs().max()).item())
            print(json.dumps({"M": M, "W": W, "rank": rank, "rows": n, "one_pass_ms": round(a, 4),
                              "phased_ms": round(b, 4), "extra_us": round((b - a) * 1e3, 1),
                              "local_phase_ms": round(c, 4),
                              "local_phase_pairs": n * n, "q_rel_diff": err}), flush=True)
