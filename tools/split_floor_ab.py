"""Column-split count of the packed forward: the default S = ceil(rounds * capacity / row
blocks) can overshoot a whole number of workgroup rounds by a few workgroups (a nearly empty
extra round); S_floor = floor(rounds * capacity / row blocks) does not.  A/B of the two by
dicp_set_option("force_splits"), alternating, HIP events, on row slices of the sizes the
bench runs (full passes, row-split parts at W = 2..8, atlas frames)."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from difficp_amd import _lib  # noqa: E402

CAP = 1280  # 256 CUs x 5 workgroups (rowred_pk_kernel, 90 VGPRs)


def tm(fn, reps=5):
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        fn()
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    dev = torch.device("cuda:0")
    out = []
    for N, rows in ((100000, 100000), (100000, 50000), (100000, 25000), (100000, 12500),
                    (200000, 200000), (200000, 25000), (50000, 50000), (50000, 6250),
                    (30000, 30000), (20000, 20000), (120000, 120000)):
        g = torch.Generator().manual_seed(N)
        q = torch.rand(N, 3, generator=g).to(dev)
        p = (0.05 * torch.randn(N, 3, generator=g)).to(dev)
        zs = torch.empty(rows, 3, device=dev)
        bx = math.ceil(rows / 512)
        rounds = min(max(rows // 16000, 1), 16)
        s_def = _lib.num_splits(_lib.WS_ODE_SELF_FWD, rows, N) if rows == N else None
        s_floor = max(1, (rounds * CAP) // bx)
        fn = lambda: _lib.euler_step_rows(q, p, 0, rows, 0.1, 0.0, 0.1, True, zs_out=zs)
        fn()
        res = {"def": [], "floor": []}
        for _ in range(4):
            _lib.set_option("force_splits", 0)
            res["def"].append(tm(fn))
            _lib.set_option("force_splits", s_floor)
            res["floor"].append(tm(fn))
        _lib.set_option("force_splits", 0)
        rec = {"N": N, "rows": rows, "bx": bx, "rounds": rounds, "S_floor": s_floor,
               "S_ceil": math.ceil(rounds * CAP / bx), "def_ms": round(min(res["def"]), 4),
               "floor_ms": round(min(res["floor"]), 4),
               "floor_over_def": round(min(res["floor"]) / min(res["def"]), 4)}
        print(json.dumps(rec), flush=True)
        out.append(rec)


if __name__ == "__main__":
    main()
