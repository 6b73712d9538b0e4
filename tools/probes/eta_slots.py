"""Which workspace slots of the packed eta != 0 VJP (lddmm_sym.hpp launch_sym_bwd_eta) does the
merge read without the pair kernel having written them?  Calls the adjoint step through the
C-ABI with a NaN-filled workspace of its own and lists, per slot, the rows whose slot entries
the merge reads (sym_nslots) but are still NaN.  Geometry as sym_geom at these sizes (L = 1).

    python tools/probes/eta_slots.py > out.jsonl
"""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from difficp_amd import _lib  # noqa: E402

G, Q4 = 128, 4


def main():
    dev = torch.device("cuda:0")
    L_ = _lib.lib()
    for M, D in ((700, 2), (3333, 2), (9000, 3), (257, 2), (1025, 3), (2000, 3)):
        g = torch.Generator().manual_seed(M)
        q = torch.rand(M, D, generator=g).to(dev)
        p = (0.05 * torch.randn(M, D, generator=g)).to(dev)
        lq = torch.randn(M, D, generator=g).to(dev)
        lp0 = torch.randn(M, D, generator=g).to(dev)
        gdiv = torch.ones(1, device=dev)
        nG = math.ceil(M / G)
        nQ = math.ceil(nG / Q4)
        Lg = 1
        for b0 in (False, True):
            for want_lq in (True, False):
                W = 2 * D if want_lq else D
                nb = int(L_.dicp_workspace_bytes(_lib.WS_ODE_SELF_BWD, M, M, D))
                ws = torch.full((nb // 4,), float("nan"), device=dev)
                lqn = torch.empty_like(q) if want_lq else None
                lpn = torch.empty_like(q)
                rc = L_.dicp_lddmm_euler_adjoint_step_zs_f32(
                    q.data_ptr(), p.data_ptr(), lq.data_ptr(), None if b0 else lp0.data_ptr(), gdiv.data_ptr(),
                    M, D, 0.1, 0.1, 0.1, None, None, None, None if lqn is None else lqn.data_ptr(),
                    lpn.data_ptr(), ws.data_ptr(), nb, _lib._stream(dev))
                torch.cuda.synchronize()
                slab = ws[: (nQ + 1 + nG) * M * W].view(nQ + 1 + nG, M, W).cpu()
                bad = {}
                for T in range(nG):
                    QT = T // Q4
                    ns = QT + 1 + math.ceil((nG - Q4 * QT) / Lg)
                    r0, r1 = T * G, min(M, (T + 1) * G)
                    for t in range(ns):
                        blk = slab[t, r0:r1]
                        nan_rows = torch.isnan(blk).any(1).nonzero().flatten()
                        if nan_rows.numel():
                            bad.setdefault(str(t), []).append([T, int(nan_rows[0]) + r0, int(nan_rows[-1]) + r0,
                                                               int(nan_rows.numel())])
                print(json.dumps({"M": M, "D": D, "b0": b0, "gq": want_lq, "rc": rc, "nG": nG, "nQ": nQ,
                                  "out_finite": bool(torch.isfinite(lpn).all()) and (lqn is None or bool(torch.isfinite(lqn).all())),
                                  "unwritten_read": bad}), flush=True)


if __name__ == "__main__":
    main()
