"""Precision probe of the matrix-core forward (fwd_alg 3) against float64 sums on sampled
rows, next to the packed VALU forward (fwd_alg 2): relative errors of v, mG and the
divergence rows g for clouds of various densities, with the MFMA branch forced for every
workgroup (mfma_rmax_x100 = 100000) and at the default spread threshold.  Prints one line per
configuration with the workgroups' row spread (scaled units) -- the data behind the default
threshold."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from difficp_amd import _lib  # noqa: E402
from difficp_amd.core.shooting import spatial_order  # noqa: E402


def ref_rows(q, p, sig, rows):
    qf, pf = q.double(), p.double()
    z = qf[rows][:, None, :] - qf[None, :, :]
    K = torch.exp(-(z ** 2).sum(-1) / (2 * sig ** 2))
    V = K @ pf
    pp = pf[rows] @ pf.t()
    mG = (1 / sig ** 2) * ((K * pp)[:, :, None] * z).sum(1)
    Z = -(1 / sig ** 2) * (K[:, :, None] * z).sum(1)
    return V, mG, (pf[rows] * Z).sum(1)


def rel(a, b):
    return float((a.double() - b).norm() / b.norm().clamp_min(1e-300))


def main():
    dev = torch.device("cuda:0")
    cfgs = [(300, 0.25, 1.0), (1000, 0.1, 1.0), (1000, 0.5, 1.0), (5000, 0.1, 1.0), (20000, 0.1, 1.0),
            (50000, 0.1, 1.0), (100000, 0.1, 1.0), (20000, 0.1, 5.0), (100000, 0.1, 5.0)]
    for M, sig, ext in cfgs:
        g = torch.Generator().manual_seed(M)
        q = (ext * torch.rand(M, 3, generator=g)).to(dev)
        p = (0.05 * torch.randn(M, 3, generator=g)).to(dev)
        order = spatial_order(q)
        a = math.sqrt(1.4426950408889634 / (2 * sig * sig))
        qs = (q.double() * a)[order.long()].cpu()
        spreads = [float(((qs[i:i + 256] - qs[i:i + 256].mean(0)) ** 2).sum(1).max().sqrt())
                   for i in range(0, M, 256)]
        spreads.sort()
        rows = torch.randperm(M, generator=g)[:256]
        ref = ref_rows(q.cpu(), p.cpu(), sig, rows)
        line = f"M={M} sigma={sig} extent={ext}: WG spread median {spreads[len(spreads) // 2]:.2f} max {spreads[-1]:.2f} |"
        for name, alg, rmax in (("pk", 2, None), ("mfma_forced", 3, 100000), ("mfma_default", 3, None)):
            _lib.set_option("fwd_alg", alg)
            if rmax is not None:
                _lib.set_option("mfma_rmax_x100", rmax)
            out = _lib.ode_self_fwd(q, p, sig, 0.0, True, order=order)
            _lib.set_option("mfma_rmax_x100", 300)
            errs = [rel(o[rows].cpu(), r) for o, r in zip((out[0], out[1], out[2]), ref)]
            line += f" {name} v {errs[0]:.1e} mG {errs[1]:.1e} g {errs[2]:.1e} |"
        _lib.set_option("fwd_alg", 3)
        print(line, flush=True)


if __name__ == "__main__":
    main()
