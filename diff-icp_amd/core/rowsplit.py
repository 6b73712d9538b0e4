"""Row-split of ONE frame's geodesic shooting over the ranks of a process group (SURVEY 8(f)
f1: a single two-set match, C2/C3, on several GPUs).

The reference has no multi-device path (one frame = one KeOps call sequence on one device).
Here every rank keeps the full support state (q, p): M x 2D floats, 2.4 MB at 100k points,
and per ODE evaluation
  * forward (Euler step): rank r computes the rows [r0, r1) of the fused step against all M
    columns (dicp_lddmm_euler_step_rows_f32), then ONE all-gather exchanges the new row
    slices (+ each rank's divergence partial sum);
  * adjoint step: rank r computes its part of the symmetric pair-once VJP (the quads
    Q = r mod W, dicp_lddmm_ode_self_bwd_part_f32) for all rows, then ONE all-reduce sums the
    parts (M x 2D floats).
Every collective returns bitwise-identical data on all ranks (all-gather is exact; an
all-reduce reduces each element once and broadcasts it), and the divergence partials are
combined in rank order, so every rank runs the same L-BFGS iterates and takes the same
decisions -- the host logic above (LBFGS, EM, PSR) runs replicated, unchanged.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class RowSplit:
    """Rank / world of a torch.distributed process group (RCCL over xGMI on the GPU box,
    gloo in the CPU tests) and the two collectives the split shooting needs."""

    def __init__(self, group=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self._gather_base = dist.get_backend(group) != "gloo"

    def rows(self, M: int):
        """(row0, nrows, per): this rank's row slice; per = ceil(M / W) (padded chunk)."""
        per = -(-M // self.world)
        r0 = min(per * self.rank, M)
        r1 = min(r0 + per, M)
        return r0, r1 - r0, per

    def all_gather(self, local: torch.Tensor) -> torch.Tensor:
        """(W * n,) concatenation of every rank's (n,) buffer, in rank order."""
        out = torch.empty(self.world * local.numel(), device=local.device, dtype=local.dtype)
        if self._gather_base:
            dist.all_gather_into_tensor(out, local, group=self.group)
        else:
            dist.all_gather(list(out.chunk(self.world)), local, group=self.group)
        return out

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t

    # -------------------------------------------------------------------------------
    def gather_rows(self, parts, M: int, scalar=None):
        """parts: this rank's (nrows, D) slices [a, b, ...] and optionally a (1,) scalar.
        Returns the full (M, D) tensors (rank order) and the rank-ordered sum of the
        scalars (or None).  ONE all-gather of a padded (per * sum(D) + 1) buffer."""
        r0, n, per = self.rows(M)
        D = parts[0].shape[1]
        k = len(parts)
        dev, dt = parts[0].device, parts[0].dtype
        buf = torch.zeros(k * per * D + 1, device=dev, dtype=dt)
        for i, t in enumerate(parts):
            if n:
                buf[i * per * D: i * per * D + n * D].copy_(t.reshape(-1))
        if scalar is not None:
            buf[-1:].copy_(scalar.reshape(1))
        allb = self.all_gather(buf).view(self.world, -1)
        outs = [allb[:, i * per * D: (i + 1) * per * D].reshape(self.world * per, D)[:M]
                for i in range(k)]
        scal = None
        if scalar is not None:
            scal = allb[0, -1:].clone()
            for r in range(1, self.world):  # rank order: identical on every rank
                scal = scal + allb[r, -1:]
        return outs, scal
