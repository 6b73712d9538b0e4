"""Row-split of ONE frame's geodesic shooting over the ranks of a process group (SURVEY 8(f)
f1: a single two-set match, C2/C3, on several GPUs).

The reference has no multi-device path (one frame = one KeOps call sequence on one device).
Here every rank keeps the full support state (q, p): M x 2D floats, 2.4 MB at 100k points,
and per ODE evaluation
  * forward (Euler step): rank r computes the rows [r0, r1) of the fused step against all M
    columns (dicp_lddmm_euler_step_rows_f32), then ONE all-gather exchanges the new row
    slices (+ each rank's divergence partial sum).  With `overlap` (W | M) the step runs in
    two column phases (dicp_lddmm_euler_step_phase_f32): the rank's rows against its own
    slice while the previous step's all-gather is in flight, then against the other points;
  * adjoint step: rank r computes its part of the symmetric pair-once VJP (the quads
    Q = r mod W, dicp_lddmm_ode_self_bwd_part_f32) for all rows, then ONE all-reduce sums the
    parts (M x 2D floats).
Every collective returns bitwise-identical data on all ranks (all-gather is exact; an
all-reduce reduces each element once and broadcasts it -- `exact_reduce` replaces it by an
all-gather + rank-ordered sum, `verify` checks it), and the scalar partials (divergence,
Hamiltonian) are combined in rank order, so every rank runs the same L-BFGS iterates and
takes the same decisions -- the host logic above (LBFGS, EM, PSR) runs replicated, unchanged.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..tools import runstats


class RowSplit:
    """Rank / world of a torch.distributed process group (RCCL over xGMI on the GPU box,
    gloo in the CPU tests) and the two collectives the split shooting needs."""

    def __init__(self, group=None, exact_reduce=None, verify=None, overlap=None):
        """exact_reduce: sum the per-step VJP parts by all-gather + rank-ordered sum instead of
        an all-reduce (bitwise identical on every rank by construction, W x the bytes; default
        from DICP_ROWSPLIT_EXACT, off).  verify: after every all-reduce, all-gather a float64
        checksum of the result and raise if the ranks disagree (one host sync per call; default
        from DICP_ROWSPLIT_VERIFY, off) -- the check that the replicated L-BFGS cannot diverge
        because a collective returned different bits on different ranks.  overlap: run each
        forward step in column phases so that the all-gather of the previous step's rows
        overlaps the rank's rows against its own slice (ShootFn, split_step_phased; default
        from DICP_ROWSPLIT_OVERLAP = 1 / 0 / auto, auto = from 4 ranks: per step the phases
        cost +47 us at W = 2, -60 us at W = 4, +17 us at W = 8 against the all-gather they
        hide, profiles/r04_rowsplit_phases.jsonl) -- a different fp32 summation order than
        the one-pass step, the same bits on every rank."""
        import os
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self._gather_base = dist.get_backend(group) != "gloo"
        env = os.environ.get
        self.exact_reduce = bool(int(env("DICP_ROWSPLIT_EXACT", "0"))) if exact_reduce is None \
            else bool(exact_reduce)
        self.verify = bool(int(env("DICP_ROWSPLIT_VERIFY", "0"))) if verify is None else bool(verify)
        if overlap is None:   # "auto": from 4 ranks (the measured break-even)
            ov = env("DICP_ROWSPLIT_OVERLAP", "auto")
            overlap = self.world >= 4 if ov == "auto" else bool(int(ov))
        self.overlap = bool(overlap)
        self.verified_calls = 0

    def rows(self, M: int):
        """(row0, nrows, per): this rank's row slice; per = ceil(M / W) (padded chunk)."""
        per = -(-M // self.world)
        r0 = min(per * self.rank, M)
        r1 = min(r0 + per, M)
        return r0, r1 - r0, per

    def all_gather(self, local: torch.Tensor) -> torch.Tensor:
        """(W * n,) concatenation of every rank's (n,) buffer, in rank order."""
        out = torch.empty(self.world * local.numel(), device=local.device, dtype=local.dtype)
        with runstats.collective():
            if self._gather_base:
                dist.all_gather_into_tensor(out, local, group=self.group)
            else:
                dist.all_gather(list(out.chunk(self.world)), local, group=self.group)
        return out

    def gather_into(self, out: torch.Tensor, local: torch.Tensor) -> torch.Tensor:
        """All-gather the ranks' equal-sized contiguous `local` slices straight into the
        contiguous `out` (W x local.numel() elements, rank order): no staging buffer, no
        copies (the row slices of a step when W divides M)."""
        flat = out.view(-1)
        if flat.numel() != self.world * local.numel():
            raise ValueError("gather_into: out must hold W x local elements")
        with runstats.collective():
            if self._gather_base:
                dist.all_gather_into_tensor(flat, local.reshape(-1), group=self.group)
            else:
                dist.all_gather(list(flat.chunk(self.world)), local.reshape(-1), group=self.group)
        return out

    def gather_into_async(self, out: torch.Tensor, local: torch.Tensor):
        """gather_into without waiting: returns the work handle, whose wait() makes the current
        stream wait for the collective (RCCL; gloo: blocks the host).  `out` and `local` must
        stay untouched until then (local may be read)."""
        flat = out.view(-1)
        if flat.numel() != self.world * local.numel():
            raise ValueError("gather_into_async: out must hold W x local elements")
        runstats.add("collectives")
        if self._gather_base:
            return dist.all_gather_into_tensor(flat, local.reshape(-1), group=self.group, async_op=True)
        return dist.all_gather(list(flat.chunk(self.world)), local.reshape(-1), group=self.group,
                               async_op=True)

    def sum_ordered(self, t: torch.Tensor) -> torch.Tensor:
        """Cross-rank sum as all-gather + a sum in rank order: the same bits on every rank
        whatever algorithm the backend picks (used for the small (H0, div) scalars and, with
        exact_reduce, for the VJP parts)."""
        allb = self.all_gather(t.reshape(-1).contiguous()).view(self.world, -1)
        s = allb[0].clone()
        for r in range(1, self.world):
            s = s + allb[r]
        return s.view(t.shape)

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        """In-place cross-rank sum of t.  An RCCL all-reduce (ring or tree) reduces each element
        once and broadcasts it, so every rank receives the same bits; exact_reduce makes that
        hold by construction, verify checks it."""
        if self.exact_reduce:
            t.copy_(self.sum_ordered(t))
        else:
            with runstats.collective():
                dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        if self.verify:
            self.check_identical(t)
        return t

    def check_identical(self, t: torch.Tensor) -> None:
        """Raise if t is not bitwise the same on every rank (float64 checksum of the values
        and of their bit patterns, all-gathered)."""
        flat = t.reshape(-1)
        bits = flat.contiguous().view(torch.int32).to(torch.float64) if flat.dtype == torch.float32 \
            else flat.to(torch.float64)
        w = torch.arange(1, flat.numel() + 1, device=flat.device, dtype=torch.float64)
        cs = torch.stack([(bits * w).sum(), flat.to(torch.float64).sum()])
        allc = self.all_gather(cs).view(self.world, 2).cpu()
        if not bool((allc == allc[0]).all()):
            raise RuntimeError(f"row split: a collective returned different data on different "
                               f"ranks (checksums {allc.tolist()}): the replicated L-BFGS would diverge")
        self.verified_calls += 1

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
