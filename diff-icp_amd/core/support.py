"""Support-point schemes and small helpers shared by the two registration drivers:
core/PSR.py (diff-ICP, `DiffPSR`) and core/PSR_standard.py (template estimation,
`DiffPSR_std`).

Reference behaviour (diffICP/core/PSR.py:430-493 and PSR_standard.py:445-503):
  * "decim"  : greedy covering decimation of each structure (point_sets.py:102-133), radius
               Rcover = rho * sigma_LDDMM -- the pair work runs on the device
               (tools/point_sets.decimate, bit-exact indices);
  * "grid"   : a regular grid of spacing Rcover over the bounding box of the points plus a 10%
               margin (visualization/visu.py:35-50 get_bounds); the reference builds it in 2D
               only (PSR.py:472-482) -- `grid_points` keeps that construction and ordering in
               2D and extends it to 3D, z varying slowest;
  * "custom" : user-given support points.
After a support change the momenta are re-projected so the initial velocity field is kept
(v2p of the old field on the new support, PSR.py:415-425).
"""
from __future__ import annotations

import warnings

import numpy as np
import torch


def bounds_with_margin(point_sets, D, relmargin=0.1):
    """(mins, maxs) of the union of point sets, widened by relmargin on each side, in the
    reference's float32 arithmetic (get_bounds, visualization/visu.py:35-50)."""
    xs = [a.detach().cpu() for a in point_sets if len(a) > 0]
    mins = torch.cat(tuple(a.min(0).values.reshape(1, D) for a in xs), 0).min(0).values.numpy()
    maxs = torch.cat(tuple(a.max(0).values.reshape(1, D) for a in xs), 0).max(0).values.numpy()
    return (1 + relmargin) * mins - relmargin * maxs, (1 + relmargin) * maxs - relmargin * mins


def grid_points(point_sets, Rcover, D, spec, ticks=None):
    """Regular support grid of spacing Rcover covering the point sets (+10% margin).

    ticks: optional per-axis tick arrays (x, y[, z]); a None entry is derived from the bounds
    as np.arange(lo - Rcover/2, hi + Rcover/2, Rcover).  The points are ordered as the
    reference's 2D grid: np.meshgrid(...) stacked on the last axis, flattened in Fortran
    order (first meshgrid axis fastest); in 3D the third axis varies slowest."""
    if D not in (2, 3):
        raise ValueError(f"grid support scheme: D = {D} not supported (2D as the reference, 3D)")
    ticks = list(ticks) if ticks is not None else [None] * D
    if len(ticks) != D:
        raise ValueError(f"grid support scheme: {D} tick arrays expected")
    if any(t is None for t in ticks):
        lo, hi = bounds_with_margin(point_sets, D)
        ticks = [np.arange(lo[d] - Rcover / 2, hi[d] + Rcover / 2, Rcover) if ticks[d] is None
                 else np.asarray(ticks[d]) for d in range(D)]
    g = np.stack(np.meshgrid(*ticks), axis=D)
    return torch.tensor(g.reshape((-1, D), order="F"), **spec).contiguous()


def decimated_points(point_sets, Rcover, spec):
    """Greedy covering decimation of each point set (point_sets.py:102-133); returns the
    concatenated kept points and the kept indices per set."""
    from ..tools.point_sets import decimate
    ids = [decimate(p.to(**spec), Rcover)[0] for p in point_sets]
    q = torch.cat(tuple(p[i] for p, i in zip(point_sets, ids)), dim=0).to(**spec).contiguous()
    return q, ids


def merged_v2p_args(defaults, given):
    """v2p keyword arguments of a support change: the caller's, unless the driver was built
    with explicit v2p_args (DiffPSR / DiffPSR_std extension) and the caller names no version --
    then the driver's, with the caller's other arguments except `rcond` (a pinv tolerance)."""
    if defaults and not given.get("version"):
        return {**defaults, **{k: v for k, v in given.items() if k != "rcond"}}
    return given


def warn_uncovered(kernel, shoot, Rw=2.0):
    """The reference's coverage check of a non-dense-support shooting (PSR.py:559-566,
    PSR_standard.py:553-560): at every time step, points carried as external points farther
    than Rw * sigma from every support point are reported."""
    for t, st in enumerate(shoot):
        q, pts = st[0], st[-1]
        unc = kernel.check_coverage(pts, q, Rw)
        if unc.any():
            n = int(unc.sum())
            print(f"WARNING : shooting, time step {t} : {n} uncovered points ({n / pts.shape[0]:.2%})")
            warnings.warn("Uncovered points during LDDMM shooting. Choose a smaller rho when "
                          "defining the support scheme.", RuntimeWarning)


def split_rows(t, counts):
    """Split a concatenation of per-structure rows back into the structures."""
    out, first = [], 0
    for n in counts:
        out.append(t[first:first + int(n)])
        first += int(n)
    return out
