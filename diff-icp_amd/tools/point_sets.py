"""Support-point helpers of diffICP/tools/point_sets.py on the device: `decimate` (greedy
covering decimation, point_sets.py:102-133) and `intrinsic_scale` (point_sets.py:13-26).

Both are O(N^2) on the host / KeOps in the reference; here the pair work runs in the HIP
kernels behind dicp_radius_count_f32 and dicp_gauss_red_f32(MIN_SQDIST_OTHER), with the
distance computed in the reference's exact float32 arithmetic so the greedy choices (and
hence the kept indices) are identical.
"""
import torch

from .. import _lib
from .spec import getspec


def intrinsic_scale(x):
    """Mean over points of the squared distance to the nearest OTHER point, square-rooted
    (point_sets.py:13-26: D_ij.Kmin(2, dim=1)[:, 1], i.e. the second smallest entry of each
    row, self included -- equal to the minimum over j != i).  Returns a Python float."""
    getspec(x)
    x = x.detach().contiguous()
    d2 = _lib.gauss_red(_lib.MIN_SQDIST_OTHER, x, x, 1.0)
    return 1 * d2.mean().sqrt().item()


def decimate(x, R):
    """Greedy decimation of point set x (N, D) with radius R (point_sets.py:102-133).

    Repeatedly keeps the not-yet-covered point with the most not-yet-covered neighbours
    (|x_i - x_j|^2 <= R^2; ties -> smallest index, as torch.argmax over the reference's
    increasing `notcovered` list) and marks its neighbours covered.  Returns (kept,
    rejected) as lists of indices, like the reference.

    Device algorithm: the neighbour counts are computed once (one N x N pass) and then
    decremented by the newly covered points of each step (N x |new| passes), so the total
    pair work is 2 N^2 instead of the reference's N^2 per step."""
    getspec(x)
    x = x.detach().contiguous()
    N = x.shape[0]
    if N == 0:
        return [], []
    dev = x.device
    counts = _lib.radius_count(x, x, R)          # neighbours (self included) of every point
    covered = torch.zeros(N, dtype=torch.bool, device=dev)
    minus1 = torch.tensor(-1.0, device=dev)
    kept = []
    while True:
        c = torch.where(covered, minus1, counts)
        idx = torch.argmax(c)                     # first maximal index
        i, best = torch.stack((idx.to(torch.float32), c[idx])).tolist()
        if best < 0:                              # every point covered
            break
        i = int(i)
        kept.append(i)
        newly = (_lib.radius_count(x, x[i:i + 1], R) > 0) & ~covered
        covered |= newly
        counts -= _lib.radius_count(x, x[newly].contiguous(), R)
    kept_set = set(kept)
    rejected = [i for i in range(N) if i not in kept_set]
    return kept, rejected
