"""Input normalisation x -> x[k][s] (mirror of diffICP/tools/in_out.py:7-47)."""
import torch


def _is_float_tensor(t):
    return isinstance(t, torch.Tensor) and t.dtype == torch.float32


def read_point_sets(x):
    """Accepts a (N,D) float32 tensor, a list x[k] of tensors, or a list of lists x[k][s].
    Returns (x as list-of-lists, K frames, S structures, D).  Same errors as the reference."""
    if _is_float_tensor(x):
        x = [[x]]
    elif isinstance(x, list):
        if _is_float_tensor(x[0]):
            x = [[xk] for xk in x]
        else:
            x = [list(xk) for xk in x]
    else:
        raise ValueError("Wrong format for input x")
    K = len(x)
    allSs = list(set(len(xk) for xk in x))
    if len(allSs) > 1:
        raise ValueError("All frames should have same number of structures")
    S = allSs[0]
    allDs = list(set(xks.shape[1] for xk in x for xks in xk))
    if len(allDs) > 1:
        raise ValueError("All point sets should have same axis-1 dimension")
    D = allDs[0]
    return x, K, S, D
