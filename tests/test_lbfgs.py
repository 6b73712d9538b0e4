"""CompactLBFGS (tools/lbfgs.py) == torch.optim.LBFGS (the reference's optimizer,
optim.py:26) up to rounding: same iterates on smooth problems in float64, incl. the
history-overflow path and the no-line-search restart mode."""
import pytest
import torch

from difficp_amd.tools.lbfgs import CompactLBFGS


def _run(opt_cls, f, x0, steps, **kw):
    x = x0.clone().requires_grad_(True)
    opt = opt_cls([x], **kw)
    traj = []

    def closure():
        opt.zero_grad()
        L = f(x)
        L.backward()
        return L

    for _ in range(steps):
        opt.step(closure)
        traj.append(x.detach().clone())
    return traj


def _rosen(x):
    return (100 * (x[1:] - x[:-1] ** 2) ** 2 + (1 - x[:-1]) ** 2).sum()


def _quad(A, b):
    return lambda x: 0.5 * x @ (A @ x) - b @ x


@pytest.mark.parametrize("ls", ["strong_wolfe", None])
@pytest.mark.parametrize("hist", [100, 5])
def test_compact_matches_torch_lbfgs(ls, hist):
    g = torch.Generator().manual_seed(0)
    x0 = torch.randn(40, generator=g, dtype=torch.float64) * 0.5
    kw = dict(max_iter=20, max_eval=100, history_size=hist, line_search_fn=ls,
              lr=1.0 if ls else 0.05)
    t1 = _run(torch.optim.LBFGS, _rosen, x0, 3, **kw)
    t2 = _run(CompactLBFGS, _rosen, x0, 3, **kw)
    # the first step (20 iterations, history overflow included for hist=5) agrees to rounding;
    # later Rosenbrock steps amplify rounding differences, so compare objective values there
    assert float((t1[0] - t2[0]).norm() / t2[0].norm()) < 1e-9
    for a, b in zip(t1[1:], t2[1:]):
        assert abs(float(_rosen(a)) - float(_rosen(b))) < 1e-3 * abs(float(_rosen(a)))


def test_compact_quadratic_convergence():
    g = torch.Generator().manual_seed(1)
    Q = torch.randn(30, 30, generator=g, dtype=torch.float64)
    A = Q @ Q.t() + 30 * torch.eye(30, dtype=torch.float64)
    b = torch.randn(30, generator=g, dtype=torch.float64)
    kw = dict(max_iter=20, history_size=100, line_search_fn="strong_wolfe")
    x = _run(CompactLBFGS, _quad(A, b), torch.zeros(30, dtype=torch.float64), 2, **kw)[-1]
    xt = _run(torch.optim.LBFGS, _quad(A, b), torch.zeros(30, dtype=torch.float64), 2, **kw)[-1]
    assert float((A @ x - b).norm() / b.norm()) < 1e-4   # stops on tolerance_change, as torch
    assert float((x - xt).norm() / xt.norm()) < 1e-10
