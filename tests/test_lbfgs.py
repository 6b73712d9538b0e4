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


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("seed", range(6))
def test_host_line_search_bitwise_torch(dtype, seed):
    """CompactLBFGS._strong_wolfe (host scalars, one transfer per evaluation) takes the same
    decisions as torch.optim.lbfgs._strong_wolfe on 0-d tensors: the same evaluations and,
    in float64, bit-identical step, loss and gradient (float32: up to the ulp of a sqrt),
    from the first-iteration step and from a unit step."""
    from torch.optim.lbfgs import _strong_wolfe
    from difficp_amd.tools.lbfgs import CompactLBFGS
    g = torch.Generator().manual_seed(seed)
    n = 50
    A = torch.randn(n, n, generator=g, dtype=torch.float64)
    A = (A @ A.T / n + 0.1 * torch.eye(n, dtype=torch.float64)).to(dtype)
    c = torch.randn(n, generator=g).to(dtype)

    def f_of(x):   # a non-quadratic objective: the line search has to bracket and zoom
        return 0.5 * x @ (A @ x) + 0.3 * torch.cos(3 * x).sum() - c @ x

    x0 = torch.randn(n, generator=g).to(dtype)
    for t0 in (None, 1.0):
        p = x0.clone().requires_grad_(True)
        opt = CompactLBFGS([p], line_search_fn="strong_wolfe")

        def closure():
            opt.zero_grad()
            L = f_of(p)
            L.backward()
            return L

        with torch.enable_grad():
            L0 = closure()
        g0 = p.grad.clone()
        d = -g0
        gtd = g0.dot(d)
        t = t0 if t0 is not None else min(1.0, 1.0 / g0.abs().sum()) * 1.0

        def obj(x, tt, dd):   # torch's _directional_evaluate
            with torch.no_grad():
                p.add_(dd, alpha=tt)
            with torch.enable_grad():
                L = float(closure())
            gr = p.grad.clone()
            with torch.no_grad():
                p.copy_(x[0])
            return L, gr

        ref = _strong_wolfe(obj, [x0.clone()], t, d, float(L0), g0, gtd)
        gtd_h, dn = opt._dt(float(gtd), float(d.abs().max()))
        t_h = t if isinstance(t, float) else opt._dt(float(t))[0]
        with torch.no_grad():   # as inside CompactLBFGS.step
            out = opt._strong_wolfe(torch.enable_grad()(closure), [x0.clone()], t_h, d, float(L0), g0,
                                    gtd_h, opt._dt(float(g0.abs().max()))[0], dn)
        assert out[3] == ref[3]                                   # same evaluations
        if dtype == torch.float64:                                # bit-identical decisions
            assert out[0] == ref[0] and float(out[2]) == float(ref[2])
            assert torch.equal(out[1], ref[1])
        else:
            # float32: torch's 0-d tensor sqrt (CPU: not correctly rounded; GPU: the device's)
            # can differ from numpy's by an ulp inside the cubic interpolation
            assert abs(float(out[2]) - float(ref[2])) <= 4e-7 * abs(float(ref[2]))
            assert abs(out[0] - ref[0]) <= 1e-6 * abs(ref[0])
