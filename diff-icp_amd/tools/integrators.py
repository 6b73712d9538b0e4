"""Explicit ODE integrators over tuples of tensors (semantics of diffICP/tools/integrators.py).

Used by LDDMMModel.ODE-level integration (the generic, per-step autograd path).  The
shooting hot path uses the fused trajectory function in core/shooting.py, which applies
exactly these update rules and their discrete adjoints.
"""


def EulerIntegrator(ODESystem, x0, nt=11, deltat=1.0):
    """x_{k+1} = x_k + dt f(x_k); returns the list of the nt+1 states (integrators.py:20-31)."""
    x = tuple(t.clone() for t in x0)
    dt = deltat / nt
    states = [x]
    for _ in range(nt):
        xdot = ODESystem(*x)
        x = tuple(a + dt * b for a, b in zip(x, xdot))
        states.append(x)
    return states


def RalstonIntegrator(ODESystem, x0, nt=11, deltat=1.0):
    """Ralston's 2nd-order scheme: k1 = f(x), k2 = f(x + 2dt/3 k1),
    x' = x + dt/4 (k1 + 3 k2) (integrators.py:36-51)."""
    x = tuple(t.clone() for t in x0)
    dt = deltat / nt
    states = [x]
    for _ in range(nt):
        k1 = ODESystem(*x)
        xi = tuple(a + (2 * dt / 3) * b for a, b in zip(x, k1))
        k2 = ODESystem(*xi)
        x = tuple(a + (0.25 * dt) * (b + 3 * c) for a, b, c in zip(x, k1, k2))
        states.append(x)
    return states
