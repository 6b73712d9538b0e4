"""Per-process counters of the PSR driver's host-visible work (no reference counterpart):
L-BFGS closure evaluations (tools/optim.py), EM steps (core/GMM.py EM_optimization) and the
collectives of the frame sharding / row split with the host wall time spent in them (which
includes waiting for the slowest rank -- the load imbalance a multi-GPU line must show).
bench.py snapshots them around its timed region and rank 0 gathers every rank's numbers.
Thread-safe: concurrent frames (one host thread each) count into the same process totals."""
import threading
import time
from contextlib import contextmanager

_lock = threading.Lock()
_c = {"closures": 0, "em_steps": 0, "collectives": 0, "collective_s": 0.0}


def add(name, n=1):
    with _lock:
        _c[name] += n


@contextmanager
def collective():
    """Count one collective and its host wall time (launch to return; for a synchronous
    backend or a result the caller reads right away, the exchange itself)."""
    t0 = time.perf_counter()
    try:
        yield
    finally:
        dt = time.perf_counter() - t0
        with _lock:
            _c["collectives"] += 1
            _c["collective_s"] += dt


def snapshot():
    with _lock:
        return dict(_c)


def delta(before, after=None):
    after = snapshot() if after is None else after
    return {k: after[k] - before[k] for k in after}
