"""CPU: the lockstep launch barrier of core/batching.py (LaunchBatcher) -- every submitted
launch runs exactly once, each frame's launches keep their order, a batch fires when every
member (a frame inside a closure) is waiting (so frames of different lengths never deadlock),
frames between closures are not waited for, the calls of a batch are ordered by frame key, and
a failing call fails every frame of its batch.  The
launches here are Python callables (no device); dicp_batch_begin / dicp_batch_end of the real
library run around them (an empty batch issues nothing)."""
import threading

import pytest


class _FakeStream:
    cuda_stream = 0


def _run(lengths, fail_at=None):
    from difficp_amd import _lib
    from difficp_amd.core.batching import LaunchBatcher
    b = LaunchBatcher(_FakeStream())
    log, batches = [], []
    lock = threading.Lock()
    start = threading.Barrier(len(lengths))
    orig_flush = b._flush

    def flush():
        batches.append(sorted((s["key"]) for s in b._pending))
        orig_flush()
    b._flush = flush
    errors = {}

    def frame(k, n):
        _lib._tl.frame_key = k
        _lib._tl.in_closure = False
        with b.closure():
            start.wait()
            for i in range(n):
                def fn(k=k, i=i):
                    with lock:
                        log.append((k, i))
                    return 1 if (k, i) == fail_at else 0
                try:
                    b.submit("ode_self_fwd", 10, 10, fn)
                except RuntimeError as e:
                    errors[k] = e
                    return
    ts = [threading.Thread(target=frame, args=(k, n)) for k, n in enumerate(lengths)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=30)
        assert not t.is_alive(), "deadlock"
    return log, batches, errors, b


def test_barrier_runs_each_launch_once_in_order():
    lengths = [3, 7, 1, 7, 5]
    log, batches, errors, b = _run(lengths)
    assert not errors
    assert sorted(log) == sorted((k, i) for k, n in enumerate(lengths) for i in range(n))
    for k, n in enumerate(lengths):
        assert [i for kk, i in log if kk == k] == list(range(n))   # per-frame order kept
    # lockstep: the first batch holds every frame; batches only shrink as frames finish
    assert batches[0] == list(range(len(lengths)))
    assert b.batches == len(batches) == max(lengths) and b.calls == sum(lengths)
    # within a batch the calls run in frame-key order
    pos = 0
    for keys in batches:
        got = [k for k, _ in log[pos:pos + len(keys)]]
        assert got == sorted(got)
        pos += len(keys)


def test_failing_call_fails_its_batch():
    log, batches, errors, b = _run([2, 2, 2], fail_at=(1, 0))
    assert set(errors) == {0, 1, 2}
    assert all("recording ode_self_fwd failed" in str(e) for e in errors.values())


def test_frames_between_closures_are_not_waited_for():
    """A frame in its host phase (outside a closure) does not hold the others' batches; its
    own launch outside a closure joins the next batch (or fires alone)."""
    import time
    from difficp_amd import _lib
    from difficp_amd.core.batching import LaunchBatcher
    b = LaunchBatcher(_FakeStream())
    log = []
    inside = threading.Event()

    def busy():                       # inside a closure, 4 launches
        _lib._tl.frame_key, _lib._tl.in_closure = 0, False
        with b.closure():
            inside.set()
            for i in range(4):
                b.submit("ode_self_fwd", 1, 1, lambda i=i: log.append(("busy", i)) or 0)

    def idle():                       # host phase, then one launch outside any closure
        _lib._tl.frame_key, _lib._tl.in_closure = 1, False
        inside.wait()
        time.sleep(0.2)
        b.submit("ode_self_fwd", 1, 1, lambda: log.append(("idle", 0)) or 0)
    ts = [threading.Thread(target=f) for f in (busy, idle)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=30)
        assert not t.is_alive(), "deadlock"
    assert sorted(log) == sorted([("busy", i) for i in range(4)] + [("idle", 0)])
    assert [x for x in log if x[0] == "busy"] == [("busy", i) for i in range(4)]
    assert b._members == 0 and not b._pending
