"""Lockstep launch batching of independent frames (the groupwise atlas, PSR.py:528-569).

The atlas optimises every frame's LDDMM registration independently (one L-BFGS run each).  At
~20k points a frame's pair kernels are too small to keep the chip busy to the end of each
launch, and the frames' host work (L-BFGS logic, launches) is serialised by the GIL.  A
LaunchBatcher runs the frames of a group in lockstep at the level of the library's launches:
each frame keeps its own host thread and its own code path (Optimize, ShootFn's forward and
exact adjoint, CompactLBFGS), but its batchable launches (the packed eta = 0 shooting passes,
_lib.BATCHABLE) are handed to the batcher, which waits until every running frame of the group
has posted one, then records them all inside ONE dicp_batch_begin / dicp_batch_end scope (the
C-ABI issues one grid over all the frames per kernel instantiation and stage) and releases
the frames.  Each recorded call keeps its own arguments, geometry and workspace, so every
frame's results are bitwise those of the sequential frame loop; only the launch count and the
tails change.  One change of route is needed for that: autograd runs every CUDA backward on
its engine's device thread, one frame after another, so under a batcher Optimize's closure
forms the loss gradient with ShootFn's adjoint called on the frame's own thread
(shooting.shoot_loss_grad: the same cotangents, hence the same bits).

Deadlock freedom: a frame waits only inside submit(); a batch fires as soon as every member
(a frame inside a closure, or one whose launch outside a closure is pending) is waiting
there; a frame inside a closure does no device read (it only launches and queues small torch
ops), so it will post or leave; leaving (also on an exception) fires a batch the others may be
waiting for.  Frames between closures (L-BFGS host logic, loss reads) are not waited for.
"""
from __future__ import annotations

import threading

import torch

from .. import _lib


class LaunchBatcher:
    """Launch barrier over the frames (host threads) of one group; see the module docstring.
    All frames of a group run on ONE HIP stream (`stream`), so the batched launch is ordered
    after every frame's previous work and before its next.

    Members: a frame is waited for only while it is inside a loss/gradient evaluation
    (`closure()`, Optimize's closures) -- between closures it runs its L-BFGS host logic and
    the others' batches go on without it -- and, outside closures, while one of its launches
    is pending.  A batch fires when every member has a launch pending.  With the default
    geometry (batch_share 1) a call's result does not depend on which calls share its batch,
    so the timing-dependent composition of the batches changes no result."""

    def __init__(self, stream):
        self.stream = stream
        self._cv = threading.Condition()
        self._members = 0
        self._pending = []
        self.batches = 0        # statistics: batched flushes and calls recorded
        self.calls = 0

    # ---- membership: a frame inside a closure ----
    def enter(self):
        with self._cv:
            self._members += 1

    def leave(self):
        with self._cv:
            self._members -= 1
            self._maybe_flush()

    class _Closure:
        def __init__(self, b):
            self.b = b

        def __enter__(self):
            self.prev = getattr(_lib._tl, "in_closure", False)
            _lib._tl.in_closure = True
            if not self.prev:
                self.b.enter()
            return self

        def __exit__(self, *exc):
            _lib._tl.in_closure = self.prev
            if not self.prev:
                self.b.leave()
            return False

    def closure(self):
        """Context manager around one loss/gradient evaluation of a frame."""
        return LaunchBatcher._Closure(self)

    def _maybe_flush(self):
        if self._pending and len(self._pending) >= self._members:
            self._flush()

    # ---- the per-launch barrier (called by _lib._launch on a frame thread) ----
    def submit(self, name, pairs, nbytes, fn):
        slot = {"key": getattr(_lib._tl, "frame_key", 0), "name": name, "pairs": int(pairs),
                "nbytes": int(nbytes), "fn": fn, "raw": _lib.get_option("coord_raw"),
                "share": _lib.get_option("batch_share"), "done": False}
        transient = not getattr(_lib._tl, "in_closure", False)
        with self._cv:
            if transient:           # a launch outside a closure: a member until it is issued
                self._members += 1
            self._pending.append(slot)
            self._maybe_flush()
            while not slot["done"]:
                self._cv.wait()
            if transient:
                self._members -= 1
                self._maybe_flush()
        if slot.get("error") is not None:
            raise slot["error"]
        return slot["rc"]

    def _flush(self):
        """Record every pending call in one batch and issue it (caller holds the lock)."""
        items = sorted(self._pending, key=lambda s: s["key"])
        self._pending = []
        err, rc = None, 0
        prof = _lib._prof
        try:
            handle = self.stream.cuda_stream
            e0 = e1 = None
            with _lib.batch(handle):
                for s in items:
                    # the submitting frame's per-thread knobs (coordinates, geometry hint)
                    with _lib.coord_mode(s["raw"]), _lib.thread_option(s["share"], "batch_share"):
                        r = s["fn"]()
                    if r:
                        raise RuntimeError(f"dicp batch: recording {s['name']} failed: "
                                           f"{_lib.lib().dicp_last_error().decode()}")
                if prof is not None:
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    e0.record(self.stream)
            if prof is not None:
                e1.record(self.stream)
                self._profile(prof, items, e0, e1)
            self.batches += 1
            self.calls += len(items)
        except Exception as e:   # every frame of the batch sees the failure
            err, rc = e, -1
        for s in items:
            s["rc"], s["error"], s["done"] = rc, err, True
        self._cv.notify_all()

    @staticmethod
    def _profile(prof, items, e0, e1):
        """One KernelProfile record per kernel name of the batch: its calls' pairs, flops
        and bytes, and the batch's time x its share of the batch's flops."""
        by = {}
        for s in items:
            d = by.setdefault(s["name"], [0, 0, 0])
            d[0] += s["pairs"]
            d[1] += int(s["pairs"] * _lib.FLOPS_PER_PAIR.get(s["name"], 0))
            d[2] += s["nbytes"]
        tot = sum(v[1] for v in by.values()) or 1
        for name, (pairs, flops, nbytes) in by.items():
            prof.records.append((name, pairs, flops, nbytes, e0, e1, flops / tot))


class frame_thread:
    """Context manager run by a frame's host thread: its batchable launches go through
    `batcher` (keyed by `key` for a deterministic order inside a batch) on the batcher's
    stream.  share > 1: the library's geometry hint "batch_share" for this thread (each launch
    sized for 1/share of the chip, csrc/batch.hpp), fixed for the whole run of the frame."""

    def __init__(self, batcher: LaunchBatcher, key: int, share: int = 1):
        self.batcher, self.key, self.share = batcher, key, int(share)

    def __enter__(self):
        _lib._tl.batcher = self.batcher
        _lib._tl.frame_key = self.key
        _lib._tl.in_closure = False
        self._opt = _lib.thread_option(self.share, "batch_share")
        self._opt.__enter__()
        self._st = torch.cuda.stream(self.batcher.stream)
        self._st.__enter__()
        return self

    def __exit__(self, *exc):
        try:
            self._st.__exit__(*exc)
            self._opt.__exit__(*exc)
        finally:
            _lib._tl.batcher = None
        return False
