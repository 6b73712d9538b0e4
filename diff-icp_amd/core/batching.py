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

Deadlock freedom: a frame waits only inside submit(); the batch fires as soon as every frame
still registered is waiting there, and a frame that finishes (or fails) unregisters, which
fires a batch the others may be waiting for.  A frame doing host work or a device read
(.item()) will eventually post or finish: the device work it waits for was issued before.
"""
from __future__ import annotations

import threading

import torch

from .. import _lib


class LaunchBatcher:
    """Lockstep launch barrier over the frames (host threads) of one group; see the module
    docstring.  All frames of a group run on ONE HIP stream (`stream`), so the batched launch
    is ordered after every frame's previous work and before its next."""

    def __init__(self, stream: torch.cuda.Stream):
        self.stream = stream
        self._cv = threading.Condition()
        self._active = 0
        self._pending = []
        self.batches = 0        # statistics: batched flushes and calls recorded
        self.calls = 0

    # ---- frame membership ----
    def register(self, n: int = 1):
        with self._cv:
            self._active += n

    def unregister(self):
        with self._cv:
            self._active -= 1
            if self._pending and len(self._pending) >= self._active:
                self._flush()

    # ---- the per-launch barrier (called by _lib._launch on a frame thread) ----
    def submit(self, name, pairs, nbytes, fn):
        slot = {"key": getattr(_lib._tl, "frame_key", 0), "name": name, "pairs": int(pairs),
                "nbytes": int(nbytes), "fn": fn, "raw": _lib.get_option("coord_raw"),
                "share": _lib.get_option("batch_share"), "done": False}
        with self._cv:
            self._pending.append(slot)
            if len(self._pending) >= self._active:
                self._flush()
            while not slot["done"]:
                self._cv.wait()
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
    stream; on exit the frame leaves the group (its registration was made up front).
    share > 1: the library's geometry hint "batch_share" for this thread (each launch sized
    for 1/share of the chip, csrc/batch.hpp) -- fixed for the whole run of the frame, so its
    results do not depend on how the batches happen to be composed."""

    def __init__(self, batcher: LaunchBatcher, key: int, share: int = 1):
        self.batcher, self.key, self.share = batcher, key, int(share)

    def __enter__(self):
        _lib._tl.batcher = self.batcher
        _lib._tl.frame_key = self.key
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
            self.batcher.unregister()
        return False
