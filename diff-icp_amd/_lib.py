"""ctypes binding of the C-ABI library ``libdifficp_hip.so`` (declared in include/difficp_hip.h).

This is the only place that talks to the native library.  It marshals device pointers of
torch tensors, the current HIP stream and a scratch workspace; it never computes anything
itself and there is no CPU fallback: if the library is missing or a tensor is not on a
HIP device the call raises.
"""
from __future__ import annotations

import ctypes
import os
import threading
from collections import OrderedDict

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# DICP_LIB_PATH selects an experiment build (tools/ab_libs.py); default: the in-tree library
LIB_PATH = os.environ.get("DICP_LIB_PATH") or os.path.join(_HERE, "libdifficp_hip.so")

# enum dicp_red_op (include/difficp_hip.h)
KBASE, KREDSCAL, KRED, GRADK, GRADK_REV, DDK, GENDK, HESSK, LAPK, GRADLAPK, GRADKSCAL, \
    GRADLAPKSCAL, MIN_SQDIST, MIN_SQDIST_OTHER = range(14)
# enum dicp_ws_kind
WS_RED, WS_ODE_SELF_FWD, WS_ODE_SELF_BWD, WS_ODE_EXT_FWD, WS_ODE_EXT_BWD, WS_GMM_ESTEP, \
    WS_GMM_MSTEP, WS_GMM_TARGETS, WS_RIDGE_CG, WS_ODE_SELF_FWD_ROWS, WS_ODE_SELF_BWD_PART, WS_GRAD, \
    WS_ODE_SELF_FWD_PHASED = range(13)
# enum dicp_grad_kind
GRAD_HESSW, GRAD_HESSWP, GRAD_ZDOTV, GRAD_HESS3, GRAD_GRADLAP3 = range(5)

_lock = threading.Lock()
_lib = None

_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_INT = ctypes.c_int
_DBL = ctypes.c_double
_SZ = ctypes.c_size_t

_SIGNATURES = {
    "dicp_gauss_red_f32": [_INT, _P, _I64, _P, _I64, _INT, _P, _P, _DBL, _P, _P, _SZ, _P],
    "dicp_radius_count_f32": [_P, _I64, _P, _I64, _INT, _DBL, _P, _P, _SZ, _P],
    "dicp_lddmm_ode_self_fwd_f32": [_P, _P, _I64, _INT, _DBL, _DBL, _P, _P, _P, _P, _P, _SZ, _P],
    "dicp_lddmm_ode_self_bwd_f32": [_P, _P, _P, _P, _P, _I64, _INT, _DBL, _DBL, _P, _P, _P, _SZ, _P],
    "dicp_lddmm_euler_step_f32": [_P, _P, _I64, _INT, _DBL, _DBL, _DBL, _P, _P, _P, _P, _SZ, _P],
    "dicp_lddmm_euler_adjoint_step_f32": [_P, _P, _P, _P, _P, _I64, _INT, _DBL, _DBL, _DBL, _P, _P,
                                          _P, _P, _P, _SZ, _P],
    "dicp_lddmm_ode_ext_fwd_f32": [_P, _I64, _P, _P, _I64, _INT, _DBL, _DBL, _P, _P, _P, _SZ, _P],
    "dicp_lddmm_ode_ext_bwd_f32": [_P, _I64, _P, _P, _I64, _INT, _DBL, _DBL, _P, _P, _P, _P, _P,
                                   _P, _SZ, _P],
    "dicp_gmm_estep_f32": [_P, _I64, _P, _P, _P, _I64, _INT, _DBL, _DBL, _P, _P, _P, _P, _SZ, _P],
    "dicp_gmm_estep_hint_f32": [_P, _I64, _P, _P, _P, _I64, _INT, _DBL, _DBL, _P, _P, _P, _P, _P, _SZ, _P],
    "dicp_gmm_mstep_f32": [_P, _P, _I64, _P, _P, _I64, _INT, _DBL, _P, _P, _SZ, _P],
    "dicp_gmm_targets_f32": [_P, _P, _I64, _P, _P, _DBL, _P, _P, _I64, _INT, _P, _P, _SZ, _P],
    "dicp_lddmm_ode_self_fwd_rows_f32": [_P, _P, _I64, _I64, _I64, _INT, _DBL, _DBL, _P, _P, _P, _P,
                                         _P, _SZ, _P],
    "dicp_lddmm_euler_step_rows_f32": [_P, _P, _I64, _I64, _I64, _INT, _DBL, _DBL, _DBL, _P, _P, _P,
                                       _P, _SZ, _P],
    "dicp_lddmm_euler_step_phase_f32": [_INT, _P, _P, _P, _P, _I64, _I64, _I64, _INT, _DBL, _DBL, _DBL,
                                        _P, _P, _P, _P, _P, _SZ, _P],
    "dicp_lddmm_ode_self_fwd_ord_f32": [_P, _P, _I64, _I64, _I64, _INT, _DBL, _DBL, _P, _P, _P, _P, _P,
                                        _P, _SZ, _P],
    "dicp_lddmm_euler_step_ord_f32": [_P, _P, _I64, _I64, _I64, _INT, _DBL, _DBL, _DBL, _P, _P, _P, _P,
                                      _P, _SZ, _P],
    "dicp_lddmm_ode_self_bwd_part_f32": [_P, _P, _P, _P, _P, _I64, _INT, _DBL, _DBL, _INT, _INT, _P,
                                         _P, _P, _SZ, _P],
    "dicp_lddmm_ode_self_fwd_zs_f32": [_P, _P, _I64, _I64, _I64, _INT, _DBL, _DBL, _P, _P, _P, _P, _P,
                                       _P, _SZ, _P],
    "dicp_lddmm_euler_step_zs_f32": [_P, _P, _I64, _I64, _I64, _INT, _DBL, _DBL, _DBL, _P, _P, _P, _P,
                                     _P, _P, _SZ, _P],
    "dicp_lddmm_euler_adjoint_step_zs_f32": [_P, _P, _P, _P, _P, _I64, _INT, _DBL, _DBL, _DBL, _P, _P,
                                             _P, _P, _P, _P, _SZ, _P],
    "dicp_lddmm_ode_self_bwd_part_zs_f32": [_P, _P, _P, _P, _P, _I64, _INT, _DBL, _DBL, _INT, _INT, _P,
                                            _I64, _I64, _P, _P, _P, _SZ, _P],
    "dicp_gauss_red_grad_f32": [_INT, _P, _I64, _P, _I64, _INT, _P, _P, _P, _P, _P, _DBL, _P, _P, _SZ, _P],
    "dicp_kernel_ridge_cg_f32": [_P, _I64, _INT, _DBL, _DBL, _DBL, _P, _P, _INT, _INT, _P, _SZ, _P],
    "dicp_workspace_bytes": [_INT, _I64, _I64, _INT],
    "dicp_last_error": [],
    "dicp_version": [],
    "dicp_supports_dim": [_INT],
    "dicp_num_splits": [_INT, _I64, _I64],
    "dicp_set_option": [ctypes.c_char_p, _INT],
    "dicp_get_option": [ctypes.c_char_p, ctypes.POINTER(_INT)],
    "dicp_batch_begin": [],
    "dicp_batch_end": [_P],
    "dicp_batch_abort": [],
}
_RESTYPES = {"dicp_workspace_bytes": _SZ, "dicp_last_error": ctypes.c_char_p,
             "dicp_version": ctypes.c_char_p}

EXPORTED_SYMBOLS = tuple(_SIGNATURES)


class HipExtensionMissing(RuntimeError):
    pass


def lib():
    """Load (once) and return the native library; raise loudly if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise HipExtensionMissing(
                    f"difficp_amd: native library {LIB_PATH} is not built. Run "
                    "`python -c 'import __graft_entry__ as g; g.build()'` or "
                    "`make -C diff-icp_amd/csrc`. There is no CPU fallback.")
            handle = ctypes.CDLL(LIB_PATH)
            for name, args in _SIGNATURES.items():
                if os.environ.get("DICP_LIB_PATH") and not hasattr(handle, name):
                    continue  # older experiment build (tools/ab_libs.py) without this entry
                fn = getattr(handle, name)
                fn.argtypes = args
                fn.restype = _RESTYPES.get(name, _INT)
            _lib = handle
    return _lib


def version() -> str:
    return lib().dicp_version().decode()


def supports_dim(D: int) -> bool:
    return bool(lib().dicp_supports_dim(int(D)))


def get_option(name: str) -> int:
    """The library's current value of a tuning knob (dicp_get_option): the kernel variant an
    entry point will run is asked from the library, never mirrored on the Python side (a
    build with other -DDICP_* defaults, or a set_option between a forward and its backward,
    stays consistent)."""
    if name not in _PER_THREAD:
        hit = _OPT_CACHE.get(name)
        if hit is not None and hit[0] == _OPTION_EPOCH[0]:
            return hit[1]
    v = _INT(0)
    _check_rc(lib().dicp_get_option(name.encode(), ctypes.byref(v)), f"get_option({name})")
    if name not in _PER_THREAD:
        # process-wide knobs change only through set_option, which bumps the epoch (a ctypes
        # round trip less per zs_ok / variant query: ~200 per diff-ICP iteration)
        _OPT_CACHE[name] = (_OPTION_EPOCH[0], int(v.value))
    return int(v.value)


_OPT_CACHE = {}


# divergence-row reuse (dicp_lddmm_*_zs_f32): the forward's per-row sums zs_i = sum_j K z_ij
# feed the VJP's divergence-cotangent term (env DICP_ZS=0 turns it off, for A/B runs)
USE_ZS = os.environ.get("DICP_ZS", "1") != "0"


def zs_ok(eta) -> bool:
    """Whether the fused Euler steps can hand divergence rows from the forward to the VJP
    (eta = 0 with a packed forward -- fwd_alg 2, the default: ordered rows or, for whole passes
    from 20k points, symmetric 4-row; 5: symmetric 4-row; 6: ordered rows -- and the packed
    symmetric VJP)."""
    return USE_ZS and eta == 0 and get_option("fwd_alg") in (2, 5, 6) and get_option("bwd_alg") == 3


def _zs_buf(zs, rows, D, dev, name="zs_out"):
    if zs is None:
        return None
    if (not zs.is_contiguous() or tuple(zs.shape) != (rows, D) or zs.dtype != torch.float32
            or zs.device != dev):
        raise ValueError(f"{name} must be a contiguous float32 ({rows}, {D}) tensor on {dev}")
    return zs


class thread_option:
    """Context manager setting a per-host-thread library knob (_PER_THREAD) for a block."""

    name = None

    def __init__(self, value: int, name: str = None):
        self.value = int(value)
        if name is not None:
            self.name = name

    def __enter__(self):
        self.old = get_option(self.name)
        if self.old != self.value:
            set_option(self.name, self.value)
        return self

    def __exit__(self, *exc):
        if self.old != self.value:
            set_option(self.name, self.old)


class coord_mode(thread_option):
    """Context manager: the packed shooting kernels in original-unit coordinates (raw=True) or
    in scaled ones (library option coord_raw, per host thread)."""

    name = "coord_raw"

    def __init__(self, raw: bool):
        super().__init__(int(bool(raw)))
        self.raw = self.value


# per-host-thread knobs (keyed separately by their users; workspace sizes never depend on them)
_PER_THREAD = frozenset({"coord_raw", "batch_share"})

# bumped by every set_option of a process-wide knob: a kernel-variant change (fwd_alg,
# bwd_alg, pk_rp, split rounds, ...) makes results computed before it not bitwise what a
# recomputation gives, so caches of results (shooting.ShootCache) key on it
_OPTION_EPOCH = [0]


def option_epoch() -> int:
    return _OPTION_EPOCH[0]


def set_option(name: str, value: int):
    """Tuning knob (see include/difficp_hip.h dicp_set_option)."""
    _check_rc(lib().dicp_set_option(name.encode(), int(value)), f"set_option({name})")
    if name not in _PER_THREAD:     # every process-wide knob may change a workspace size
        _WS_BYTES.clear()
        _OPTION_EPOCH[0] += 1


def _zero_b_ok(eta) -> bool:
    """Whether a zero mG cotangent may be passed as NULL (the symmetric packed VJPs skip its
    terms); otherwise the caller materialises zeros."""
    return eta == 0 or get_option("bwd_eta_alg") == 2


def _bwd_name(eta, want_gq: bool, zero_b: bool) -> str:
    base = "ode_self_bwd_eta" if eta else "ode_self_bwd"
    if zero_b:
        return base + "_b0"
    return base if want_gq else base + "_gp"


def num_splits(kind: int, M: int, N: int) -> int:
    return int(lib().dicp_num_splits(int(kind), int(M), int(N)))


def _check_rc(rc: int, what: str):
    if rc != 0:
        msg = lib().dicp_last_error().decode()
        if rc == 2:
            raise NotImplementedError(f"{what}: {msg}")
        raise RuntimeError(f"{what} failed (status {rc}): {msg}")


def _dev(t: torch.Tensor, name: str) -> torch.Tensor:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if t.device.type != "cuda":
        raise RuntimeError(f"difficp_amd HIP kernels need device tensors; {name} is on {t.device} "
                           "(no CPU fallback)")
    if t.dtype != torch.float32:
        raise TypeError(f"{name}: expected float32, got {t.dtype}")
    return t.contiguous()


def _ptr(t):
    # a plain int: ctypes converts it for the c_void_p parameters without an object per call
    return None if t is None else t.data_ptr()


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _stream(device):
    """Handle of the current HIP stream of `device` (torch's current stream: concurrent frames
    set their own with torch.cuda.stream)."""
    if _raw_stream is not None:
        return _raw_stream(device.index if device.index is not None else torch.cuda.current_device())
    return torch.cuda.current_stream(device).cuda_stream


def _order(order, n: int, device):
    """Optional row visit order (int32 permutation of n rows, on the device) or None."""
    if order is None:
        return None
    if (not isinstance(order, torch.Tensor) or order.dtype != torch.int32 or order.numel() != n
            or order.device != device):
        raise ValueError(f"row order must be an int32 device tensor of {n} row indices")
    return order.contiguous()


# ---------------------------------------------------------------------------------------
# Optional live kernel accounting (bench.py): HIP events around each launch on the launch
# stream, algorithmic pair / flop / byte counts per launch.
# Algorithmic cost per ordered (row, column) pair for D = 3 (FMA = 2 flop; one exp2 per pair):
# the per-unit figures of SURVEY.md 8(d) where it gives one (KRed 15, fused ODE forward 33,
# fused VJP ~70), otherwise counted from the pair operators (csrc/lddmm_ops.hpp, gmm.hip).
# These price the OPERATION, not a kernel's instruction stream: the symmetric VJP
# (lddmm_sym.hpp) executes ~53 flop per ordered pair because it evaluates each unordered
# pair once, so its effective rate can exceed the rate of executed arithmetic.
FLOPS_PER_PAIR = {
    "gauss_red": 15, "ode_self_fwd": 33, "ode_self_fwd_eta": 70, "ode_self_bwd": 70, "ode_self_bwd_eta": 120,
    "ode_ext_fwd": 22, "ode_ext_bwd": (36 + 49) / 2, "gmm_estep": 37, "gmm_mstep": 31,
    "gmm_targets": 32, "ridge_cg": 15,
}
# Executed fp32 arithmetic per ordered pair where it differs from the algorithmic figure
# (FMA = 2 flop, from the hot loop's instruction counts, tools/isa_loop_stats.py): the
# symmetric pair-once VJP evaluates each unordered pair once.  bench.py reports the fraction
# of the peak on both counts (roofline.frac = algorithmic, roofline.frac_executed).
EXEC_FLOPS_PER_PAIR = {"ode_self_bwd": 53,
                       # the symmetric pair-once forward (from 20k points; the 6-row loop: 60
                       # v_pk_fma + 24 other v_pk + 18 scalar adds + 6 exp per step of 6
                       # unordered pairs = 306 flop, i.e. 25.5 per ordered pair)
                       "ode_self_fwd": 25.5}
# the gp-only VJP (last adjoint step when q0 needs no gradient): 32 of the 60 packed
# instructions of the full symmetric loop -> priced at that share of the full VJP's figure
FLOPS_PER_PAIR["ode_self_bwd_gp"] = round(70 * 32 / 60)
# zero momentum cotangent (first adjoint step): 40 of 60 packed instructions remain
FLOPS_PER_PAIR["ode_self_bwd_b0"] = round(70 * 40 / 60)
# forward without the momentum update (last step of a shooting whose p1 is unused): V, Z'
FLOPS_PER_PAIR["ode_self_fwd_nog"] = 33 - 14
# eta != 0 (logdet model), same pricing by packed-instruction share of the full loop: gp only
# 39 of 98 per column, zero mG cotangent 56 of 98; forward without mG 14 of 39
FLOPS_PER_PAIR["ode_self_bwd_eta_gp"] = round(120 * 39 / 98)
FLOPS_PER_PAIR["ode_self_bwd_eta_b0"] = round(120 * 56 / 98)
FLOPS_PER_PAIR["ode_self_fwd_eta_nog"] = round(70 * 14 / 39)


def flops_per_pair(name: str, D: int = 3) -> float:
    """The algorithmic figure of `name` at dimension D.  The table above is for D = 3; every
    term of the pair operators is a D-vector operation, counted from SURVEY.md Appendix A
    (FMA = 2): the fused forward (v, G, g) is 11 D flop per pair (33 at D = 3), KRed 5 D (15),
    the fused VJP's Appendix A.3 terms 31 D + 2 written out (95 at D = 3, which the table's
    ~70 prices with shared subexpressions) -- so the VJP family scales by (31 D + 2) / 95 and
    every other figure by D / 3."""
    f = FLOPS_PER_PAIR.get(name)
    if f is None or D == 3:
        return f
    if name.startswith("ode_self_bwd"):
        return f * (31 * D + 2) / 95.0
    return f * D / 3.0


class KernelProfile:
    """Context manager collecting (name, pairs, flops, bytes, start, end[, share]) per launch;
    a batched launch over several calls (LaunchBatcher) is one record per kernel name, whose
    time is the batch's time x that name's share of the batch's flops."""

    def __init__(self):
        self.records = []

    def __enter__(self):
        global _prof
        _prof = self
        return self

    def __exit__(self, *exc):
        global _prof
        _prof = None

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for rec in self.records:
            name, pairs, flops, nbytes, e0, e1 = rec[:6]
            share = rec[6] if len(rec) > 6 else 1.0
            d = out.setdefault(name, {"launches": 0, "pairs": 0, "flops": 0, "bytes": 0, "ms": 0.0})
            d["launches"] += 1
            d["pairs"] += pairs
            d["flops"] += flops
            d["bytes"] += nbytes
            d["ms"] += e0.elapsed_time(e1) * share
        return out


_prof = None


# per host thread: the LaunchBatcher (core/batching.py) its batchable launches go through
_tl = threading.local()
# the launches a LaunchBatcher may batch: the packed eta = 0 shooting passes (fwd_alg 2 /
# bwd_alg 3, the C-ABI's batchable paths, include/difficp_hip.h dicp_batch_begin)
BATCHABLE = frozenset({"ode_self_fwd", "ode_self_fwd_nog", "ode_self_bwd", "ode_self_bwd_b0",
                       "ode_self_bwd_gp"})


def _launch(name, pairs, nbytes, fn):
    b = getattr(_tl, "batcher", None)
    if b is not None and name in BATCHABLE:
        return b.submit(name, pairs, nbytes, fn)
    keep = getattr(_tl, "batch_keep", None)
    if keep is not None:
        # a batch is open on this thread: the call's launches run at the batch's end, so every
        # tensor the call captured (inputs, outputs the caller may drop, workspace) must stay
        # allocated until then -- a freed block could be handed to the next call of the batch
        keep.append(fn)
    if _prof is None:
        return fn()
    st = torch.cuda.current_stream()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record(st)
    r = fn()
    e1.record(st)
    _prof.records.append((name, int(pairs), int(pairs * FLOPS_PER_PAIR.get(name, 0)), int(nbytes), e0, e1))
    return r


_WS_BYTES = {}   # (kind, M, N, D) -> dicp_workspace_bytes; cleared by set_option
# Scratch workspaces reused per (stream, size): the launches of one stream run in order, so a
# workspace handed to the next call on the same stream is free by the time that call's kernels
# run -- one torch.empty less per library call (host floor, tools/host_floor.py).  Never for a
# call that may run inside a launch batch (a batch open on this thread, or a frame thread of
# the lockstep batches, whose calls from several frames share one stream and run together:
# each needs its own -- tests/test_gpu_batch.py caught the shared one), nor inside a graph
# capture; a few recent streams only (concurrent frames open a stream per Reg_opt call).  The
# cache is keyed by host thread too (ctypes releases the GIL, so two threads issuing calls on
# one stream could otherwise interleave the kernels of two multi-kernel calls on one buffer).
# A cached workspace is valid within ONE library call only: a workspace that must survive
# between calls (euler_step_phase_ws) is requested with exclusive=True and bypasses the cache.
_WS_CACHE = OrderedDict()
_WS_CACHE_MAX = 8
_ws_lock = threading.Lock()
# debugging aid: DICP_WS_POISON=1 fills every workspace with NaN bytes before its call, so a
# kernel reading workspace it did not write shows up as NaN instead of stale finite values
_WS_POISON = os.environ.get("DICP_WS_POISON", "0") != "0"


def _poison(ws):
    if _WS_POISON and ws is not None:
        ws.fill_(255)
    return ws


def _workspace(kind: int, M: int, N: int, D: int, device, exclusive: bool = False):
    key = (kind, int(M), int(N), int(D))
    nbytes = _WS_BYTES.get(key)
    if nbytes is None:
        nbytes = _WS_BYTES[key] = int(lib().dicp_workspace_bytes(kind, int(M), int(N), int(D)))
    if nbytes == 0:
        return None, 0
    keep = getattr(_tl, "batch_keep", None)
    if keep is not None:   # a batch open on this thread: the launch runs at its end
        ws = _poison(torch.empty(nbytes, dtype=torch.uint8, device=device))
        keep.append(ws)
        return ws, nbytes
    if getattr(_tl, "batcher", None) is not None:
        # a frame of lockstep launch batches (core/batching.py): its launch may be recorded
        # into one batch together with other frames' calls on the batcher's shared stream --
        # each call needs a workspace of its own (the call's closure keeps it alive)
        return _poison(torch.empty(nbytes, dtype=torch.uint8, device=device)), nbytes
    if exclusive or torch.cuda.is_current_stream_capturing():
        # a HIP-graph capture (core/shooting.py): the workspace must come from the graph's own
        # pool, never a cached tensor that could be freed while the graph still points at it;
        # exclusive: the caller keeps it across several library calls
        return _poison(torch.empty(nbytes, dtype=torch.uint8, device=device)), nbytes
    ck = (_stream(device), device.index, threading.get_ident())
    with _ws_lock:
        ws = _WS_CACHE.get(ck)
        if ws is not None:
            _WS_CACHE.move_to_end(ck)
    if ws is None or ws.numel() < nbytes:
        ws = torch.empty(nbytes, dtype=torch.uint8, device=device)
        with _ws_lock:
            _WS_CACHE[ck] = ws
            _WS_CACHE.move_to_end(ck)
            while len(_WS_CACHE) > _WS_CACHE_MAX:
                _WS_CACHE.popitem(last=False)
    return _poison(ws), int(ws.numel())


# ---------------------------------------------------------------------------------------
# Gaussian-kernel reductions
# ---------------------------------------------------------------------------------------
_RED_OUT_VEC = {KRED, GRADK, DDK, GENDK, HESSK, GRADLAPK, GRADKSCAL, GRADLAPKSCAL}


def gauss_red(op: int, x, y, sigma: float, b=None, c=None):
    """One Gaussian-kernel reduction (dicp_gauss_red_f32). Returns (M,D) or (M,)."""
    x = _dev(x, "x")
    y = _dev(y, "y")
    b = None if b is None else _dev(b, "b")
    c = None if c is None else _dev(c, "c")
    M, D = x.shape
    N = y.shape[0]
    if y.shape[1] != D:
        raise ValueError("x and y must have the same dimension")
    out = torch.empty((M, D) if op in _RED_OUT_VEC else (M,), device=x.device, dtype=torch.float32)
    if M == 0:
        return out
    ws, nb = _workspace(WS_RED, M, N, D, x.device)
    rc = _launch("gauss_red", M * N, 4 * (2 * M * D + 2 * N * D),
                 lambda: lib().dicp_gauss_red_f32(int(op), _ptr(x), M, _ptr(y), N, D, _ptr(b), _ptr(c),
                                  float(sigma), _ptr(out), _ptr(ws), nb, _stream(x.device)))
    _check_rc(rc, f"gauss_red(op={op})")
    return out


def gauss_red_grad(kind: int, x, y, sigma: float, r1=None, r2=None, c1=None, c2=None, cw=None):
    """One gradient reduction (dicp_gauss_red_grad_f32; include/difficp_hip.h lists the five
    pair formulas): rows x with optional row vectors r1, r2, columns y with optional column
    vectors c1, c2 and column scalar cw; None reads as zeros (cw: ones).  Returns (M, D)."""
    x = _dev(x, "x")
    y = _dev(y, "y")
    M, D = x.shape
    N = y.shape[0]
    if y.shape[1] != D:
        raise ValueError("x and y must have the same dimension")
    r1, r2 = (None if t is None else _dev(t, n) for t, n in ((r1, "r1"), (r2, "r2")))
    c1, c2 = (None if t is None else _dev(t, n) for t, n in ((c1, "c1"), (c2, "c2")))
    cw = None if cw is None else _dev(cw, "cw")
    for t, n, shp in ((r1, "r1", (M, D)), (r2, "r2", (M, D)), (c1, "c1", (N, D)), (c2, "c2", (N, D)),
                      (cw, "cw", (N,))):
        if t is not None and tuple(t.shape) != shp:
            raise ValueError(f"gauss_red_grad: {n} must be shaped {shp}")
    out = torch.empty((M, D), device=x.device, dtype=torch.float32)
    if M == 0:
        return out
    ws, nb = _workspace(WS_GRAD, M, N, D, x.device)
    rc = _launch("gauss_red_grad", M * N, 4 * (3 * M * D + 3 * N * D + N),
                 lambda: lib().dicp_gauss_red_grad_f32(int(kind), _ptr(x), M, _ptr(y), N, D, _ptr(r1), _ptr(r2),
                                                       _ptr(c1), _ptr(c2), _ptr(cw), float(sigma), _ptr(out),
                                                       _ptr(ws), nb, _stream(x.device)))
    _check_rc(rc, f"gauss_red_grad(kind={kind})")
    return out


def radius_count(x, y, R: float):
    """counts_i = #{j : |x_i - y_j|^2 <= R^2} (float32, exact integers), torch-exact distances
    (dicp_radius_count_f32)."""
    x = _dev(x, "x")
    y = _dev(y, "y")
    M, D = x.shape
    N = y.shape[0]
    if y.shape[1] != D:
        raise ValueError("x and y must have the same dimension")
    out = torch.empty((M,), device=x.device, dtype=torch.float32)
    if M == 0:
        return out
    ws, nb = _workspace(WS_RED, M, N, D, x.device)
    rc = _launch("radius_count", M * N, 4 * (M * D + N * D + M),
                 lambda: lib().dicp_radius_count_f32(_ptr(x), M, _ptr(y), N, D, float(R), _ptr(out),
                                                     _ptr(ws), nb, _stream(x.device)))
    _check_rc(rc, "radius_count")
    return out


# ---------------------------------------------------------------------------------------
# Fused LDDMM ODE
# ---------------------------------------------------------------------------------------
def ode_self_fwd(q, p, sigma: float, eta: float, want_div: bool, want_h: bool = False, order=None,
                 zs_out=None):
    """(v, mG, g rows, h rows) of the fused ODE (dicp_lddmm_ode_self_fwd_ord_f32); order: optional
    int32 row visit order (spatial grouping for the matrix-core forward, see spatial_order);
    zs_out: (M, D) divergence rows instead of h (dicp_lddmm_ode_self_fwd_zs_f32, eta = 0)."""
    q = _dev(q, "q")
    p = _dev(p, "p")
    M, D = q.shape
    dev = q.device
    order = _order(order, M, dev)
    if zs_out is not None:
        if want_h:
            raise ValueError("ode_self_fwd: zs_out replaces h (want_h must be False)")
        return ode_self_fwd_rows(q, p, 0, M, sigma, eta, want_div, order=order, zs_out=zs_out)
    v = torch.empty_like(q)
    mG = torch.empty_like(q)
    g = torch.empty(M, device=dev, dtype=torch.float32) if (want_div or eta != 0) else None
    h = torch.empty(M, device=dev, dtype=torch.float32) if want_h else None
    if M == 0:
        return v, mG, g, h
    ws, nb = _workspace(WS_ODE_SELF_FWD, M, M, D, dev)
    rc = _launch(("ode_self_fwd_eta" if eta else "ode_self_fwd"), M * M, 4 * M * (4 * D + 2),
                 lambda: lib().dicp_lddmm_ode_self_fwd_ord_f32(_ptr(q), _ptr(p), M, 0, M, D, float(sigma),
                                                               float(eta), _ptr(order), _ptr(v), _ptr(mG),
                                                               _ptr(g), _ptr(h), _ptr(ws), nb, _stream(dev)))
    _check_rc(rc, "ode_self_fwd")
    return v, mG, g, h


def euler_step(q, p, sigma: float, eta: float, dt: float, want_div: bool, q_out=None, p_out=None,
               g_out=None, order=None, want_p: bool = True, zs_out=None):
    """(q + dt v, p + dt mG, g rows or None) in one fused pass (dicp_lddmm_euler_step_ord_f32);
    q_out / p_out / g_out: optional contiguous destinations (must not overlap q, p); order:
    optional int32 row visit order (see ode_self_fwd); want_p=False: (q_next, None, g) -- the
    momentum update is not formed (the packed pass skips the sums that feed mG only);
    zs_out: optional (M, D) destination of the divergence rows (dicp_lddmm_euler_step_zs_f32,
    eta = 0)."""
    q = _dev(q, "q")
    p = _dev(p, "p")
    M, D = q.shape
    order = _order(order, M, q.device)
    zs_out = _zs_buf(zs_out, M, D, q.device)
    qn = torch.empty_like(q) if q_out is None else q_out
    pn = (torch.empty_like(q) if p_out is None else p_out) if want_p else None
    for t, name in ((qn, "q_out"), (pn, "p_out")):
        if t is None:
            continue
        if not t.is_contiguous() or t.shape != q.shape or t.dtype != torch.float32:
            raise ValueError(f"{name} must be a contiguous float32 tensor shaped like q")
    g = None
    if want_div or eta != 0:
        g = torch.empty(M, device=q.device, dtype=torch.float32) if g_out is None else g_out
        if not g.is_contiguous() or g.shape != (M,) or g.dtype != torch.float32:
            raise ValueError("g_out must be a contiguous float32 (M,) tensor")
    if M == 0:
        return qn, pn, g
    ws, nb = _workspace(WS_ODE_SELF_FWD, M, M, D, q.device)
    name = ("ode_self_fwd_eta" if eta else "ode_self_fwd") + ("" if want_p else "_nog")
    rc = _launch(name, M * M, 4 * M * (4 * D + 1),
                 lambda: lib().dicp_lddmm_euler_step_zs_f32(_ptr(q), _ptr(p), M, 0, M, D, float(sigma),
                                                            float(eta), float(dt), _ptr(order), _ptr(qn),
                                                            _ptr(pn), _ptr(g), _ptr(zs_out), _ptr(ws), nb,
                                                            _stream(q.device)))
    _check_rc(rc, "euler_step")
    return qn, pn, g


def euler_adjoint_step(q, p, lq, lp, gdiv, sigma: float, eta: float, dt: float, addq=None, addp=None,
                       want_lq: bool = True, zs=None):
    """(lq + dt gq + addq, lp + dt gp + addp) with (gq, gp) the ODE VJP for cotangents
    (lq, lp, gdiv) -- one fused pass (dicp_lddmm_euler_adjoint_step_f32).  want_lq=False:
    (None, lp_next) only -- the gq half of the pair algebra is skipped.  lp=None: a zero
    momentum cotangent (the b terms of the pair algebra are skipped).  zs: the forward's
    divergence rows at q (euler_step zs_out; dicp_lddmm_euler_adjoint_step_zs_f32)."""
    q = _dev(q, "q")
    p = _dev(p, "p")
    lq = _dev(lq, "lq")
    if lp is None and not _zero_b_ok(eta):
        lp = torch.zeros_like(q)        # this VJP variant has no zero-cotangent shortcut
    lp = None if lp is None else _dev(lp, "lp")
    gdiv = None if gdiv is None else _dev(gdiv.reshape(-1)[:1], "gdiv")
    addq = None if addq is None else _dev(addq, "addq")
    addp = None if addp is None else _dev(addp, "addp")
    M, D = q.shape
    zs = _zs_buf(zs, M, D, q.device, "zs")
    lqn = torch.empty_like(q) if want_lq else None
    lpn = torch.empty_like(q)
    if M == 0:
        return lqn, lpn
    ws, nb = _workspace(WS_ODE_SELF_BWD, M, M, D, q.device)
    name = _bwd_name(eta, want_lq, lp is None)
    rc = _launch(name, M * M, 4 * M * (8 * D if want_lq else 7 * D),
                 lambda: lib().dicp_lddmm_euler_adjoint_step_zs_f32(
                     _ptr(q), _ptr(p), _ptr(lq), _ptr(lp), _ptr(gdiv), M, D, float(sigma), float(eta),
                     float(dt), _ptr(addq), _ptr(addp), _ptr(zs), _ptr(lqn), _ptr(lpn), _ptr(ws), nb,
                     _stream(q.device)))
    _check_rc(rc, "euler_adjoint_step")
    return lqn, lpn


def ode_self_bwd(q, p, gv, gmG, gdiv, sigma: float, eta: float):
    """gdiv: None or a device tensor with one element (cotangent of sum_i g_i)."""
    q = _dev(q, "q")
    p = _dev(p, "p")
    gv = _dev(gv, "gv")
    gmG = _dev(gmG, "gmG")
    gdiv = None if gdiv is None else _dev(gdiv.reshape(-1)[:1], "gdiv")
    M, D = q.shape
    gq = torch.empty_like(q)
    gp = torch.empty_like(q)
    if M == 0:
        return gq, gp
    ws, nb = _workspace(WS_ODE_SELF_BWD, M, M, D, q.device)
    rc = _launch(("ode_self_bwd_eta" if eta else "ode_self_bwd"), M * M, 4 * M * 6 * D,
                 lambda: lib().dicp_lddmm_ode_self_bwd_f32(_ptr(q), _ptr(p), _ptr(gv), _ptr(gmG), _ptr(gdiv), M,
                                           D, float(sigma), float(eta), _ptr(gq), _ptr(gp),
                                           _ptr(ws), nb, _stream(q.device)))
    _check_rc(rc, "ode_self_bwd")
    return gq, gp


def ode_ext_fwd(x, q, p, sigma: float, eta: float, want_div: bool):
    x = _dev(x, "x")
    q = _dev(q, "q")
    p = _dev(p, "p")
    N, D = x.shape
    M = q.shape[0]
    vx = torch.empty_like(x)
    gx = torch.empty(N, device=x.device, dtype=torch.float32) if want_div else None
    if N == 0:
        return vx, gx
    ws, nb = _workspace(WS_ODE_EXT_FWD, M, N, D, x.device)
    rc = _launch("ode_ext_fwd", N * M, 4 * (N * (2 * D + 1) + 2 * M * D),
                 lambda: lib().dicp_lddmm_ode_ext_fwd_f32(_ptr(x), N, _ptr(q), _ptr(p), M, D, float(sigma),
                                          float(eta), _ptr(vx), _ptr(gx), _ptr(ws), nb,
                                          _stream(x.device)))
    _check_rc(rc, "ode_ext_fwd")
    return vx, gx


def ode_ext_bwd(x, q, p, gvx, gdiv, sigma: float, eta: float, gq, gp):
    """Returns gx; ACCUMULATES the (q, p) gradients into gq, gp (contiguous, in place)."""
    x = _dev(x, "x")
    q = _dev(q, "q")
    p = _dev(p, "p")
    gvx = _dev(gvx, "gvx")
    gdiv = None if gdiv is None else _dev(gdiv.reshape(-1)[:1], "gdiv")
    if not (gq.is_contiguous() and gp.is_contiguous()):
        raise ValueError("gq/gp accumulators must be contiguous")
    N, D = x.shape
    M = q.shape[0]
    gx = torch.empty_like(x)
    if N == 0:
        return gx
    ws, nb = _workspace(WS_ODE_EXT_BWD, M, N, D, x.device)
    rc = _launch("ode_ext_bwd", 2 * N * M, 4 * (3 * N * D + 6 * M * D),
                 lambda: lib().dicp_lddmm_ode_ext_bwd_f32(_ptr(x), N, _ptr(q), _ptr(p), M, D, float(sigma),
                                          float(eta), _ptr(gvx), _ptr(gdiv), _ptr(gx), _ptr(gq),
                                          _ptr(gp), _ptr(ws), nb, _stream(x.device)))
    _check_rc(rc, "ode_ext_bwd")
    return gx


# ---------------------------------------------------------------------------------------
# GMM EM passes
# ---------------------------------------------------------------------------------------
def gmm_estep(X, mu, w2, mu2, sigma: float, lgn: float, want_stats: bool, hint=None):
    """hint: optional (N,) float32 device tensor, the rows' expected log2 LSE (e.g. the T2 of the
    previous EM step over the same rows) -- dicp_gmm_estep_hint_f32's shift hint."""
    X = _dev(X, "X")
    mu = _dev(mu, "mu")
    w2 = _dev(w2, "w2")
    mu2 = _dev(mu2, "mu2")
    N, D = X.shape
    C = mu.shape[0]
    dev = X.device
    if hint is not None:
        hint = _dev(hint, "hint")
        if hint.shape != (N,):
            raise ValueError(f"gmm_estep: hint must be shaped ({N},)")
    T = torch.empty(N, device=dev, dtype=torch.float32)
    T2 = torch.empty(N, device=dev, dtype=torch.float32)
    stats = torch.empty((N, D + 4), device=dev, dtype=torch.float32) if want_stats else None
    if N == 0:
        return T, T2, stats
    ws, nb = _workspace(WS_GMM_ESTEP, N, C, D, dev)
    rc = _launch("gmm_estep", N * C, 4 * (N * (2 * D + 6) + C * (D + 2)),
                 lambda: lib().dicp_gmm_estep_hint_f32(_ptr(X), N, _ptr(mu), _ptr(w2), _ptr(mu2), C, D,
                                                       float(sigma), float(lgn), _ptr(hint), _ptr(T), _ptr(T2),
                                                       _ptr(stats), _ptr(ws), nb, _stream(dev)))
    _check_rc(rc, "gmm_estep")
    return T, T2, stats


def gmm_mstep(X, T2, mu, w2, sigma: float):
    X = _dev(X, "X")
    T2 = _dev(T2, "T2")
    mu = _dev(mu, "mu")
    w2 = _dev(w2, "w2")
    N, D = X.shape
    C = mu.shape[0]
    colstats = torch.empty((C, D + 1), device=X.device, dtype=torch.float32)
    if N == 0:
        # neutral statistics of an empty shard (a rank that owns no points in a sharded
        # atlas): log-weight -inf, mean 0; the cross-rank combine in GMM.EM_step gives them
        # weight exp(-inf) = 0
        colstats[:, 0] = float("-inf")
        colstats[:, 1:] = 0.0
        return colstats
    ws, nb = _workspace(WS_GMM_MSTEP, N, C, D, X.device)
    rc = _launch("gmm_mstep", N * C, 4 * (N * (D + 1) + 2 * C * (D + 1)),
                 lambda: lib().dicp_gmm_mstep_f32(_ptr(X), _ptr(T2), N, _ptr(mu), _ptr(w2), C, D, float(sigma),
                                  _ptr(colstats), _ptr(ws), nb, _stream(X.device)))
    _check_rc(rc, "gmm_mstep")
    return colstats


def gmm_targets(X, T2, mu_old, w2_old, sigma_old: float, mu_new, lpi_new):
    X = _dev(X, "X")
    T2 = _dev(T2, "T2")
    mu_old = _dev(mu_old, "mu_old")
    w2_old = _dev(w2_old, "w2_old")
    mu_new = _dev(mu_new, "mu_new")
    lpi_new = _dev(lpi_new, "lpi_new")
    N, D = X.shape
    C = mu_old.shape[0]
    rows = torch.empty((N, D + 4), device=X.device, dtype=torch.float32)
    if N == 0:
        return rows
    ws, nb = _workspace(WS_GMM_TARGETS, N, C, D, X.device)
    rc = _launch("gmm_targets", N * C, 4 * (N * (2 * D + 5) + C * (2 * D + 3)),
                 lambda: lib().dicp_gmm_targets_f32(_ptr(X), _ptr(T2), N, _ptr(mu_old), _ptr(w2_old),
                                    float(sigma_old), _ptr(mu_new), _ptr(lpi_new), C, D,
                                    _ptr(rows), _ptr(ws), nb, _stream(X.device)))
    _check_rc(rc, "gmm_targets")
    return rows


# ---------------------------------------------------------------------------------------
# Kernel ridge solve (v2p)
# ---------------------------------------------------------------------------------------
CG_DONE_NAMES = {0: "running", 1: "converged", 2: "breakdown"}


def kernel_ridge_cg(x, v, sigma: float, alpha: float, eps: float = 1e-6, maxiter: int = 5000,
                    chunk: int = 32):
    """b with (K(x,x) + alpha I) b = v by conjugate gradients on the device
    (dicp_kernel_ridge_cg_f32; KeOps LazyTensor.solve semantics, kernel.py:239-241: one CG on
    the flattened (M,D) system, stop when |r|^2 < M*D*eps^2).  Launches `chunk` iterations at
    a time and reads the 16-byte device status between chunks.  Returns (b, info) with
    info = {"status", "iterations", "residual2", "threshold"}."""
    x = _dev(x, "x")
    v = _dev(v, "v")
    M, D = x.shape
    if v.shape != x.shape:
        raise ValueError("v must have the shape of x")
    b = torch.zeros_like(v)
    info = {"status": "converged", "iterations": 0, "residual2": 0.0, "threshold": 0.0}
    if M == 0:
        return b, info
    ws, nb = _workspace(WS_RIDGE_CG, M, 0, D, x.device)
    st = _stream(x.device)
    done, it = 0, 0
    start = 1
    while it < maxiter:
        n = min(int(chunk), maxiter - it)
        rc = _launch("ridge_cg", M * M * n, 4 * (3 * M * D + 4 * M * D) * n,
                     lambda: lib().dicp_kernel_ridge_cg_f32(_ptr(x), M, D, float(sigma), float(alpha),
                                                            float(eps), _ptr(v), _ptr(b), start, n,
                                                            _ptr(ws), nb, st))
        _check_rc(rc, "kernel_ridge_cg")
        start = 0
        head = ws[:16].cpu()          # one 16-byte read per chunk (synchronises the stream)
        done, it = (int(t) for t in head[:8].view(torch.int32))
        if done:
            break
    rr, thr = (float(t) for t in head[8:16].view(torch.float32))
    info = {"status": CG_DONE_NAMES.get(done, str(done)) if done else "maxiter",
            "iterations": it, "residual2": rr, "threshold": thr}
    return b, info


# ---------------------------------------------------------------------------------------
# Row-split of one frame over ranks (core/rowsplit.py)
# ---------------------------------------------------------------------------------------
def ode_self_fwd_rows(q, p, row0: int, nrows: int, sigma: float, eta: float, want_div: bool,
                      want_h: bool = False, order=None, zs_out=None):
    """Rows [row0, row0 + nrows) of ode_self_fwd against all columns
    (dicp_lddmm_ode_self_fwd_ord_f32).  Returns (v, mG, g, h) for the slice; order: optional
    int32 visit order of the slice's rows (indices into the slice); zs_out: (nrows, D)
    divergence rows instead of h (dicp_lddmm_ode_self_fwd_zs_f32; h is then None)."""
    q = _dev(q, "q")
    p = _dev(p, "p")
    M, D = q.shape
    dev = q.device
    order = _order(order, nrows, dev)
    if zs_out is not None:
        if want_h:
            raise ValueError("ode_self_fwd_rows: zs_out replaces h (want_h must be False)")
        zs_out = _zs_buf(zs_out, nrows, D, dev)
        v = torch.empty((nrows, D), device=dev, dtype=torch.float32)
        mG = torch.empty_like(v)
        g = torch.empty(nrows, device=dev, dtype=torch.float32) if (want_div or eta != 0) else None
        if nrows == 0:
            return v, mG, g, None
        ws, nb = _workspace(WS_ODE_SELF_FWD_ROWS, nrows, M, D, dev)
        rc = _launch("ode_self_fwd", nrows * M, 4 * (nrows * (3 * D + 1) + 2 * M * D),
                     lambda: lib().dicp_lddmm_ode_self_fwd_zs_f32(_ptr(q), _ptr(p), M, int(row0), int(nrows), D,
                                                                  float(sigma), float(eta), _ptr(order), _ptr(v),
                                                                  _ptr(mG), _ptr(g), _ptr(zs_out), _ptr(ws), nb,
                                                                  _stream(dev)))
        _check_rc(rc, "ode_self_fwd_zs")
        return v, mG, g, None
    v = torch.empty((nrows, D), device=dev, dtype=torch.float32)
    mG = torch.empty_like(v)
    g = torch.empty(nrows, device=dev, dtype=torch.float32) if (want_div or eta != 0) else None
    h = torch.empty(nrows, device=dev, dtype=torch.float32) if want_h else None
    if nrows == 0:
        return v, mG, g, h
    ws, nb = _workspace(WS_ODE_SELF_FWD_ROWS, nrows, M, D, dev)
    rc = _launch(("ode_self_fwd_eta" if eta else "ode_self_fwd"), nrows * M, 4 * (nrows * (2 * D + 2) + 2 * M * D),
                 lambda: lib().dicp_lddmm_ode_self_fwd_ord_f32(_ptr(q), _ptr(p), M, int(row0), int(nrows), D,
                                                               float(sigma), float(eta), _ptr(order), _ptr(v),
                                                               _ptr(mG), _ptr(g), _ptr(h), _ptr(ws), nb,
                                                               _stream(dev)))
    _check_rc(rc, "ode_self_fwd_rows")
    return v, mG, g, h


def euler_step_rows(q, p, row0: int, nrows: int, sigma: float, eta: float, dt: float,
                    want_div: bool, q_out=None, p_out=None, order=None, want_p: bool = True,
                    zs_out=None):
    """Rows [row0, row0 + nrows) of euler_step (dicp_lddmm_euler_step_ord_f32):
    (q + dt v, p + dt mG, g) for the slice; q_out / p_out: optional contiguous (nrows, D);
    order: optional int32 visit order of the slice's rows; want_p=False: p_next is None (not
    formed, as euler_step); zs_out: optional (nrows, D) divergence rows of the slice."""
    q = _dev(q, "q")
    p = _dev(p, "p")
    M, D = q.shape
    dev = q.device
    order = _order(order, nrows, dev)
    zs_out = _zs_buf(zs_out, nrows, D, dev)
    qn = torch.empty((nrows, D), device=dev, dtype=torch.float32) if q_out is None else q_out
    pn = (torch.empty((nrows, D), device=dev, dtype=torch.float32) if p_out is None else p_out) if want_p else None
    for t, name in ((qn, "q_out"), (pn, "p_out")):
        if t is None:
            continue
        if not t.is_contiguous() or tuple(t.shape) != (nrows, D) or t.dtype != torch.float32:
            raise ValueError(f"{name} must be a contiguous float32 ({nrows}, {D}) tensor")
    g = torch.empty(nrows, device=dev, dtype=torch.float32) if (want_div or eta != 0) else None
    if nrows == 0:
        return qn, pn, g
    ws, nb = _workspace(WS_ODE_SELF_FWD_ROWS, nrows, M, D, dev)
    name = ("ode_self_fwd_eta" if eta else "ode_self_fwd") + ("" if want_p else "_nog")
    rc = _launch(name, nrows * M, 4 * (nrows * (4 * D + 1) + 2 * M * D),
                 lambda: lib().dicp_lddmm_euler_step_zs_f32(_ptr(q), _ptr(p), M, int(row0), int(nrows), D,
                                                            float(sigma), float(eta), float(dt), _ptr(order),
                                                            _ptr(qn), _ptr(pn), _ptr(g), _ptr(zs_out), _ptr(ws),
                                                            nb, _stream(dev)))
    _check_rc(rc, "euler_step_rows")
    return qn, pn, g


def euler_step_phase_ws(nrows: int, M: int, D: int, device):
    """A workspace for the two calls of euler_step_phase (the partial slots of phase 0 must
    survive until phase 1 has merged them, whatever runs on the stream in between: a fresh
    buffer, never the per-stream cache)."""
    return _workspace(WS_ODE_SELF_FWD_PHASED, nrows, M, D, device, exclusive=True)[0]


def euler_step_phase(phase: int, q_loc, p_loc, q, p, row0: int, nrows: int, sigma: float, eta: float,
                     dt: float, q_out, p_out=None, g_out=None, zs_out=None, ws=None):
    """One of the two column phases of a row-split Euler step of rows [row0, row0 + nrows)
    (dicp_lddmm_euler_step_phase_f32): phase 0 = the rows (q_loc, p_loc) against themselves,
    partial sums into ws; phase 1 = the rows of (q, p) against the other points, then
    q_out = q_row + dt v, p_out = p_row + dt mG (None: not formed), g_out, zs_out (None: not
    formed) -- the one-pass slice step up to fp32 summation order.  Both calls take the same
    output tensors and the same ws (euler_step_phase_ws)."""
    ref = q_loc if phase == 0 else q
    ref = _dev(ref, "q")
    D = ref.shape[1]
    dev = ref.device
    if phase == 0:
        q_loc, p_loc = _dev(q_loc, "q_loc"), _dev(p_loc, "p_loc")
        if q is not None:
            q, p = _dev(q, "q"), _dev(p, "p")
    else:
        q, p = _dev(q, "q"), _dev(p, "p")
    M = q.shape[0] if q is not None else None
    if M is None:
        raise ValueError("euler_step_phase: q (M, D) is needed for the sizes")
    for t, name, shape in ((q_out, "q_out", (nrows, D)), (p_out, "p_out", (nrows, D)),
                           (g_out, "g_out", (nrows,)), (zs_out, "zs_out", (nrows, D))):
        if t is None:
            continue
        if not t.is_contiguous() or tuple(t.shape) != shape or t.dtype != torch.float32:
            raise ValueError(f"{name} must be a contiguous float32 {shape} tensor")
    if q_out is None:
        raise ValueError("q_out is required")
    if nrows == 0:
        return q_out
    if ws is None:
        raise ValueError("euler_step_phase: pass the same ws (euler_step_phase_ws) to both phases")
    nb = ws.numel()
    name = ("ode_self_fwd_eta" if eta else "ode_self_fwd") + ("" if p_out is not None else "_nog")
    ncols = nrows if phase == 0 else M - nrows
    rc = _launch(name, nrows * ncols, 4 * (nrows * (4 * D + 1) + 2 * ncols * D),
                 lambda: lib().dicp_lddmm_euler_step_phase_f32(
                     int(phase), _ptr(q_loc), _ptr(p_loc), _ptr(q), _ptr(p), M, int(row0), int(nrows), D,
                     float(sigma), float(eta), float(dt), _ptr(q_out), _ptr(p_out), _ptr(g_out),
                     _ptr(zs_out), _ptr(ws), nb, _stream(dev)))
    _check_rc(rc, f"euler_step_phase({phase})")
    return q_out


def ode_self_bwd_part(q, p, gv, gmG, gdiv, sigma: float, eta: float, part: int, nparts: int,
                      want_gq: bool = True, zs=None, zrow0: int = 0, gq_out=None, gp_out=None):
    """Part `part` of `nparts` of ode_self_bwd (dicp_lddmm_ode_self_bwd_part_zs_f32): (gq, gp)
    over a pair subset; the sum over the parts is the full VJP.  want_gq=False: (None, gp).
    zs: the forward's divergence rows of rows [zrow0, zrow0 + len(zs)) (this rank's slice).
    gq_out / gp_out: optional contiguous (M, D) destinations."""
    q = _dev(q, "q")
    p = _dev(p, "p")
    gv = _dev(gv, "gv")
    if gmG is None and not _zero_b_ok(eta):
        gmG = torch.zeros_like(q)       # this VJP variant has no zero-cotangent shortcut
    gmG = None if gmG is None else _dev(gmG, "gmG")
    gdiv = None if gdiv is None else _dev(gdiv.reshape(-1)[:1], "gdiv")
    M, D = q.shape
    zn = 0
    if zs is not None:
        zn = int(zs.shape[0])
        zs = _zs_buf(zs, zn, D, q.device, "zs")
    gq = (torch.empty_like(q) if gq_out is None else _zs_buf(gq_out, M, D, q.device, "gq_out")) \
        if want_gq else None
    gp = torch.empty_like(q) if gp_out is None else _zs_buf(gp_out, M, D, q.device, "gp_out")
    if M == 0:
        return gq, gp
    ws, nb = _workspace(WS_ODE_SELF_BWD_PART, M, nparts, D, q.device)
    pairs = (M * M) // nparts
    name = _bwd_name(eta, want_gq, gmG is None)
    rc = _launch(name, pairs, 4 * M * 6 * D,
                 lambda: lib().dicp_lddmm_ode_self_bwd_part_zs_f32(_ptr(q), _ptr(p), _ptr(gv), _ptr(gmG),
                                                                   _ptr(gdiv), M, D, float(sigma), float(eta),
                                                                   int(part), int(nparts), _ptr(zs), int(zrow0),
                                                                   zn, _ptr(gq), _ptr(gp), _ptr(ws), nb,
                                                                   _stream(q.device)))
    _check_rc(rc, "ode_self_bwd_part")
    return gq, gp


class batch:
    """Context manager around dicp_batch_begin / dicp_batch_end(stream) on this host thread:
    the batchable library calls made inside record their launches, which are issued grouped
    on `stream` at exit (include/difficp_hip.h).  An exception inside discards the batch."""

    def __init__(self, stream_handle):
        self.stream = stream_handle

    def __enter__(self):
        _check_rc(lib().dicp_batch_begin(), "batch_begin")
        # workspaces allocated by the recorded calls stay referenced until the batch is issued
        # (a freed block could be handed to the next call of the same batch)
        self._prev_keep = getattr(_tl, "batch_keep", None)
        _tl.batch_keep = []
        return self

    def __exit__(self, exc_type, *exc):
        try:
            if exc_type is not None:
                lib().dicp_batch_abort()
                return False
            _check_rc(lib().dicp_batch_end(self.stream), "batch_end")
            return False
        finally:
            # issued on self.stream: blocks freed now are reused in that stream's order
            _tl.batch_keep = self._prev_keep
