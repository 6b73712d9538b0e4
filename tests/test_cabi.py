"""The C-ABI library loads and exports every symbol include/difficp_hip.h declares (CPU,
no compute calls); the Python binding binds exactly those symbols."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "difficp_hip.h")
LIB = os.path.join(ROOT, "diff-icp_amd", "libdifficp_hip.so")


def declared():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(dicp_\w+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        pytest.fail(f"{LIB} not built (run __graft_entry__.build())")
    return ctypes.CDLL(LIB)


def test_header_symbols_exported(lib):
    names = declared()
    assert len(names) >= 12
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_binding_matches_header():
    from difficp_amd import _lib
    assert set(_lib.EXPORTED_SYMBOLS) == set(declared())


def test_host_only_entry_points(lib):
    lib.dicp_version.restype = ctypes.c_char_p
    assert b"gfx950" in lib.dicp_version()
    assert lib.dicp_supports_dim(3) == 1 and lib.dicp_supports_dim(2) == 1
    assert lib.dicp_supports_dim(7) == 0
    lib.dicp_last_error.restype = ctypes.c_char_p
    # invalid arguments are rejected before any device work, with a message
    rc = lib.dicp_gauss_red_f32(2, None, ctypes.c_int64(5), None, ctypes.c_int64(5), 3, None, None,
                                ctypes.c_double(1.0), None, None, ctypes.c_size_t(0), None)
    assert rc == 1
    assert b"invalid" in lib.dicp_last_error()


def test_no_cpu_fallback():
    """The product refuses host tensors instead of computing on the CPU."""
    import torch
    from difficp_amd import _lib
    x = torch.rand(4, 3)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        _lib.gauss_red(_lib.KRED, x, x, 0.5, b=x)


def test_option_epoch_bumps_on_kernel_variant_change(lib):
    """ShootCache keys on _lib.option_epoch(): a set_option of a kernel variant between two
    shootings makes the cached trajectory a miss; the per-thread coordinate
    mode does not bump it (it is keyed separately)."""
    from difficp_amd import _lib
    e0 = _lib.option_epoch()
    old = _lib.get_option("bwd_alg")
    _lib.set_option("bwd_alg", old)
    assert _lib.option_epoch() == e0 + 1
    with _lib.coord_mode(True):
        pass
    assert _lib.option_epoch() == e0 + 1


def test_batch_scope_host_contract(lib):
    """dicp_batch_begin / dicp_batch_end / dicp_batch_abort (include/difficp_hip.h), host side
    only: one open batch per thread, end without begin is an error, an empty batch issues
    nothing, calls recorded with M = 0 record nothing, abort discards."""
    import ctypes as C
    lib.dicp_batch_end.argtypes = [C.c_void_p]
    lib.dicp_last_error.restype = C.c_char_p
    assert lib.dicp_batch_end(None) != 0                  # no open batch
    assert lib.dicp_batch_begin() == 0
    assert lib.dicp_batch_begin() != 0                    # already open on this thread
    assert b"already open" in lib.dicp_last_error()
    # an empty shooting step (M = 0) validates and records nothing
    f = lib.dicp_lddmm_euler_step_zs_f32
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_int64, C.c_int64, C.c_int, C.c_double,
                  C.c_double, C.c_double, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                  C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]
    assert f(None, None, 0, 0, 0, 3, 0.1, 0.0, 0.1, None, None, None, None, None, None, 0, None) == 0
    assert lib.dicp_batch_end(None) == 0                  # nothing recorded: nothing issued
    assert lib.dicp_batch_begin() == 0
    assert lib.dicp_batch_abort() == 0
    assert lib.dicp_batch_end(None) != 0                  # the abort closed it
    assert lib.dicp_batch_abort() == 0                    # no-op without a batch
