"""ORACLE -- test / cpu-baseline infrastructure only.  ctypes wrapper of build/liboracle.so
(the C restatement in difficp_ref.c).  Inputs/outputs are CPU float32 tensors."""
import ctypes
import os
import subprocess

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_PATH):
            subprocess.run(["make", "-C", _HERE], check=True, capture_output=True)
        L = ctypes.CDLL(_PATH)
        P, I64, I, Dd = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_double
        L.oracle_ode_self_fwd.argtypes = [P, P, I64, I, Dd, P, P, P]
        L.oracle_ode_self_bwd.argtypes = [P, P, P, P, Dd, I64, I, Dd, P, P]
        L.oracle_gmm_estep.argtypes = [P, I64, P, P, I64, I, Dd, P, P]
        _lib = L
    return _lib


def _c(t):
    return t.detach().to(dtype=torch.float32, device="cpu").contiguous()


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


def ode_self_fwd(q, p, sigma):
    q, p = _c(q), _c(p)
    M, D = q.shape
    v, mG, g = torch.empty_like(q), torch.empty_like(q), torch.empty(M)
    lib().oracle_ode_self_fwd(_p(q), _p(p), M, D, float(sigma), _p(v), _p(mG), _p(g))
    return v, mG, g


def ode_self_bwd(q, p, a, b, gam, sigma):
    q, p, a, b = _c(q), _c(p), _c(a), _c(b)
    M, D = q.shape
    gq, gp = torch.empty_like(q), torch.empty_like(q)
    lib().oracle_ode_self_bwd(_p(q), _p(p), _p(a), _p(b), float(gam), M, D, float(sigma), _p(gq), _p(gp))
    return gq, gp


def gmm_estep(X, mu, w, sigma):
    X, mu, w = _c(X), _c(mu), _c(w)
    N, D = X.shape
    T, gD2 = torch.empty(N), torch.empty(N)
    lib().oracle_gmm_estep(_p(X), N, _p(mu), _p(w), mu.shape[0], D, float(sigma), _p(T), _p(gD2))
    return T, gD2
