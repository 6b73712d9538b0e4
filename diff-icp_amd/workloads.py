"""Synthetic workloads of the headline configurations (BASELINE.json configs)
and the PSR iteration they are measured on.  The drivers reproduce the semantics of the
reference's api/ICP_two_set.py:138-288 (two-set) and api/ICP_atlas.py:124-298 (atlas):
one iteration = GMM_opt(max_repeat_GMM, tol) + Reg_opt(tol, nmax=1).

    C2  two-set 3D 50k vs 50k   C3  two-set 3D 200k vs 200k
    C4  atlas 32 frames x 20k 3D, shared GMM (C=512), frames sharded over ranks
    C5  64 frames x 4 structures x 7.5k 3D, one GMM (C=256) per structure
"""
from __future__ import annotations

import math

import torch

from .core.GMM import GaussianMixtureUnif
from .core.LDDMM import LDDMMModel
from .core.PSR import DiffPSR


def _gmm_cloud(n, ncent, sig, g, D=3):
    cent = torch.rand(ncent, D, generator=g)
    lab = torch.randint(0, ncent, (n,), generator=g)
    return cent[lab] + sig * torch.randn(n, D, generator=g)


def _phi(x, amp, perm=None):
    """Smooth synthetic deformation x + amp sin(2 pi x_perm) (perm: a cyclic shift of the axes)."""
    if perm is None:
        perm = [(d + 1) % x.shape[1] for d in range(x.shape[1])]
    return x + amp * torch.sin(2 * math.pi * x[:, list(perm)])


def two_set_points(N, seed=0, D=3):
    """C2/C3 inputs: xB from a 64-centre GMM in D dimensions (sigma 0.02); xA = phi(xB) +
    N(0, 0.005^2).  D = 2 is the planar form of the same generator (the reference's examples
    are 2D: diffICP_basic.py, the Chui sets)."""
    g = torch.Generator().manual_seed(seed)
    xB = _gmm_cloud(N, 64, 0.02, g, D)
    xA = _phi(xB, 0.03) + 0.005 * torch.randn(N, D, generator=g)
    return xA.float().contiguous(), xB.float().contiguous()


def atlas_frames(K, N, seed=0):
    """C4 inputs: K frames, each phi_k(template sample of N points), a_k ~ U[0.01, 0.04]."""
    g = torch.Generator().manual_seed(seed)
    frames = []
    for k in range(K):
        gk = torch.Generator().manual_seed(seed * 1000 + k + 1)
        tpl = _gmm_cloud(N, 64, 0.02, gk)
        a = 0.01 + 0.03 * torch.rand(1, generator=gk).item()
        frames.append(_phi(tpl, a).float().contiguous())
    return frames


def multi_structure_frames(K, S, N, seed=0):
    """C5 inputs: K frames x S structures of N points (structure s = shifted cloud)."""
    out = []
    for k in range(K):
        gk = torch.Generator().manual_seed(seed * 1000 + k + 1)
        a = 0.01 + 0.03 * torch.rand(1, generator=gk).item()
        fr = []
        for s in range(S):
            tpl = _gmm_cloud(N, 16, 0.02, gk) * 0.5 + 0.5 * torch.tensor([s % 2, (s // 2) % 2, 0.0])
            fr.append(_phi(tpl, a).float().contiguous())
        out.append(fr)
    return out


def build_two_set(N, device, seed=0, sigma_gmm=0.05, sigma_lddmm=0.1, lam=1e3, nt=10,
                  scheme="Euler", version="hybrid", v2p_args=None, D=3):
    """ICP_two_set (ICP_two_set.py:176-226): GMM with mu = xB, w frozen, sigma optimised;
    LDDMM hybrid (withlogdet, gradcomponent False), Euler nt=10, dense support.
    version="logdet" is the exact ICP_two_set model (gradcomponent=True, ICP_two_set.py:203-207;
    SURVEY C2'): its a0 is initialised by v2p, here the device ridge CG (v2p_args)."""
    spec = {"device": device, "dtype": torch.float32}
    xA, xB = two_set_points(N, seed, D)
    G = GaussianMixtureUnif(xB.to(device), sigma=sigma_gmm, spec=spec)
    G.to_optimize = {"mu": False, "sigma": True, "w": False, "eta0": False}
    LM = LDDMMModel(sigma=sigma_lddmm, D=D, lambd=lam, version=version, scheme=scheme, nt=nt, spec=spec)
    psr = DiffPSR(xA.to(device), G, LM, dataspec=spec, compspec=spec, v2p_args=v2p_args)
    psr.printstuff = False
    return psr


def build_atlas(K, N, C, device, comm=None, seed=0, sigma_lddmm=0.1, lam=1e3, nt=10,
                scheme="Euler", S=1):
    """ICP_atlas (ICP_atlas.py:170-260): one GMM per structure (C components, mu/sigma/w
    optimised, reinitialize_GMM), LDDMM hybrid Euler nt=10, dense support."""
    spec = {"device": device, "dtype": torch.float32}
    if S == 1:
        x = [f.to(device) for f in atlas_frames(K, N, seed)]
    else:
        x = [[f.to(device) for f in fr] for fr in multi_structure_frames(K, S, N, seed)]
    G = GaussianMixtureUnif(torch.zeros(C, 3), spec=spec)
    G.to_optimize = {"mu": True, "sigma": True, "w": True, "eta0": False}
    LM = LDDMMModel(sigma=sigma_lddmm, D=3, lambd=lam, version="hybrid", scheme=scheme, nt=nt, spec=spec)
    torch.manual_seed(seed)
    psr = DiffPSR(x, G, LM, dataspec=spec, compspec=spec, comm=comm)
    psr.printstuff = False
    psr.reinitialize_GMM()
    return psr


def psr_iteration(psr, max_repeat_GMM=10, tol=1e-3):
    """One diff-ICP iteration (ICP_two_set.py:254-282, ICP_atlas.py:269-298)."""
    psr.GMM_opt(max_iterations=max_repeat_GMM, tol=tol)
    psr.Reg_opt(tol=tol, nmax=1)
