"""BASELINE configs[3] / [4] shapes on one GPU.

  * EM at the C4 shape (32 frames x 20k = 640k points, C = 512) and the C5 structure shape
    (64 frames x 7.5k = 480k points, C = 256): two full EM steps (E, M, targets, free
    energy; GMM.py:236-325) against the oracle's dense float64 EM step run on the device
    (oracle/torch_ref.py em_step, pinned by the reference goldens), with the SURVEY 8(c)
    criterion  err <= max(2e-5, 2 x the float32 oracle's own deviation);
  * one atlas_c4-shaped diff-ICP iteration (4 frames x 20k, C = 512, ICP_atlas.py:269-298):
    bitwise deterministic across fresh runs, concurrent frames == the sequential frame loop,
    and the free energy does not increase across GMM_opt / Reg_opt.
"""
import math

import pytest
import torch

from conftest import rel_err
from oracle import torch_ref as R

pytestmark = pytest.mark.gpu

OPT = {"mu": True, "w": True, "sigma": True, "eta0": False}


def _atlas_points(K, N, S, dev):
    from difficp_amd import workloads
    if S == 1:
        return torch.cat(workloads.atlas_frames(K, N, seed=0), 0).to(dev)
    fr = workloads.multi_structure_frames(K, S, N, seed=0)
    return torch.cat([f[0] for f in fr], 0).to(dev)     # structure 0 of every frame


@pytest.mark.parametrize("K,N,C,S", [(32, 20000, 512, 1), (64, 7500, 256, 4)], ids=["C4", "C5"])
def test_em_steps_at_atlas_shape(dev, K, N, C, S):
    from difficp_amd.core.GMM import GaussianMixtureUnif
    X = _atlas_points(K, N, S, dev)
    g = torch.Generator().manual_seed(7)
    mean, std = X.mean(0), X.std()
    mu0 = (mean + 0.05 * std * torch.randn(C, 3, generator=g).to(dev)).contiguous()
    sig0 = 0.25 * float(std)                                  # reinitialize_GMM, PSR.py:143-167
    GM = GaussianMixtureUnif(mu0, sigma=sig0, spec={"device": dev, "dtype": torch.float32})
    GM.to_optimize = dict(OPT)
    st64 = dict(mu=mu0.double(), w=torch.zeros(C, dtype=torch.float64, device=dev), sigma=sig0)
    st32 = dict(mu=mu0.clone(), w=torch.zeros(C, device=dev), sigma=sig0)
    for it in range(2):
        Y, Cfe, FE = GM.EM_step(X)
        Y64, Cfe64, FE64, n64 = R.em_step(X.double(), st64["mu"], st64["w"], st64["sigma"], OPT)
        Y32, Cfe32, FE32, n32 = R.em_step(X, st32["mu"], st32["w"], st32["sigma"], OPT)
        tol = lambda a32, a64: max(2e-5, 2 * rel_err(a32, a64))
        assert rel_err(Y, Y64) < tol(Y32, Y64), (it, rel_err(Y, Y64))
        assert rel_err(GM.mu, n64["mu"]) < tol(n32["mu"], n64["mu"]), it
        assert rel_err(GM.w, n64["w"]) < tol(n32["w"], n64["w"]), it
        assert abs(GM.sigma - n64["sigma"]) < max(1e-5, 2 * abs(n32["sigma"] - n64["sigma"])) * n64["sigma"]
        for a, a64, a32 in ((float(FE), float(FE64), float(FE32)), (float(Cfe), float(Cfe64), float(Cfe32))):
            assert abs(a - a64) <= max(2e-5, 2 * abs(a32 - a64) / abs(a64)) * abs(a64), (it, a, a64, a32)
        st64, st32 = n64, n32
        del Y64, Y32
    # sum_c gamma_nc = 1 for every n: the targets are convex combinations of the new centroids
    lo, hi = GM.mu.min(0).values, GM.mu.max(0).values
    assert bool(((Y >= lo - 1e-5) & (Y <= hi + 1e-5)).all())


def _c4_run(dev, conc, iters=2, share=0):
    from difficp_amd import workloads
    psr = workloads.build_atlas(4, 20000, 512, dev, seed=0)
    psr.concurrent_frames = conc
    psr.batch_share = share
    fes = [psr.FE]
    for _ in range(iters):
        psr.GMM_opt(max_iterations=10, tol=1e-3)
        fes.append(psr.FE)
        psr.Reg_opt(tol=1e-3, nmax=1)
        fes.append(psr.FE)
    return fes, [a.detach().cpu().clone() for a in psr.a0], \
        [psr.x1[k, 0].detach().cpu().clone() for k in range(4)], psr.GMMi[0].mu.cpu().clone()


def test_atlas_c4_iteration_deterministic_concurrent_monotone(dev):
    # sequential runs with the 4 concurrent frames' default geometry (batch_share 4: the
    # 4-row kernels at 20k): concurrency itself changes no bit
    seq1 = _c4_run(dev, 1, share=4)
    seq2 = _c4_run(dev, 1, share=4)
    conc = _c4_run(dev, 4)
    for other in (seq2, conc):
        assert other[0] == seq1[0]                       # identical FE sequence
        for a, b in zip(seq1[1] + seq1[2] + [seq1[3]], other[1] + other[2] + [other[3]]):
            assert torch.equal(a, b)
    fes = seq1[0]
    for f0, f1 in zip(fes[:-1], fes[1:]):              # FE never increases (PSR.py:234-235)
        assert f1 <= f0 + 1e-6 * abs(f0), fes
