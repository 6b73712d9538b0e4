"""Launch batching (include/difficp_hip.h dicp_batch_begin / dicp_batch_end, csrc/batch.hpp)
and the lockstep frame batches of the atlas (core/batching.py, DiffPSR.batch_frames).

* Every call recorded in a batch computes bitwise what it computes alone: the packed forward
  steps (with / without divergence rows, mG-less last step, first step with zs) and the packed
  symmetric VJPs (full, zero mG cotangent, gp only; 2 and 4 rows per lane; scaled and raw
  coordinates), for frames of different sizes in one batch (different split counts, column
  groups, stage counts).
* A call whose path has no batched form fails the whole batch loudly.
* An atlas Reg_opt with the frames in lockstep launch batches is bitwise the sequential
  frame loop (PSR.py:528-569), and FE-monotone.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

SIG = 0.1


def _lib():
    from difficp_amd import _lib
    return _lib


def _frame(M, seed, dev):
    g = torch.Generator().manual_seed(seed)
    q = torch.rand(M, 3, generator=g).to(dev)
    p = (0.01 * torch.randn(M, 3, generator=g)).to(dev)
    a = torch.randn(M, 3, generator=g).to(dev)
    b = torch.randn(M, 3, generator=g).to(dev)
    gd = torch.full((1,), 0.7, device=dev)
    return q, p, a, b, gd


def _calls(L, fr, zs):
    """The launch forms of one frame's shooting (each returns its outputs as a list); zs: the
    frame's divergence rows, precomputed (read by the adjoint forms)."""
    q, p, a, b, gd = fr
    return [
        lambda: (lambda z: list(L.ode_self_fwd(q, p, SIG, 0.0, True, zs_out=z)[:3]) + [z])(torch.empty_like(q)),
        lambda: (lambda z: list(L.euler_step(q, p, SIG, 0.0, 0.1, True, zs_out=z)) + [z])(torch.empty_like(q)),
        lambda: [L.euler_step(q, p, SIG, 0.0, 0.1, True, want_p=False)[0]],
        lambda: list(L.euler_adjoint_step(q, p, a, b, gd, SIG, 0.0, 0.1, zs=zs)),
        lambda: list(L.euler_adjoint_step(q, p, a, None, gd, SIG, 0.0, 0.1, zs=zs)),
        lambda: [L.euler_adjoint_step(q, p, a, b, gd, SIG, 0.0, 0.1, want_lq=False, zs=zs)[1]],
        lambda: list(L.ode_self_bwd(q, p, a, b, gd, SIG, 0.0)),
    ]


@pytest.mark.parametrize("raw", [False, True])
@pytest.mark.parametrize("sizes", [(3001, 3001, 3001), (20000, 7777, 1, 300, 20000), (70001, 20000)])
def test_batched_calls_bitwise_equal_single(dev, sizes, raw):
    L = _lib()
    frames = [_frame(M, 100 + i, dev) for i, M in enumerate(sizes)]
    st = torch.cuda.current_stream()
    with L.coord_mode(raw):
        zss = []
        for fr in frames:
            z = torch.empty_like(fr[0])
            L.euler_step(fr[0], fr[1], SIG, 0.0, 0.1, True, zs_out=z)
            zss.append(z)
        for form in range(7):
            alone = [[t.clone() for t in _calls(L, fr, z)[form]()] for fr, z in zip(frames, zss)]
            torch.cuda.synchronize()
            outs = []
            with L.batch(st.cuda_stream):
                for fr, z in zip(frames, zss):
                    outs.append(_calls(L, fr, z)[form]())
            torch.cuda.synchronize()
            for i, (o, a) in enumerate(zip(outs, alone)):
                assert len(o) == len(a)
                for x, y in zip(o, a):
                    assert torch.equal(x, y), (form, i, sizes[i])


def test_batch_rejects_unbatchable_call(dev):
    """The eta != 0 symmetric VJP has no batched form: the call fails loudly, the batch is
    discarded (the eta = 0 step recorded before it never runs), the thread stays usable."""
    L = _lib()
    q, p, a, b, gd = _frame(5000, 7, dev)
    st = torch.cuda.current_stream()
    qn = torch.full_like(q, 123.0)
    with pytest.raises(RuntimeError):
        with L.batch(st.cuda_stream):
            L.euler_step(q, p, SIG, 0.0, 0.1, True, q_out=qn)
            L.ode_self_bwd(q, p, a, b, gd, SIG, 1e-3)
    torch.cuda.synchronize()
    assert bool((qn == 123.0).all())       # discarded: nothing of the batch was issued
    qn2, _, _ = L.euler_step(q, p, SIG, 0.0, 0.1, True)
    torch.cuda.synchronize()
    assert torch.isfinite(qn2).all()


@pytest.mark.parametrize("K,N,groups,share", [(6, 3000, 2, 1), (5, 2500, 1, 1), (6, 20000, 2, 0)])
def test_atlas_reg_opt_batched_bitwise_sequential(dev, K, N, groups, share):
    """DiffPSR.Reg_opt with the frames in lockstep launch batches == the sequential frame loop
    (PSR.py:528-569) bitwise: momenta, final trajectories and losses of every frame.
    share 0: the batched launches sized for the group (geometry hint batch_share = frames per
    group, csrc/batch.hpp) == the sequential loop run with the same hint."""
    from difficp_amd import workloads
    per = -(-K // groups)
    res = {}
    for mode in ("seq", "batched"):
        torch.manual_seed(0)
        psr = workloads.build_atlas(K, N, 64, dev, seed=3)
        if mode == "seq":
            psr.concurrent_frames = 1
            psr.batch_frames = False
            psr.batch_share = per if share == 0 else 1   # the batched run's geometry
        else:
            psr.concurrent_frames = groups
            psr.batch_frames = True
            psr.batch_share = share
        psr.GMM_opt(max_iterations=3, tol=1e-3)
        FE0 = psr.FE
        psr.Reg_opt(tol=1e-3, nmax=2)
        torch.cuda.synchronize()
        res[mode] = ([a.clone() for a in psr.a0], [s.Q.clone() for s in psr.shoot], list(psr.regloss),
                     psr.FE, FE0, getattr(psr, "batch_stats", None))
    (a_s, Q_s, r_s, FE_s, _, _), (a_b, Q_b, r_b, FE_b, FE0, stats) = res["seq"], res["batched"]
    for k in range(K):
        assert torch.equal(a_s[k], a_b[k]) and torch.equal(Q_s[k], Q_b[k]), k
    assert r_s == r_b and FE_s == FE_b
    assert FE_b <= FE0 + 1e-6 * abs(FE0)
    assert stats is not None and stats["batches"] > 0 and stats["calls"] >= stats["batches"]
    # lockstep: most batched launches carry several frames
    assert stats["calls"] / stats["batches"] > 1.5
