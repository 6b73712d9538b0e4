"""EM passes on inputs that exercise the single-sweep LSE's re-referencing (csrc/gmm.hip
lse_rowred_kernel): the shift of a column chunk is the maximum over its first 64 columns, so
rows whose nearby columns come later re-reference their sums (tile-end or per pair,
csrc/gmm.hip kLseSlack; both modes forced in test_estep_reref_modes).

  * E-step (rows = points, columns = components): the first components sit far from the
    points of one cluster (~2^-1000 of the near ones);
  * M-step (rows = components, columns = points): the first points are far from the
    components of the other cluster;
  * the wave-per-row merge of many column chunks (the M-step at the atlas shape);
  * small sigma against the sample's spacing (events in most tiles), with and without the
    shift hint (exact, and 300 too high: the chunk partials' normalised store);
  * the many-component E-step's bound shift (no sample, no events) and the exact re-sum of the
    rows whose LSE ends far below it (rows 30 sigma from every component, stale hints).

Criterion: err vs the float64 oracle (oracle/torch_ref.py em_step, pinned by the
reference's EM goldens) <= max(2e-5, 2 x the float32 oracle's own deviation)."""
import math

import pytest
import torch

from conftest import rel_err
from oracle import torch_ref as R

pytestmark = pytest.mark.gpu

OPT = {"mu": True, "w": True, "sigma": True, "eta0": False}


def _two_clusters(N, C, far, dev, seed=0):
    g = torch.Generator().manual_seed(seed)
    X = torch.cat([torch.tensor([far, far, far]) + 0.05 * torch.randn(N // 2, 3, generator=g),
                   0.05 * torch.randn(N - N // 2, 3, generator=g)])
    mu = torch.cat([torch.tensor([far, far, far]) + 0.05 * torch.randn(C // 2, 3, generator=g),
                    0.05 * torch.randn(C - C // 2, 3, generator=g)])
    # E-step: the first 256 components are the far cluster's; M-step: the first N/2 points
    return X.to(dev), mu.to(dev)


@pytest.mark.parametrize("N,C,far,sigma", [(4000, 600, 3.0, 0.05), (3000, 520, 1.0, 0.2),
                                           (200000, 512, 2.0, 0.03)])
def test_em_rescaled_shift(dev, N, C, far, sigma):
    from difficp_amd.core.GMM import GaussianMixtureUnif
    X, mu0 = _two_clusters(N, C, far, dev)
    GM = GaussianMixtureUnif(mu0, sigma=sigma, spec={"device": dev, "dtype": torch.float32})
    GM.to_optimize = dict(OPT)
    st64 = dict(mu=mu0.double(), w=torch.zeros(C, dtype=torch.float64, device=dev), sigma=sigma)
    st32 = dict(mu=mu0.clone(), w=torch.zeros(C, device=dev), sigma=sigma)
    for it in range(2):
        Y, Cfe, FE = GM.EM_step(X)
        Y64, Cfe64, FE64, n64 = R.em_step(X.double(), st64["mu"], st64["w"], st64["sigma"], OPT)
        Y32, Cfe32, FE32, n32 = R.em_step(X, st32["mu"], st32["w"], st32["sigma"], OPT)
        tol = lambda a32, a64: max(2e-5, 2 * rel_err(a32, a64))
        assert rel_err(Y, Y64) < tol(Y32, Y64), (it, rel_err(Y, Y64))
        assert rel_err(GM.mu, n64["mu"]) < tol(n32["mu"], n64["mu"]), it
        assert rel_err(GM.w, n64["w"]) < tol(n32["w"], n64["w"]), (it, rel_err(GM.w, n64["w"]))
        assert abs(GM.sigma - n64["sigma"]) < max(1e-5, 2 * abs(n32["sigma"] - n64["sigma"]) / n64["sigma"]) * n64["sigma"]
        for a, a64, a32 in ((float(FE), float(FE64), float(FE32)), (float(Cfe), float(Cfe64), float(Cfe32))):
            assert abs(a - a64) <= max(2e-5, 2 * abs(a32 - a64) / abs(a64)) * abs(a64), (it, a, a64, a32)
        st64, st32 = n64, n32
        assert torch.isfinite(GM.w).all() and torch.isfinite(Y).all()


def _estep64(X, mu, lpi, sigma):
    """float64 E-step rows (GMM.py:260-282, :296, :303, :312-314): T, T2 and the (D+4) stats."""
    D = X.shape[1]
    lgn = D * (math.log(sigma) + 0.5 * math.log(2 * math.pi))
    D2 = ((X[:, None, :] - mu[None]) ** 2).sum(-1)
    t = lpi[None] - D2 / (2 * sigma ** 2) - lgn
    T = t.logsumexp(1)
    lg = t - T[:, None]
    gam = lg.exp()
    live = gam > 0
    wsum = lambda v: torch.where(live, gam * v, torch.zeros_like(gam)).sum(1)
    stats = torch.cat([gam @ mu, wsum((mu * mu).sum(-1)[None])[:, None], wsum(lg)[:, None],
                       wsum(lpi[None].expand_as(gam))[:, None], wsum(D2)[:, None]], 1)
    return T, (T + lgn) / math.log(2), stats, lgn


@pytest.mark.parametrize("D", [2, 3])
@pytest.mark.parametrize("case", ["plain", "dead", "far_first", "chunks", "uniform"])
def test_estep_stats_match_fp64(dev, D, case):
    """Every output of dicp_gmm_estep_f32 (T, T2 and the D+4 stats, include/difficp_hip.h)
    against float64 rows: random weights; dead components (w = -inf, 350 of them, kLseDead);
    a far cluster in the first columns; many column chunks (the wave-per-row merge; sigma small
    against the shift sample's spacing: re-references)."""
    from difficp_amd import _lib
    g = torch.Generator().manual_seed(11 * D + len(case))
    N, C, sigma = {"plain": (3000, 700, 0.1), "dead": (3000, 900, 0.1), "far_first": (2500, 800, 0.05),
                   "chunks": (300, 60000, 0.02), "uniform": (2000, 20000, 0.05)}[case]
    X = torch.rand(N, D, generator=g, dtype=torch.float64)
    mu = torch.rand(C, D, generator=g, dtype=torch.float64)
    w = 0.3 * torch.randn(C, generator=g, dtype=torch.float64)
    if case == "uniform":     # equal weights: the tiles' sum e v formed as v0 sum e
        w = torch.zeros(C, dtype=torch.float64)
    if case == "dead":
        w[:300] = -math.inf
        w[600:650] = -math.inf
    if case == "far_first":
        mu[:400] += 3.0
    X, mu = X.float().double(), mu.float().double()
    lpi = w - w.logsumexp(0)
    T64, T264, st64, lgn = _estep64(X, mu, lpi, sigma)
    f = lambda t: t.float().to(dev).contiguous()
    T, T2, st = _lib.gmm_estep(f(X), f(mu), f(lpi / math.log(2)), f((mu * mu).sum(-1)), sigma, lgn, True)
    T, T2, st = T.cpu().double(), T2.cpu().double(), st.cpu().double()
    assert rel_err(T, T64) < 1e-5 and rel_err(T2, T264) < 1e-5
    for k in range(D + 4):
        assert torch.isfinite(st[:, k]).all(), k
        # the entropy and the squared distance are sums of O(1/sigma^2)-scaled logits (2e-5)
        assert rel_err(st[:, k], st64[:, k]) < (2e-5 if k >= D else 1e-5), (k, rel_err(st[:, k], st64[:, k]))


@pytest.mark.parametrize("case", ["plain", "dead", "far_first", "chunks", "uniform"])
def test_lse_packed_rows_bitwise(dev, case):
    """The packed-row E and M passes (lse_rowred_pk_kernel, option lse_pk 1: two rows per
    v_pk_fma_f32) against the scalar-row kernel (lse_pk 0): same rows, same order, same fmas --
    bitwise, including dead components and re-referenced tiles."""
    from difficp_amd import _lib
    g = torch.Generator().manual_seed(len(case))
    N, C, sigma = {"plain": (3001, 701, 0.1), "dead": (3000, 900, 0.1), "far_first": (2500, 800, 0.05),
                   "chunks": (301, 60000, 0.02), "uniform": (2001, 20000, 0.05)}[case]
    X = torch.rand(N, 3, generator=g)
    mu = torch.rand(C, 3, generator=g)
    w = 0.3 * torch.randn(C, generator=g, dtype=torch.float64)
    if case == "uniform":
        w = torch.zeros(C, dtype=torch.float64)
    if case == "dead":
        w[:300] = -math.inf
    if case == "far_first":
        mu[:400] += 3.0
    lpi = (w - w.logsumexp(0)).float()
    f = lambda t: t.float().to(dev).contiguous()
    args = (f(X), f(mu), f(lpi / math.log(2)), f((mu * mu).sum(-1)), sigma, 0.5)
    old = _lib.get_option("lse_pk")
    out = {}
    try:
        for pk in (0, 1):
            _lib.set_option("lse_pk", pk)
            T, T2, st = _lib.gmm_estep(*args, True)
            col = _lib.gmm_mstep(args[0], T2, args[1], args[2], sigma)
            out[pk] = (T, T2, st, col)
    finally:
        _lib.set_option("lse_pk", old)
    for a, b in zip(out[0], out[1]):
        assert torch.equal(torch.nan_to_num(a, nan=7.0), torch.nan_to_num(b, nan=7.0))


@pytest.mark.parametrize("adapt", [0, 1, 1000])
@pytest.mark.parametrize("hinted", [False, True])
def test_estep_reref_modes(dev, adapt, hinted):
    """The E-step at sigma 0.01 over 40k random components (the 64-column shift sample sits
    hundreds of log2 units below most rows' nearest component): per-pair re-referencing from the
    start (lse_adapt 0), the adaptive default (1), tile-end only (1000); with and without the
    shift hint (the float64 T2, and the hint shifted up by 300: clamped) -- every output against
    float64 rows."""
    from difficp_amd import _lib
    g = torch.Generator().manual_seed(5)
    N, C, D, sigma = 1500, 40000, 3, 0.01
    X = torch.rand(N, D, generator=g, dtype=torch.float64).float().double()
    mu = torch.rand(C, D, generator=g, dtype=torch.float64).float().double()
    w = 0.3 * torch.randn(C, generator=g, dtype=torch.float64)
    lpi = w - w.logsumexp(0)
    T64, T264, st64, lgn = _estep64(X, mu, lpi, sigma)
    f = lambda t: t.float().to(dev).contiguous()
    old = _lib.get_option("lse_adapt")
    try:
        _lib.set_option("lse_adapt", adapt)
        hints = [None] if not hinted else [f(T264), f(T264 + 300.0)]
        for hint in hints:
            T, T2, st = _lib.gmm_estep(f(X), f(mu), f(lpi / math.log(2)), f((mu * mu).sum(-1)), sigma,
                                       lgn, True, hint=hint)
            T, T2, st = T.cpu().double(), T2.cpu().double(), st.cpu().double()
            assert rel_err(T, T64) < 1e-5 and rel_err(T2, T264) < 1e-5
            for k in range(D + 4):
                assert torch.isfinite(st[:, k]).all(), k
                assert rel_err(st[:, k], st64[:, k]) < (2e-5 if k >= D else 1e-5), (k, rel_err(st[:, k], st64[:, k]))
    finally:
        _lib.set_option("lse_adapt", old)



@pytest.mark.parametrize("bound", [1, 0])
def test_estep_bound_shift_fixup(dev, bound):
    """The many-component E-step's bound shift (csrc/gmm.hip lse_bound_kernel, option
    lse_bound): half of the rows lie 30 sigma from every component (their LSE ends far below
    the shift: listed and summed again exactly by lse_fixup_kernel), and hints exact, 100 too
    high (a shift 92 above the LSE: listed) and 300 too high (capped at the bound) -- every
    output against float64 rows, with the bound shift on and off."""
    from difficp_amd import _lib
    g = torch.Generator().manual_seed(21)
    N, C, D, sigma = 1000, 20000, 3, 0.01
    X = torch.rand(N, D, generator=g, dtype=torch.float64)
    X[N // 2:, 0] += 1.3
    X = X.float().double()
    mu = torch.rand(C, D, generator=g, dtype=torch.float64).float().double()
    w = 0.3 * torch.randn(C, generator=g, dtype=torch.float64)
    lpi = w - w.logsumexp(0)
    T64, T264, st64, lgn = _estep64(X, mu, lpi, sigma)
    # the float32 restatement's own deviation (the far rows' entropy sums cancel more)
    _, _, st32, _ = _estep64(X.float(), mu.float(), lpi.float(), sigma)
    f = lambda t: t.float().to(dev).contiguous()
    old = _lib.get_option("lse_bound")
    try:
        _lib.set_option("lse_bound", bound)
        for hint in (None, f(T264), f(T264 + 100.0), f(T264 + 300.0)):
            T, T2, st = _lib.gmm_estep(f(X), f(mu), f(lpi / math.log(2)), f((mu * mu).sum(-1)), sigma,
                                       lgn, True, hint=hint)
            T, T2, st = T.cpu().double(), T2.cpu().double(), st.cpu().double()
            assert rel_err(T, T64) < 1e-5 and rel_err(T2, T264) < 1e-5
            for k in range(D + 4):
                assert torch.isfinite(st[:, k]).all(), k
                tol = max(2e-5 if k >= D else 1e-5, 2 * rel_err(st32[:, k].double(), st64[:, k]))
                assert rel_err(st[:, k], st64[:, k]) < tol, (k, rel_err(st[:, k], st64[:, k]), tol)
    finally:
        _lib.set_option("lse_bound", old)


def test_em_hint_history_independent(dev):
    """the E-step's shift hint comes only from the same (unmodified) point set, so
    an EM run gives bitwise the same result and step count whether or not the model ran EM
    on another point set of the same size before."""
    import copy
    from difficp_amd.core.GMM import GaussianMixtureUnif
    X, mu0 = _two_clusters(20000, 256, 1.0, dev, seed=3)
    Xo, _ = _two_clusters(20000, 256, 1.0, dev, seed=4)
    GM = GaussianMixtureUnif(mu0, sigma=0.02, spec={"device": dev, "dtype": torch.float32})
    GM.to_optimize = dict(OPT)
    G1, G2 = copy.deepcopy(GM), copy.deepcopy(GM)
    G2.EM_step(Xo)                     # history: an E-step over another set of the same N
    G2.mu, G2.sigma, G2.w = G1.mu.clone(), G1.sigma, G1.w.clone()
    r1 = G1.EM_optimization(X, max_iterations=6, tol=1e-9)
    r2 = G2.EM_optimization(X, max_iterations=6, tol=1e-9)
    assert torch.equal(G1.mu, G2.mu) and G1.sigma == G2.sigma and torch.equal(G1.w, G2.w)
    for a, b in zip(r1, r2):
        if isinstance(a, torch.Tensor):
            assert torch.equal(a, b)
        else:
            assert a == b
    # within one EM loop the hint is used (same X object, unmodified)
    assert G1._estep_hint[0]() is X


@pytest.mark.parametrize("where", ["x", "mu"])
def test_estep_nan_propagates(dev, where):
    """a NaN point (or component) comes out as NaN in T / T2 (not as an empty row
    with T = -inf), the way the reference's torch EM propagates it; the other rows' T are those
    of the same call without the NaN (row-wise independent)."""
    from difficp_amd import _lib
    g = torch.Generator().manual_seed(9)
    N, C, D, sigma = 3000, 700, 3, 0.05
    X = torch.rand(N, D, generator=g)
    mu = torch.rand(C, D, generator=g)
    lpi = torch.full((C,), -math.log(C))
    f = lambda t: t.to(dev).contiguous()
    Xn, mun = X.clone(), mu.clone()
    if where == "x":
        Xn[17, 1] = float("nan")
    else:
        mun[300, 0] = float("nan")
    outs = []
    for XX, mm in ((X, mu), (Xn, mun)):
        T, T2, st = _lib.gmm_estep(f(XX), f(mm), f(lpi / math.log(2)), f((mm * mm).sum(-1)), sigma, 0.0, True)
        outs.append((T.cpu(), T2.cpu(), st.cpu()))
    (T, T2, st), (Tn, T2n, stn) = outs
    if where == "x":
        assert torch.isnan(Tn[17]) and torch.isnan(T2n[17]), (Tn[17], T2n[17])
        keep = torch.arange(N) != 17
        assert torch.isfinite(Tn[keep]).all()
        assert rel_err(Tn[keep], T[keep]) < 1e-6
    else:
        # every row's LSE reads the NaN component
        assert torch.isnan(Tn).all() and torch.isnan(T2n).all()
