"""Shared body of the ShootCache stale-hit regression test (CPU spec and GPU)."""
import torch


def shoot_cache_stale_check(LM, M, D, dev, rounds=8):
    """Shoot fresh same-shape q0 tensors with equal (zero) p0 through one model, freeing each
    q0 in between (its storage becomes reusable by the allocator); every result must equal a
    cache-free shooting of the same q0, and none may be a cache hit.  Then a repeated shooting
    of one live q0 must hit and still be bitwise right.  Returns the model's cache."""
    from difficp_amd.core.LDDMM import LDDMMModel
    ref = LDDMMModel(sigma=LM.sigma, D=D, lambd=LM.lam, version="hybrid", scheme=LM.scheme,
                     nt=LM.nt, spec={"device": dev, "dtype": torch.float32})
    ref.shoot_cache = None
    g = torch.Generator().manual_seed(17)
    cache = LM.shoot_cache
    h0 = cache.hits
    p0 = torch.zeros(M, D, device=dev)
    for _ in range(rounds):
        q0 = torch.rand(M, D, generator=g).to(dev)
        sh = LM.Shoot(q0, p0.clone())
        r = ref.Shoot(q0, p0.clone())
        assert torch.equal(sh.Q, r.Q) and torch.equal(sh.C, r.C)
        del q0, sh, r
    assert cache.hits == h0                    # never a hit on different content
    q0 = torch.rand(M, D, generator=g).to(dev)
    p1 = 0.05 * torch.randn(M, D, generator=g).to(dev)
    a = LM.Shoot(q0, p1)
    b = LM.Shoot(q0, p1.clone())
    assert cache.hits == h0 + 1                # the Reg_opt-style reuse still fires
    assert torch.equal(a.Q, b.Q) and torch.equal(a.P, b.P)
    b.P[-1].fill_(123.0)                       # the caller's copy: the cache is not touched
    c = LM.Shoot(q0, p1.clone())
    assert cache.hits == h0 + 2 and torch.equal(c.P, a.P)
    return cache

