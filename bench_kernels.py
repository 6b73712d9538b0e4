"""Per-kernel throughput of the gfx950 hot path (diagnostic companion of bench.py).

Prints one JSON object per kernel: time per launch (HIP events on the launch stream),
pairs/s, algorithmic flop/s and transcendental/s against the probed VALU peaks
(libdifficp_microbench.so), algorithmic HBM GB/s.

    python bench_kernels.py [--quick] [--only KRED,ODE_FWD,...]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from difficp_amd import _lib  # noqa: E402

# Algorithmic cost per pair for D = 3 (FMA = 2 flop; exp2 = 1 transcendental "T").
# Counted from the pair operators in diff-icp_amd/csrc/lddmm_ops.hpp / gmm.hip.
FLOPS_PER_PAIR = {
    "KRED": 15, "GRADK": 15, "GENDK": 21,
    "ODE_FWD": 33,            # v, Z, G with DIV (eta = 0)
    "ODE_BWD": 80,            # fused VJP (eta = 0)
    "GMM_ESTEP": 2 * 13 + 12,  # two sweeps (max, then exp + 6 weighted sums)
    "GMM_MSTEP": 2 * 13 + 6,
    "GMM_TARGETS": 30,
}
# HBM bytes per launch (algorithmic: each input read once, each output written once).


def timed(fn, warm=2, reps=10):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        fn()
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def probe_peaks():
    path = os.path.join(ROOT, "diff-icp_amd", "libdifficp_microbench.so")
    mb = ctypes.CDLL(path)
    mb.dicp_mb_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                  ctypes.c_void_p]
    chains = mb.dicp_mb_chains()
    out = torch.zeros(256, device="cuda")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    blocks, iters = 256 * 8 * 4, 4096
    res = {}
    for kind, name, mult in ((0, "exp2_per_s", 1), (1, "fma_flops", 2), (2, "pk_fma_flops", 4),
                             (3, "dpp_wave_rol_add_per_s", 1), (4, "dpp_row_ror_add_per_s", 1),
                             (5, "fma_flops_with_1exp_per_8fma", 2)):
        t = timed(lambda: mb.dicp_mb_launch(kind, blocks, iters, ctypes.c_void_p(out.data_ptr()), st),
                  warm=2, reps=5)
        res[name] = blocks * 256 * iters * chains * mult / t
    # SIMD cycles per wave64 instruction at the nominal 2.4 GHz, 1024 SIMDs
    res["cycles_per_wave_instr"] = {k: 1024 * 2.4e9 * 64 * m / res[k] for k, m in (
        ("exp2_per_s", 1), ("fma_flops", 2), ("dpp_wave_rol_add_per_s", 1),
        ("dpp_row_ror_add_per_s", 1))}
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--only", default="")
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    only = set(args.only.split(",")) if args.only else None
    results = []

    peaks = probe_peaks()
    print(json.dumps({"peaks": peaks}), flush=True)
    results.append({"peaks": peaks})

    def rep(name, t, pairs, bytes_, extra=None):
        fl = FLOPS_PER_PAIR.get(name.split("@")[0], 0) * pairs
        r = {"kernel": name, "ms": t * 1e3, "Gpairs_per_s": pairs / t / 1e9,
             "TFLOPs": fl / t / 1e12, "Texp_per_s": pairs / t / 1e12,
             "frac_fp32_peak": fl / t / peaks["pk_fma_flops"],
             "frac_exp_peak": pairs / t / peaks["exp2_per_s"],
             "alg_GBps": bytes_ / t / 1e9, "splits": None}
        if extra:
            r.update(extra)
        print(json.dumps(r), flush=True)
        results.append(r)

    D = 3
    n_big = 20000 if args.quick else 100000
    if only is None or "KRED" in only:
        x = torch.rand(n_big, D, device=dev)
        b = torch.randn(n_big, D, device=dev)
        t = timed(lambda: _lib.gauss_red(_lib.KRED, x, x, 0.1, b=b))
        rep(f"KRED@{n_big}x{n_big}", t, n_big * n_big, 4 * (3 * n_big + 6 * n_big + 3 * n_big),
            {"splits": _lib.num_splits(_lib.WS_RED, n_big, n_big)})
    for M in ([20000] if args.quick else [20000, 50000, 200000]):
        if only is not None and "ODE" not in only:
            break
        q = torch.rand(M, D, device=dev)
        p = 0.01 * torch.randn(M, D, device=dev)
        t = timed(lambda: _lib.ode_self_fwd(q, p, 0.1, 0.0, True), reps=5)
        rep(f"ODE_FWD@{M}", t, M * M, 4 * (6 * M + 6 * M + 7 * M))
        a = torch.randn(M, D, device=dev)
        bm = torch.randn(M, D, device=dev)
        gd = torch.ones(1, device=dev)
        t = timed(lambda: _lib.ode_self_bwd(q, p, a, bm, gd, 0.1, 0.0), reps=5)
        rep(f"ODE_BWD@{M}", t, M * M, 4 * (12 * M + 12 * M + 6 * M))
    if only is None or "GMM" in only:
        for (N, C) in ([(50000, 50000)] if args.quick else [(50000, 50000), (640000, 512), (200000, 200000)]):
            X = torch.rand(N, D, device=dev)
            mu = torch.rand(C, D, device=dev)
            w2 = torch.zeros(C, device=dev)
            mu2 = (mu * mu).sum(-1)
            t = timed(lambda: _lib.gmm_estep(X, mu, w2, mu2, 0.05, 0.0, True), reps=5)
            rep(f"GMM_ESTEP@{N}x{C}", t, N * C, 4 * (3 * N + 5 * C + 9 * N))
            T, T2, _ = _lib.gmm_estep(X, mu, w2, mu2, 0.05, 0.0, False)
            t = timed(lambda: _lib.gmm_mstep(X, T2, mu, w2, 0.05), reps=5)
            rep(f"GMM_MSTEP@{N}x{C}", t, N * C, 4 * (4 * N + 4 * C + 4 * C))
            t = timed(lambda: _lib.gmm_targets(X, T2, mu, w2, 0.05, mu, w2), reps=5)
            rep(f"GMM_TARGETS@{N}x{C}", t, N * C, 4 * (4 * N + 9 * C + 7 * N))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
