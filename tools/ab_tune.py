"""Interleaved A/B timing of tuning variants in ONE process (cdna_hip_programming.md 5.4
rule 24): rows-per-thread of the fused ODE forward / backward (--mode rsplit) and the
backward's pair-algebra variants (--mode alg).

    python tools/ab_tune.py [--M 50000] [--rounds 5]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from difficp_amd import _lib  # noqa: E402


def t_once(fn, reps=3):
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        fn()
    e1.record(st)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps


def run_rounds(M, rounds):
    """Fixed split rounds sweep of the fused ODE passes and the E-step."""
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    q = torch.rand(M, 3, device=dev)
    p = 0.01 * torch.randn(M, 3, device=dev)
    ga = torch.randn(M, 3, device=dev)
    gb = torch.randn(M, 3, device=dev)
    gd = torch.ones(1, device=dev)
    w2 = torch.zeros(M, device=dev)
    mu2 = (q * q).sum(-1)
    fns = {"fwd": lambda: _lib.ode_self_fwd(q, p, 0.1, 0.0, True),
           "bwd": lambda: _lib.ode_self_bwd(q, p, ga, gb, gd, 0.1, 0.0),
           "estep": lambda: _lib.gmm_estep(q, q, w2, mu2, 0.05, 0.0, True)}
    res = {}
    reps = 3 if M <= 60000 else 1
    sweep = (1, 2, 3, 4, 6, 8, 12, 16, 24)
    for r in sweep:
        _lib.set_option("split_rounds", r)
        for fn in fns.values():
            fn()
    torch.cuda.synchronize()
    for _ in range(rounds):
        for r in sweep:
            _lib.set_option("split_rounds", r)
            for k, fn in fns.items():
                res.setdefault(k, {}).setdefault(r, []).append(t_once(fn, reps))
    _lib.set_option("split_rounds", 0)
    return {k: {str(r): round(min(v), 4) for r, v in d.items()} for k, d in res.items()}


def run_splits(M, rounds):
    """Forced split-count sweep (force_splits) of the ODE forward and VJP at M rows: shows the
    wave-quantisation sawtooth (period = resident slots / row blocks)."""
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    q = torch.rand(M, 3, device=dev)
    p = 0.01 * torch.randn(M, 3, device=dev)
    ga = torch.randn(M, 3, device=dev)
    gb = torch.randn(M, 3, device=dev)
    gd = torch.ones(1, device=dev)
    fns = {"fwd": lambda: _lib.ode_self_fwd(q, p, 0.1, 0.0, True),
           "bwd": lambda: _lib.ode_self_bwd(q, p, ga, gb, gd, 0.1, 0.0)}
    auto = {"fwd": _lib.num_splits(1, M, M), "bwd": _lib.num_splits(2, M, M)}
    sweep = list(range(8, 97, 2))
    res = {}
    for s in sweep:
        _lib.set_option("force_splits", s)
        for fn in fns.values():
            fn()
    torch.cuda.synchronize()
    for _ in range(rounds):
        for s in sweep:
            _lib.set_option("force_splits", s)
            for k, fn in fns.items():
                res.setdefault(k, {}).setdefault(s, []).append(t_once(fn, 2))
    _lib.set_option("force_splits", 0)
    return {"auto": auto, **{k: {str(s): round(min(v), 4) for s, v in d.items()} for k, d in res.items()}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=50000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--mode", default="rsplit", choices=["rsplit", "alg", "rounds", "splits", "fwd", "symL", "eta", "pk", "fwdeta"])
    ap.add_argument("--Ms", default="20000,50000,200000", help="row counts for --mode rounds")
    a = ap.parse_args()
    if a.mode == "splits":
        print(json.dumps({"splits_ab": run_splits(a.M, a.rounds)}))
        return
    if a.mode == "rounds":
        print(json.dumps({"rounds_ab": {str(M): run_rounds(int(M), a.rounds) for M in a.Ms.split(",")}}))
        return
    M, D = a.M, 3
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    q = torch.rand(M, D, device=dev)
    p = 0.01 * torch.randn(M, D, device=dev)
    ga = torch.randn(M, D, device=dev)
    gb = torch.randn(M, D, device=dev)
    gd = torch.ones(1, device=dev)
    variants = []
    fwd = lambda: _lib.ode_self_fwd(q, p, 0.1, 0.0, True)
    bwd = lambda: _lib.ode_self_bwd(q, p, ga, gb, gd, 0.1, 0.0)
    if a.mode == "rsplit":
        for sr in (1, 2, 4, 8):
            for r in (1, 2):
                variants.append((f"fwd_r{r}_s{sr}", {"r_fwd": r, "split_rounds": sr}, fwd))
                variants.append((f"bwd_r{r}_s{sr}", {"r_bwd": r, "split_rounds": sr}, bwd))
    elif a.mode == "eta":  # eta != 0 VJP: ordered vs symmetric pair-once
        bwde = lambda: _lib.ode_self_bwd(q, p, ga, gb, gd, 0.1, 1e-3)
        variants.append(("bwd_eta_ordered", {"bwd_eta_alg": 0}, bwde))
        variants.append(("bwd_eta_sym", {"bwd_eta_alg": 1}, bwde))
        variants.append(("bwd_eta_sym_pk", {"bwd_eta_alg": 2}, bwde))
        variants.append(("bwd_eta0_sym", {"bwd_eta_alg": 1}, bwd))
    elif a.mode == "fwdeta":  # eta != 0 forward: scalar ordered rows vs packed-FP32 rows
        fwde = lambda: _lib.ode_self_fwd(q, p, 0.1, 1e-3, True)
        variants.append(("fwd_eta_alg0_scalar", {"fwd_alg": 0}, fwde))
        variants.append(("fwd_eta_alg2_packed", {"fwd_alg": 2}, fwde))
    elif a.mode == "pk":  # symmetric VJP: scalar rows vs packed-FP32 rows (lddmm_sym_pk.hpp)
        for L in (0, 2, 4):
            variants.append((f"bwd_alg2_sym_L{L}", {"bwd_alg": 2, "sym_L": L}, bwd))
            variants.append((f"bwd_alg3_pk_L{L}", {"bwd_alg": 3, "sym_L": L}, bwd))
    elif a.mode == "symL":  # symmetric VJP column groups per workgroup (0 = automatic)
        for L in (0, 1, 2, 4):
            variants.append((f"bwd_sym_L{L}", {"bwd_alg": 2, "sym_L": L}, bwd))
    elif a.mode == "fwd":  # ordered vs symmetric forward (and the symmetric VJP), sym_L sweep
        variants.append(("fwd_alg0_r2", {"fwd_alg": 0, "r_fwd": 2, "split_rounds": 0}, fwd))
        variants.append(("fwd_alg2_packed", {"fwd_alg": 2, "split_rounds": 0}, fwd))
        for L in (4,):
            variants.append((f"fwd_alg1_sym_L{L}", {"fwd_alg": 1, "sym_L": L}, fwd))
            variants.append((f"bwd_alg2_sym_L{L}", {"bwd_alg": 2, "sym_L": L}, bwd))
    else:  # pair-algebra variants of the backward, automatic splits
        for alg in (0, 1):
            for r in (1, 2, 4):
                variants.append((f"bwd_alg{alg}_r{r}", {"bwd_alg": alg, "r_bwd": r, "split_rounds": 0}, bwd))
        for L in (1, 2, 4, 8):
            variants.append((f"bwd_alg2_sym_L{L}", {"bwd_alg": 2, "sym_L": L, "split_rounds": 0}, bwd))
        variants.append(("fwd_r2", {"r_fwd": 2, "split_rounds": 0}, fwd))
    res = {v[0]: [] for v in variants}

    def setopts(o):
        for k, v in o.items():
            _lib.set_option(k, v)

    for name, o, fn in variants:  # warm every variant once
        setopts(o)
        fn()
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for name, o, fn in variants:
            setopts(o)
            res[name].append(t_once(fn))
    out = {k: {"median_ms": statistics.median(v), "min_ms": min(v),
               "Gpairs_per_s": M * M / (min(v) * 1e-3) / 1e9} for k, v in res.items()}
    print(json.dumps({"M": M, "ab": out}))


if __name__ == "__main__":
    main()
