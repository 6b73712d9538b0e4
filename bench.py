"""Headline benchmark: diff-ICP PSR iterations/sec on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
                    [--workload two_set_100k|two_set_100k_2d|two_set_50k|two_set_200k|two_set_50k_exact|atlas_c4|atlas_c4_fixed|c5|c5_alt]
    (N > 1: one rank per GPU over RCCL.  Under torch.distributed.run WORLD_SIZE must equal N;
     started without it, bench.py starts `python -m torch.distributed.run --nproc-per-node N`
     on itself as a child process -- before anything touches the GPU -- and exits with the
     child's status; rank 0's JSON line reaches stdout through the child.)

A "step" is one diff-ICP iteration on the workload -- GMM_opt(max_repeat_GMM=10, tol=1e-3)
+ Reg_opt(nmax=1, tol=1e-3), the loop body of ICP_two_set.py:254-282 / ICP_atlas.py:269-298 --
with every point set resident in HBM.  Default workload (the point count BASELINE.json's
metric names, "100k-pt 3D"; configs[1] is two_set_50k):
two-point-set 3D match, 100k vs 100k synthetic points, hybrid LDDMM (sigma 0.1, lambda 1e3,
Euler nt=10, dense support), GMM on xB with sigma optimised.  The atlas workloads shard
frames over ranks with an RCCL exchange of the GMM sufficient statistics: atlas_c4 / c5 /
c5_alt keep the frames per rank fixed (weak scaling), atlas_c4_fixed keeps the whole
32-frame C4 atlas fixed (strong scaling, value = atlas iterations per second).

Rank 0 prints ONE JSON line (value = iterations of all ranks / max-over-ranks time) with a
"roofline" object for the dominant kernel (algorithmic flop per launch / average launch
time from HIP events on the launch stream, vs the 157.3 TFLOP/s fp32 peak) and a
"cpu_baseline" object (the oracle's C restatement timed on this host on a bounded sample,
extrapolated to one iteration of the same workload from the live pair counts).

Two-set workloads at N > 1 row-split the ONE match over the ranks by default (SURVEY f1,
core/rowsplit.py; "scaling": "strong", value = iterations of that match per second);
--replicas runs N independent copies instead (weak scaling).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

FP32_PEAK_TFLOPS = 157.3   # MI355X dense fp32 (vector v_pk_fma_f32 = f32 MFMA), MI355X_MICROARCH.md
# v_exp_f32: 8 issue cycles per wave64 instruction (MI355X_MICROARCH.md "vector-instruction
# ISSUE cost") -> 64 / 8 lanes per cycle x 1024 SIMDs x 2.4 GHz
EXP_PEAK_TPS = 64 / 8 * 1024 * 2.4e9 / 1e12
HBM_PEAK_GBPS = 8000.0
# measured issue costs on MI355X (tools/probes/coissue.py, profiles/r03_probe_coissue.json): SIMD
# cycles per wave64 instruction at the nominal 2.4 GHz; a v_exp_f32 does not overlap the FMAs
FMA_ISSUE_CYC, EXP_ISSUE_CYC = 2.36, 10.2

# BASELINE.json "metric": value is the PSR iterations/sec half; the kernel-sum HBM GB/s half
# (algorithmic bytes of all hot-path launches / their summed device time) is kernel_sum_hbm_GBps
METRIC = "PSR iterations/sec + kernel-sum HBM GB/s, 100k-pt 3D, 1/2/4/8 MI355X"

WORKLOADS = {
    "two_set_50k": dict(kind="two_set", N=50000),
    "two_set_200k": dict(kind="two_set", N=200000),
    # the point count BASELINE.json's metric string names ("100k-pt 3D")
    "two_set_100k": dict(kind="two_set", N=100000),
    # the north_star's "synthetic 2D/3D point sets": the same match in the plane (the
    # reference's own examples are 2D: diffICP_basic.py, the Chui sets)
    "two_set_100k_2d": dict(kind="two_set", N=100000, D=2),
    # SURVEY C2': the exact ICP_two_set model (gradcomponent=True, eta = 1/lambda), a0 from
    # the device ridge CG (v2p version "ridge_keops", alpha 1e-3, PSR.py:402)
    "two_set_50k_exact": dict(kind="two_set", N=50000, version="logdet",
                              v2p_args={"version": "ridge_keops", "alpha": 1e-3}),
    "atlas_c4": dict(kind="atlas", K_per_rank=4, N=20000, C=512, S=1),
    # BASELINE configs[3] as a FIXED workload: 32 frames x 20k whatever the rank count (frames
    # sharded over the ranks), so the 1 -> 8 GPU lines measure strong scaling of one atlas
    # (ICP_atlas.py:269-298); value = iterations of the whole 32-frame atlas per second
    "atlas_c4_fixed": dict(kind="atlas", K_total=32, N=20000, C=512, S=1),
    "c5": dict(kind="atlas", K_per_rank=8, N=7500, C=256, S=4),
    # SURVEY 8(d) C5, alternative reading: 30k points per structure (120k per frame)
    "c5_alt": dict(kind="atlas", K_per_rank=8, N=30000, C=256, S=4),
}


def log(msg):
    print(msg, file=sys.stderr, flush=True)


def _pair_kind(name):
    """CPU-rate class of a live kernel name: the VJP variants (ode_self_bwd*, ode_ext_bwd)
    are priced at the backward rate, the EM passes at the E-step rate, the rest (forward
    passes, reductions, CG mat-vecs) at the forward rate."""
    if name.startswith("ode_self_bwd") or name.startswith("ode_ext_bwd") or name == "gauss_red_grad":
        return "bwd"
    if name.startswith("gmm_"):
        return "em"
    return "fwd"


def _cpu_threads():
    return int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)


def _round_robin(calls, budget_s):
    times = {k: [] for k in calls}
    t_start = time.perf_counter()
    while True:  # round-robin until the sample budget is spent (at least one of each)
        for k, f in calls.items():
            t0 = time.perf_counter()
            f()
            times[k].append(time.perf_counter() - t0)
        if time.perf_counter() - t_start > budget_s:
            break
    return times, time.perf_counter() - t_start


def cpu_baseline_c(pair_counts, M_work, budget_s=15.0, D=3):
    """The oracle's C restatement (OpenMP) of the dominant pair kernels, timed on this host on
    a bounded sample -- repeated ODE-forward / VJP / E-step evaluations at M x M pairs (the
    workload's size, capped at 50k so one evaluation stays ~1 s) -- then extrapolated to one
    iteration from the live pair counts (the C kernels' pair rate is flat in M)."""
    from oracle import c_ref
    threads = _cpu_threads()
    torch.manual_seed(0)
    M = int(M_work)
    q = torch.rand(M, D)
    p = 0.01 * torch.randn(M, D)
    a = torch.randn(M, D)
    X = torch.rand(M, D)
    w0 = torch.zeros(M)
    calls = {"fwd": lambda: c_ref.ode_self_fwd(q, p, 0.1),
             "bwd": lambda: c_ref.ode_self_bwd(q, p, a, a, 1.0, 0.1),
             "em": lambda: c_ref.gmm_estep(X, X, w0, 0.05)}
    times, took = _round_robin(calls, budget_s)
    rates = {k: M * M / (sum(v) / len(v)) for k, v in times.items()}
    secs = sum(v / rates[_pair_kind(k)] for k, v in pair_counts.items())
    return {"value": 1.0 / secs, "unit": "PSR iterations/sec", "cores": threads, "kind": "port",
            "sample": (f"oracle/difficp_ref.c (OpenMP C, {threads} threads): {len(times['fwd'])} x (ODE fwd + VJP + "
                       f"E-step) at {M}x{M} pairs, D = {D} ({took:.1f} s), rates fwd {rates['fwd'] / 1e9:.3f} / bwd "
                       f"{rates['bwd'] / 1e9:.3f} / EM {rates['em'] / 1e9:.3f} Gpair/s, extrapolated to the live "
                       "pair counts of one iteration")}


def cpu_baseline_torch(pair_counts, budget_s=15.0, M=4000, D=3):
    """The reference's CPU path as SURVEY 8(d) defines the baseline: the chunked torch
    restatement of the reference's operators (oracle/torch_ref.py: the torch arithmetic of
    kernel.py / LDDMM.py / GMM.py, float32, torch.set_num_threads = the host threads), timed on
    a bounded sample -- one hybrid ODE evaluation (KRed + GenDKRed + GradKRed, LDDMM.py:176-227),
    the same with its torch-autograd backward (optim.py:46), one torch-path EM step
    (GMM.py:236-325) at M x M/4 -- and extrapolated to one iteration from the live pair counts.
    Cross-timed against the imported reference at M <= 4000 in the build container:
    profiles/r03_cpu_crosstime.json (restatement / reference within 1.2x)."""
    from oracle import torch_ref as R
    threads = _cpu_threads()
    old_threads = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        g = torch.Generator().manual_seed(0)
        q = torch.rand(M, D, generator=g)
        p = 0.01 * torch.randn(M, D, generator=g)
        a = torch.randn(M, D, generator=g)
        b = torch.randn(M, D, generator=g)
        C = M // 4
        X = torch.rand(M, D, generator=g)
        mu = torch.rand(C, D, generator=g)
        w0 = torch.zeros(C)
        m = R.LDDMM(0.1, D, 1e3, False, True)
        c0 = torch.zeros(1)
        opt = {"mu": True, "w": True, "sigma": True, "eta0": False}

        def fwd_bwd():
            qq = q.clone().requires_grad_(True)
            pp = p.clone().requires_grad_(True)
            v, mG, dc = m.ODE(qq, pp, c0)
            torch.autograd.grad((a * v).sum() + (b * mG).sum() + dc.sum(), (qq, pp))

        calls = {"fwd": lambda: m.ODE(q, p, c0), "fwd_bwd": fwd_bwd,
                 "em": lambda: R.em_step(X, mu, w0, 0.05, opt)}
        times, took = _round_robin(calls, budget_s)
    finally:
        torch.set_num_threads(old_threads)
    avg = {k: sum(v) / len(v) for k, v in times.items()}
    rates = {"fwd": M * M / avg["fwd"], "bwd": M * M / max(avg["fwd_bwd"] - avg["fwd"], 1e-9),
             "em": M * C / avg["em"]}
    secs = sum(v / rates[_pair_kind(k)] for k, v in pair_counts.items())
    return {"value": 1.0 / secs, "unit": "PSR iterations/sec", "cores": threads, "kind": "port",
            "sample": (f"oracle/torch_ref.py (the reference's torch arithmetic, float32, {threads} threads): "
                       f"{len(times['fwd'])} x (hybrid ODE eval, ODE eval + autograd backward, EM step) at "
                       f"{M} points, D = {D} ({took:.1f} s); rates fwd {rates['fwd'] / 1e9:.4f} / bwd {rates['bwd'] / 1e9:.4f} / "
                       f"EM {rates['em'] / 1e9:.4f} Gpair/s, extrapolated to the live pair counts of one "
                       "iteration; cross-timed vs the imported reference within 1.2x at N <= 4000 "
                       "(profiles/r03_cpu_crosstime.json)")}


def cpu_baseline(pair_counts, M_work, D=3):
    """cpu_baseline object of the bench line: the reference-path torch restatement (SURVEY
    8(d)) as the value, the faster OpenMP C restatement beside it."""
    base = cpu_baseline_torch(pair_counts, D=D)
    try:
        base["c_openmp"] = cpu_baseline_c(pair_counts, M_work, budget_s=10.0, D=D)
    except Exception as e:  # informative only
        base["c_openmp"] = {"error": repr(e)}
    return base


def kernel_sum_probe(dev, M, reps=5, same=True):
    """The north_star's "100k x 100k 3D Gaussian kernel sum": KRed (kernel.py:138,
    X_i = sum_j K(x_i - y_j) b_j) at M x M on this GPU, HIP events on the launch stream, best of
    `reps`.  Reported beside the compute roofline because the north_star quotes this sum
    against the HBM roofline: its algorithmic HBM bytes (4 (3M + 6M + 3M)) over the launch are a
    few GB/s, while the bytes a non-reusing (streaming) evaluation would read, 2 D 4 B per pair,
    are labelled as "effective pair-stream GB/s" (SURVEY 8(d)), never as HBM."""
    from difficp_amd import _lib
    g = torch.Generator(device="cpu").manual_seed(1)
    x = torch.rand(M, 3, generator=g).to(dev)
    b = (0.01 * torch.randn(M, 3, generator=g)).to(dev)
    y = x if same else torch.rand(M, 3, generator=g).to(dev)
    st = torch.cuda.current_stream(dev)
    _lib.gauss_red(_lib.KRED, x, y, 0.1, b=b)
    # throughput: `back` calls back to back between two events (each call's prep pass, sort
    # and merge included), best of `reps` -- a lone call also carries the launch gaps between
    # its ~10 small prep / merge kernels (+0.2 ms at 100k, measured in round 5)
    back = 4
    best = None
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(back):
            _lib.gauss_red(_lib.KRED, x, y, 0.1, b=b)
        e1.record(st)
        e1.synchronize()
        ms = e0.elapsed_time(e1) / back
        best = ms if best is None else min(best, ms)
    pairs = float(M) * M
    s = best * 1e-3
    fl = _lib.FLOPS_PER_PAIR.get("gauss_red", 15)
    # the compute bound of the sum is max(flops / P_fp32, exps / P_exp)
    bound_s = max(pairs * fl / (FP32_PEAK_TFLOPS * 1e12), pairs * 1.0 / (EXP_PEAK_TPS * 1e12))
    centred = _lib.get_option("red_alg") and M >= 32768 and float(M) * M >= 2.5e9
    if centred and same and _lib.get_option("sym_red"):
        path = ("pair-once centred sum (csrc/sym_cx.hpp: Morton-sorted 256-point groups, each unordered "
                "pair once -- 3 FMA exponent + 1 exp, row and column sides, 4 rows per lane; prep pass "
                "and merge included in the time)")
    elif centred:
        path = ("centred expansion (csrc/centred.hpp: Morton-sorted 64-column sub-tiles, 6 FMA + 1 exp "
                "per pair, 4 rows per thread packed in pairs, prep pass included in the time)")
    else:
        path = "packed scaled-coordinate kernel (ext_pk.hpp)"
    return {"op": f"KRed (kernel.py:138) {'x = y' if same else 'x != y (two independent clouds)'}, D = 3, sigma 0.1",
            "M": M, "ms": round(best, 4), "timing": f"{back} calls back to back per event pair, best of {reps}",
            "path": path, "Tpair_per_s": round(pairs / s / 1e12, 3),
            "tflops": round(pairs * fl / s / 1e12, 2), "frac_fp32_peak": round(pairs * fl / s / 1e12 / FP32_PEAK_TFLOPS, 4),
            "compute_bound_ms": round(bound_s * 1e3, 4),
            "frac_of_compute_bound": round(bound_s / s, 4),
            "compute_bound": (f"max(15 flop x M^2 / {FP32_PEAK_TFLOPS} TFLOP/s, 1 exp x M^2 / "
                              f"{EXP_PEAK_TPS:.2f} Texp/s) (SURVEY 8(d))"),
            # the pair loop's instruction-stream floor: 6 FMA + 1 exp per pair (centred path) at
            # the probed issue costs, 1024 SIMDs x 64 lanes at 2.4 GHz -- what the kernel could
            # reach if nothing but its pair arithmetic issued (no prep, sub-tile or loop work)
            "issue_floor_ms": round(pairs / 64 / 1024 * (6 * FMA_ISSUE_CYC + EXP_ISSUE_CYC) / 2.4e9 * 1e3, 4),
            "frac_of_issue_floor": round(pairs / 64 / 1024 * (6 * FMA_ISSUE_CYC + EXP_ISSUE_CYC) / 2.4e9 / s, 4),
            "alg_hbm_GBps": round(4 * 12 * M / s / 1e9, 3),
            "effective_pair_stream_GBps": round(pairs * 2 * 3 * 4 / s / 1e9, 1),
            "note": "compute-bound (15 flop + 1 exp per pair, O(M) bytes): the HBM roofline does not "
                    "bind; effective pair-stream GB/s = bytes a non-reusing kernel would stream "
                    "(2 D floats per pair), not HBM traffic"}


def load_traffic(kernel_name):
    """HBM bytes per launch from the committed rocprofv3 PMC summary, if present."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get(kernel_name, {}).get("hbm_bytes_per_launch")
    except Exception:
        return None


def load_issue(kernel_name):
    """Effective clock under load and VALU issue occupancy from the committed SQ/GRBM pass
    (tools/pmc_issue.py -> profiles/pmc_issue.json), if present."""
    path = os.path.join(ROOT, "profiles", "pmc_issue.json")
    try:
        with open(path) as f:
            d = json.load(f).get(kernel_name, {})
        return d.get("eff_clock_GHz"), d.get("valu_issue_busy_per_simd")
    except Exception:
        return None, None


def launch_plan(argv, env):
    """How `bench.py argv` runs, decided before any GPU call: ("run", world) in this process
    (world 1, or a rank started by torch.distributed.run with WORLD_SIZE = --gpus), or
    ("spawn", cmd) -- the torch.distributed.run command a plain `bench.py --gpus N` (N > 1)
    starts as its child, one rank per GPU, with every argument passed through.  A WORLD_SIZE
    that disagrees with --gpus raises SystemExit (the line would claim the wrong GPU count)."""
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    a, _ = ap.parse_known_args(argv)
    if a.gpus < 1:
        raise SystemExit(f"bench.py: --gpus {a.gpus} must be >= 1")
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != a.gpus:
            raise SystemExit(f"bench.py: WORLD_SIZE={ws} but --gpus {a.gpus}: launch {a.gpus} ranks "
                             "or pass --gpus WORLD_SIZE")
        return ("run", int(ws))
    if a.gpus == 1:
        return ("run", 1)
    port = env.get("MASTER_PORT") or str(_free_port())
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    return ("spawn", cmd)


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def main():
    plan = launch_plan(sys.argv[1:], os.environ)
    if plan[0] == "spawn":
        # a child process, never an exec: nothing here has touched the GPU, and the ranks'
        # stdout (rank 0's JSON line) is this process's stdout
        import subprocess
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        log(f"bench: --gpus > 1 without WORLD_SIZE, starting the ranks: {' '.join(plan[1])}")
        rc = subprocess.run(plan[1], env=env).returncode
        sys.exit(rc)
    # the driver parses ONE JSON line from stdout: everything else (e.g. the reference's
    # "GMM optimization - reached maximum number of iterations" message) goes to stderr
    real_stdout = sys.stdout
    sys.stdout = sys.stderr
    try:
        _main(real_stdout)
    finally:
        sys.stdout = real_stdout


def _main(out):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="two_set_100k", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-profile", action="store_true", help="skip live per-kernel events")
    ap.add_argument("--concurrent-frames", type=int, default=None,
                    help="atlas workloads: frames optimised concurrently (host threads / HIP "
                         "streams); default automatic (4), 1 = the reference's sequential loop")
    ap.add_argument("--batch-frames", choices=["on", "off"], default="off",
                    help="atlas workloads: the local frames' shooting launches in lockstep batches "
                         "(core/batching.py, opt-in), --concurrent-frames groups of them on their own "
                         "HIP streams")
    ap.add_argument("--batch-share", type=int, default=0,
                    help="atlas: kernel geometry per frame sized for the frame's share of the chip "
                         "(0, default: the concurrent frames / the frames per batch group), as if "
                         "alone (1), or for 1/n of it (n)")
    ap.add_argument("--lib-opt", action="append", default=[], metavar="NAME=VALUE",
                    help="dicp_set_option before the run (A/B experiments; repeatable)")
    ap.add_argument("--replicas", action="store_true",
                    help="two-set workloads at N > 1: N independent replicas (weak scaling) "
                         "instead of row-splitting the one match over the N GPUs")
    args = ap.parse_args()

    world = launch_plan(sys.argv[1:], os.environ)[1]
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal on a 1-GPU box (never the driver's runs): DICP_BENCH_REHEARSE=1 puts every rank
    # on cuda:0 and uses gloo, which RCCL cannot do (one rank per GPU)
    rehearse = os.environ.get("DICP_BENCH_REHEARSE") == "1"
    if rehearse:
        local = 0
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        if rehearse:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from difficp_amd import _lib, workloads
    for kv in args.lib_opt:
        k, v = kv.split("=")
        _lib.set_option(k, int(v))

    wl = WORKLOADS[args.workload]
    t_setup = time.perf_counter()
    if wl["kind"] == "two_set":
        # N > 1: the ONE match is row-split over the ranks (core/rowsplit.py: per ODE step an
        # RCCL all-gather of the new row slices, per adjoint step an all-reduce of the VJP
        # parts) -- strong scaling; --replicas: N independent copies (weak scaling)
        version = wl.get("version", "hybrid")
        D = wl.get("D", 3)
        psr = workloads.build_two_set(wl["N"], dev, seed=0, version=version,
                                      v2p_args=wl.get("v2p_args"), D=D)
        split = world > 1 and not args.replicas
        if split:
            psr.LMi.set_row_split()
        src = {50000: "BASELINE configs[1]", 200000: "BASELINE configs[2]",
               100000: "BASELINE metric's 100k-pt 3D"}.get(wl["N"], "two-set")
        if D != 3:
            src = f"the north_star's 2D/3D point sets, {D}D"
        cfg = {"workload": f"two-set {D}D {wl['N']} vs {wl['N']} ({src})" +
               (" exact ICP_two_set model" if version == "logdet" else ""),
               "points_per_set": wl["N"], "lddmm": f"{version} sigma=0.1 lambda=1e3 Euler nt=10 dense",
               "gmm": "mu=xB fixed, sigma optimised", "max_repeat_GMM": 10, "tol": 1e-3,
               "parallelism": (f"row-split x{world} (RCCL all-gather / all-reduce per ODE step)" if split
                               else f"replicas x{world}")}
        scaling = "strong" if split else "weak"
    else:
        fixed = "K_total" in wl
        K = wl["K_total"] if fixed else wl["K_per_rank"] * world
        comm = True if world > 1 else None
        psr = workloads.build_atlas(K, wl["N"], wl["C"], dev, comm=comm, seed=0, S=wl["S"])
        psr.concurrent_frames = args.concurrent_frames
        psr.batch_frames = args.batch_frames == "on"
        psr.batch_share = args.batch_share
        cfg = {"workload": f"groupwise atlas {K} frames x {wl['S']} structures x {wl['N']} 3D points, "
                           f"C={wl['C']} per structure" + (" (BASELINE configs[3], fixed)" if fixed else ""),
               "frames_per_rank": (f"{K // world}-{-(-K // world)}" if fixed else wl["K_per_rank"]),
               "lddmm": "hybrid sigma=0.1 lambda=1e3 Euler nt=10 dense", "max_repeat_GMM": 10,
               "tol": 1e-3, "parallelism": f"frame-sharded dp{world} (RCCL suff-stat exchange)",
               "concurrent_frames": args.concurrent_frames or "auto",
               "batch_frames": args.batch_frames, "batch_share": args.batch_share}
        scaling = "strong" if fixed else "weak"
    torch.cuda.synchronize()
    log(f"[rank {rank}] setup {time.perf_counter() - t_setup:.1f}s")

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()

    # row split: the warmup iterations check after every VJP all-reduce that all ranks hold
    # the same bits (RowSplit.verify; the replicated L-BFGS must take identical decisions) --
    # a mismatch raises on every rank at once instead of letting the ranks diverge
    rs = getattr(getattr(psr, "LMi", None), "row_split", None)
    if rs is not None:
        rs.verify = True
    for i in range(args.warmup):
        t0 = time.perf_counter()
        workloads.psr_iteration(psr)
        torch.cuda.synchronize()
        log(f"[rank {rank}] warmup {i}: {time.perf_counter() - t0:.2f}s FE={psr.FE:.6g}")
    if rs is not None:
        log(f"[rank {rank}] row split: {rs.verified_calls} all-reduces verified bitwise identical across ranks")
        rs.verify = False

    # frames optimised concurrently (atlas, one HIP stream per frame thread): kernels of
    # different frames overlap, so per-launch event times are not kernel durations -- the
    # per-kernel accounting (roofline) then comes from one extra sequential-frame iteration
    # after the timed region
    concurrent = (wl["kind"] == "atlas" and len(list(psr.frames)) > 1 and
                  (psr.concurrent_frames is None or psr.concurrent_frames > 1))
    prof = _lib.KernelProfile() if not args.no_profile else None
    prof_iters = args.steps
    from difficp_amd.tools import runstats
    barrier()
    torch.cuda.synchronize()
    rs0 = runstats.snapshot()
    t0 = time.perf_counter()
    if prof is not None and not concurrent:
        with prof:
            for i in range(args.steps):
                workloads.psr_iteration(psr)
                log(f"[rank {rank}] step {i} FE={psr.FE:.6g}")
    else:
        for i in range(args.steps):
            workloads.psr_iteration(psr)
            log(f"[rank {rank}] step {i} FE={psr.FE:.6g}")
    torch.cuda.synchronize()
    t_done = time.perf_counter() - t0       # this rank's own work (before waiting for the others)
    rs1 = runstats.snapshot()
    barrier()
    elapsed = time.perf_counter() - t0
    # per-rank diagnostics of the timed region (a first multi-GPU line that misses its target
    # must say why: uneven work, closures, time inside the collectives)
    mine = {"rank": rank, "FE": psr.FE, "work_s": round(t_done, 4), "frames": len(list(getattr(psr, "frames", [0]))),
            **{k: (round(v, 4) if isinstance(v, float) else v) for k, v in runstats.delta(rs0, rs1).items()}}
    if prof is not None and not concurrent:
        mine["kernel_busy_s"] = round(sum(v["ms"] for v in prof.summary().values()) * 1e-3, 4)
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        ranks = [None] * world
        dist.all_gather_object(ranks, mine)
    else:
        ranks = [mine]
    if prof is not None and concurrent:
        # the frames one after another, with the kernel geometry the timed (concurrent)
        # iterations used (batch_share 0 = the concurrent frames): the same kernels, timed alone
        saved = psr.concurrent_frames, psr.batch_share
        nconc = min(psr.concurrent_frames or 4, len(list(psr.frames)))
        psr.concurrent_frames = 1
        if psr.batch_share == 0 and not getattr(psr, "batch_stats", None):
            psr.batch_share = nconc
        with prof:
            workloads.psr_iteration(psr)
        torch.cuda.synchronize()
        psr.concurrent_frames, psr.batch_share = saved
        prof_iters = 1

    if rank == 0:
        # row-split two-set / fixed atlas: all ranks advance the SAME problem; replicas /
        # per-rank atlas: every rank's own work
        iters = args.steps * (1 if scaling == "strong" else world)
        value = iters / elapsed
        summ = prof.summary() if prof is not None else {}
        roof = None
        pair_counts = {k: v["pairs"] / prof_iters for k, v in summ.items()}
        if summ:
            dom = max(summ, key=lambda k: summ[k]["ms"])
            d = summ[dom]
            avg_s = d["ms"] / d["launches"] * 1e-3
            Dw = wl.get("D", 3)
            fpp = _lib.flops_per_pair(dom, Dw)     # the D = 3 table, rescaled for 2D workloads
            flops_per_launch = d["pairs"] / d["launches"] * fpp if fpp else d["flops"] / d["launches"]
            # executed-instruction figure: counted from the D = 3 hot loop only
            efpp = _lib.EXEC_FLOPS_PER_PAIR.get(dom, _lib.FLOPS_PER_PAIR.get(dom)) if Dw == 3 else None
            achieved = flops_per_launch / avg_s / 1e12
            # committed PMC summary: whole-size single-device launches of the default workload
            # (tools/pmc_probe.py); not the pair-subset launches of a row split
            traffic = (load_traffic(dom) if world == 1 and wl.get("N") == 100000 and wl.get("D", 3) == 3
                       else None)
            # compute-bound on the VALU (the north_star: "MFMA not used"): priced against the
            # dense FP32 peak, 157.3 TF/s on MI355X, which is the packed-VALU rate (and also the
            # f32 MFMA rate, MI355X_MICROARCH.md); 3-wide dot products + exp, no contraction
            roof = {"bound": "valu", "compute_unit": "VALU (fp32 packed v_pk_* + v_exp_f32; dense fp32 "
                                                     "peak = packed-VALU peak = f32 MFMA peak)",
                    "achieved": round(achieved, 3), "peak": FP32_PEAK_TFLOPS,
                    "unit": "TFLOP/s", "frac": round(achieved / FP32_PEAK_TFLOPS, 4),
                    "traffic": traffic, "kernel": dom, "launches": d["launches"],
                    "avg_launch_ms": round(d["ms"] / d["launches"], 4),
                    "pairs_per_launch": d["pairs"] / d["launches"],
                    "flops_per_pair": round(fpp, 3) if fpp else fpp,
                    "flops_source": ("SURVEY.md 8(d) per-unit figure x ordered pairs (M^2)" if Dw == 3 else
                                     f"SURVEY.md 8(d) per-unit figure (D = 3) rescaled to D = {Dw} by the "
                                     "operator's term count in D (_lib.flops_per_pair) x ordered pairs"),
                    "exec_flops_per_pair": efpp,
                    "frac_executed": (round(achieved / FP32_PEAK_TFLOPS * efpp / fpp, 4)
                                      if efpp and fpp else None),
                    "alg_bytes_per_launch": d["bytes"] / d["launches"],
                    "alg_hbm_GBps": round(d["bytes"] / d["launches"] / avg_s / 1e9, 3),
                    "share_of_step_time": round(d["ms"] / prof_iters * 1e-3 / (elapsed / args.steps), 3),
                    "measured_on": (("one extra iteration after the timed region with all local frames "
                                     "in ONE lockstep launch batch (the timed iterations overlap several "
                                     "batches on HIP streams)") if getattr(psr, "batch_stats", None)
                                    else ("one extra sequential-frame iteration after the timed region, "
                                          "with the timed iterations' kernel geometry (they overlap "
                                          "frames on HIP streams)")) if concurrent
                                   else "the timed iterations",
                    "note": "pair kernels are fp32 VALU/exp-bound (O(N) bytes, O(N^2) work): "
                            "compute roofline, HBM bytes reported as alg_hbm_GBps/traffic; traffic "
                            "(rocprofv3 2 x FETCH_SIZE + WRITE_SIZE per launch, the gfx950 correction of "
                            "MI355X_MICROARCH.md; profiles/pmc_traffic.json; default workload at N=1 only) "
                            "is dominated by the deterministic partial slots (written once, read once "
                            "by the merge), ~2% of HBM bandwidth over the launch"}
            # the second kernel by time (on the two-set workloads the symmetric forward), priced
            # the same way: its algorithmic and executed fractions of the peak
            rest = sorted((k for k in summ if k != dom), key=lambda k: -summ[k]["ms"])
            if rest:
                k2 = rest[0]
                d2 = summ[k2]
                avg2 = d2["ms"] / d2["launches"] * 1e-3
                f2 = _lib.flops_per_pair(k2, Dw)
                e2 = _lib.EXEC_FLOPS_PER_PAIR.get(k2, f2) if Dw == 3 else None
                a2 = d2["pairs"] / d2["launches"] * f2 / avg2 / 1e12 if f2 else None
                roof["second"] = {"kernel": k2, "launches": d2["launches"],
                                  "avg_launch_ms": round(d2["ms"] / d2["launches"], 4),
                                  "achieved": round(a2, 3) if a2 else None,
                                  "frac": round(a2 / FP32_PEAK_TFLOPS, 4) if a2 else None,
                                  "flops_per_pair": f2, "exec_flops_per_pair": e2,
                                  "frac_executed": (round(a2 / FP32_PEAK_TFLOPS * e2 / f2, 4)
                                                    if a2 and e2 else None),
                                  "share_of_step_time": round(d2["ms"] / prof_iters * 1e-3 / (elapsed / args.steps), 3)}
            # whole-iteration view: the algorithmic flops of every pair pass of one iteration
            # over its wall time (host gaps, E-steps and small kernels included) -- for
            # concurrent frames the throughput the overlapped streams reach, which the per-launch
            # timing above (one frame's kernels alone) cannot show
            it_flops = sum(v["pairs"] * (_lib.flops_per_pair(k, Dw) or 0) for k, v in summ.items()) / prof_iters
            it_s = elapsed / args.steps
            roof["aggregate_achieved"] = round(it_flops / it_s / 1e12, 3)
            roof["aggregate_frac"] = round(it_flops / it_s / 1e12 / FP32_PEAK_TFLOPS, 4)
            roof["aggregate_note"] = ("algorithmic flops of all pair passes of one iteration "
                                      + ("(counted on the profiled sequential iteration) " if concurrent else "")
                                      + "/ the timed iterations' wall time per iteration / peak")
            clk, busy = load_issue(dom) if traffic is not None else (None, None)
            if clk:
                # the 157.3 TF/s peak assumes the 2.4 GHz peak clock; under this load the chip
                # runs at the DVFS clock GRBM_GUI_ACTIVE reports (profiles/pmc_issue.json)
                roof["pmc_eff_clock_GHz"] = round(clk, 3)
                roof["pmc_valu_issue_busy"] = round(busy, 3) if busy else None
                # the EXECUTED flops (hot-loop instruction count, exec_flops_per_pair) against
                # the peak at that clock: the algorithmic count prices work the pair-once
                # kernels do not execute, so its ratio to the clock-scaled peak can exceed 1
                if efpp and fpp:
                    roof["frac_executed_at_eff_clock"] = round(
                        achieved * efpp / fpp / (FP32_PEAK_TFLOPS * clk / 2.4), 4)
        base = None
        if not args.no_cpu_baseline and world == 1 and pair_counts:
            try:
                base = cpu_baseline(pair_counts, min(wl["N"], 50000), D=wl.get("D", 3))
            except Exception as e:  # baseline is informative; never fail the bench on it
                base = {"error": repr(e)}
        ksum = ksum_xy = None
        if world == 1 and wl.get("N") == 100000 and wl.get("D", 3) == 3:
            try:
                ksum = kernel_sum_probe(dev, wl["N"])
                ksum_xy = kernel_sum_probe(dev, wl["N"], same=False)
            except Exception as e:  # informative; never fail the bench on it
                ksum = {"error": repr(e)}
        tot_ms = sum(v["ms"] for v in summ.values())
        kern_gbps = (round(sum(v["bytes"] for v in summ.values()) / (tot_ms * 1e-3) / 1e9, 3)
                     if tot_ms > 0 else None)
        if getattr(psr, "batch_stats", None):
            cfg["batch_stats_last_reg_opt"] = psr.batch_stats
        if rehearse:
            cfg["parallelism"] = (cfg["parallelism"].replace("RCCL", "gloo")
                                  + " -- REHEARSAL: every rank on cuda:0 over gloo, not RCCL")
        works = [r["work_s"] for r in ranks]
        per_rank = {"ranks": ranks, "FE_identical_on_all_ranks": len({r["FE"] for r in ranks}) == 1,
                    "work_s_max_over_min": round(max(works) / max(min(works), 1e-9), 4),
                    "closures_max_over_min": (round(max(r["closures"] for r in ranks)
                                                    / max(min(r["closures"] for r in ranks), 1), 4)),
                    "note": "per rank over the timed steps: work_s = time to its own last kernel "
                            "(before the closing barrier), closures = L-BFGS loss evaluations, "
                            "em_steps, collectives (count) and collective_s (host wall time inside "
                            "the blocking ones: the exchange plus waiting for the slowest rank), "
                            "kernel_busy_s = summed kernel time (timed iterations only; absent when frames run concurrently, whose per-launch event times overlap)"}
        line = {
            "metric": METRIC, "value": round(value, 5), "unit": "PSR iterations/sec",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": scaling, "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": cfg, "roofline": roof, "cpu_baseline": base,
            "kernel_sum_hbm_GBps": kern_gbps,
            "kernel_sum_100k": ksum,
            "kernel_sum_100k_xy": ksum_xy,
            "per_rank": per_rank,
            "kernels": {k: {"launches": v["launches"], "ms": round(v["ms"], 3),
                            "Gpairs": round(v["pairs"] / 1e9, 3)} for k, v in summ.items()},
        }
        print(json.dumps(line), file=out, flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
