"""A/B of the 2k-point host floor (tools/host_floor.py's measurement) between two copies of the
Python package on the same box, alternated in subprocesses: the round-6 host-floor changes
(tools/_ab_old = the package at 81c00d0, tools/_ab_mid = dad1162 with the L-BFGS algebra
still on the device; same HIP library) against the tree's own.

    python tools/probes/host_floor_ab.py [--reps 3] [--iters 5] [--N 2000]
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def child(root, N, iters):
    sys.path.insert(0, root)
    import torch
    from difficp_amd import workloads
    dev = torch.device("cuda:0")
    psr = workloads.build_two_set(N, dev, seed=0)
    workloads.psr_iteration(psr)
    workloads.psr_iteration(psr)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        workloads.psr_iteration(psr)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--N", type=int, default=2000)
    ap.add_argument("--child")
    a = ap.parse_args()
    if a.child:
        print(json.dumps({"ms_per_iter": child(a.child, a.N, a.iters)}), flush=True)
        return
    variants = {"r06_start_81c00d0": os.path.join(ROOT, "tools", "_ab_old"),
                "device_lbfgs_algebra_dad1162": os.path.join(ROOT, "tools", "_ab_mid"), "tree": ROOT}
    res = {k: [] for k in variants}
    env = dict(os.environ, DICP_LIB_PATH=os.path.join(ROOT, "diff-icp_amd", "libdifficp_hip.so"))
    for _ in range(a.reps):
        for k, root in variants.items():
            out = subprocess.run([sys.executable, __file__, "--child", root, "--N", str(a.N),
                                  "--iters", str(a.iters)], capture_output=True, text=True, env=env,
                                 timeout=300)
            if out.returncode != 0:
                print(out.stdout[-2000:], out.stderr[-4000:])
                sys.exit(out.returncode)
            line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1]
            res[k].append(round(json.loads(line)["ms_per_iter"], 2))
            print(k, res[k][-1], flush=True)
    print(json.dumps({"N": a.N, "iters": a.iters, "ms_per_iter": res,
                      "best": {k: min(v) for k, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
