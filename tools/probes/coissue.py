"""FMA / v_exp_f32 co-issue probe (libdifficp_microbench.so kinds 30-35): per iteration 16
independent v_fma_f32 chains plus NE exps (inputs: chain values, results: the next iteration's
multipliers), compiler-scheduled (exps clustered) or interleaved one exp per 16/NE FMAs
(LLVM sched_group_barrier).  Prints SIMD cycles per wave-iteration at the nominal 2.4 GHz and
the extra cycles per exp against NE = 0.

    python tools/probes/coissue.py
"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    mb = ctypes.CDLL(os.path.join(ROOT, "diff-icp_amd", "libdifficp_microbench.so"))
    mb.dicp_mb_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    out = torch.zeros(256, device="cuda")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    blocks, iters = 256 * 8 * 4, 4096
    kinds = {30: ("NE=0", 0), 31: ("NE=2 clustered", 2), 32: ("NE=4 clustered", 4),
             33: ("NE=8 clustered", 8), 35: ("NE=2 interleaved", 2), 34: ("NE=4 interleaved", 4)}
    res = {}
    for rep in range(2):
        for k, (name, ne) in kinds.items():
            best = None
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                rc = mb.dicp_mb_launch(k, blocks, iters, ctypes.c_void_p(out.data_ptr()), st)
                e1.record()
                e1.synchronize()
                assert rc == 0
                ms = e0.elapsed_time(e1)
                best = ms if best is None else min(best, ms)
            cyc = best * 1e-3 * 2.4e9 * 1024 / (blocks * 4 * iters)
            res[name] = min(res.get(name, 1e9), cyc)
    base = res["NE=0"]
    line = {"cycles_per_wave_iter_at_2.4GHz": {k: round(v, 2) for k, v in res.items()},
            "extra_cycles_per_exp": {k: round((v - base) / ne, 2) for k, (n, ne) in
                                     ((n, (n, ne)) for _, (n, ne) in kinds.items()) if ne for v in [res[k]]},
            "fma_cycles_per_instr": round(base / 16, 2)}
    print(json.dumps(line))


if __name__ == "__main__":
    main()
