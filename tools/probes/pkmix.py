"""Issue cost of packed / scalar / DPP f32 instruction mixes (libdifficp_microbench.so kinds
40-47, `pkmix_probe`): SIMD cycles per wave-iteration at the nominal 2.4 GHz, and per
instruction class solved from the pure streams.

    python tools/probes/pkmix.py
"""
import ctypes
import json
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
KINDS = {40: ("16 v_fma_f32", 0, 16, 0), 41: ("16 v_fmac_f32", 0, 16, 0), 42: ("8 v_pk_fma_f32", 8, 0, 0),
         43: ("8 pk + 8 v_fma", 8, 8, 0), 44: ("8 pk + 8 v_fmac", 8, 8, 0), 45: ("16 v_add_f32_dpp", 0, 0, 16),
         46: ("8 pk + 8 v_add_f32_dpp", 8, 0, 8), 47: ("12 pk + 4 v_fmac", 12, 4, 0)}


def main():
    mb = ctypes.CDLL(os.path.join(ROOT, "diff-icp_amd", "libdifficp_microbench.so"))
    mb.dicp_mb_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    out = torch.zeros(256, device="cuda")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    blocks, iters = 256 * 8 * 4, 4096
    res = {}
    for _ in range(2):
        for k, (name, npk, nsc, ndpp) in KINDS.items():
            best = None
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                assert mb.dicp_mb_launch(k, blocks, iters, ctypes.c_void_p(out.data_ptr()), st) == 0
                e1.record()
                e1.synchronize()
                ms = e0.elapsed_time(e1)
                best = ms if best is None else min(best, ms)
            cyc = best * 1e-3 * 2.4e9 * 1024 / (blocks * 4 * iters)
            res[name] = round(min(res.get(name, 1e9), cyc), 2)
    per = {"v_fma_f32": res["16 v_fma_f32"] / 16, "v_fmac_f32": res["16 v_fmac_f32"] / 16,
           "v_pk_fma_f32": res["8 v_pk_fma_f32"] / 8, "v_add_f32_dpp": res["16 v_add_f32_dpp"] / 16}
    pred = {"8 pk + 8 v_fma": 8 * (per["v_pk_fma_f32"] + per["v_fma_f32"]),
            "8 pk + 8 v_fmac": 8 * (per["v_pk_fma_f32"] + per["v_fmac_f32"]),
            "8 pk + 8 v_add_f32_dpp": 8 * (per["v_pk_fma_f32"] + per["v_add_f32_dpp"]),
            "12 pk + 4 v_fmac": 12 * per["v_pk_fma_f32"] + 4 * per["v_fmac_f32"]}
    print(json.dumps({"cycles_per_wave_iter_at_2.4GHz": res,
                      "cycles_per_instr_pure": {k: round(v, 2) for k, v in per.items()},
                      "mix_measured_vs_sum_of_pure": {k: [res[k], round(v, 2)] for k, v in pred.items()}}))


if __name__ == "__main__":
    main()
