"""Accuracy of v_exp_f32 (the pair kernels' fast_exp2, libdifficp_microbench.so
dicp_mb_exp2_eval) against the float64 exp2 of the same float32 argument: mean (bias) and RMS
relative error per argument range.  A bias that depends on the argument is a systematic error
of every kernel value K = 2^-r2 (tools/probes/logdet_cost_diag.py).

    python tools/probes/exp2_bias.py > out.jsonl   (GPU box)"""
import ctypes
import json
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    mb = ctypes.CDLL(os.path.join(ROOT, "diff-icp_amd", "libdifficp_microbench.so"))
    mb.dicp_mb_exp2_eval.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    dev = torch.device("cuda:0")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    g = torch.Generator(device=dev).manual_seed(0)
    for lo, hi in ((-1e-3, 0.0), (-0.05, 0.0), (-0.5, -0.05), (-1.0, -0.5), (-2.0, -1.0), (-4.0, -2.0),
                   (-8.0, -4.0), (-16.0, -8.0), (-30.0, -16.0)):
        x = lo + (hi - lo) * torch.rand(1 << 24, generator=g, device=dev)
        y = torch.empty_like(x)
        assert mb.dicp_mb_exp2_eval(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(y.data_ptr()), x.numel(), st) == 0
        torch.cuda.synchronize()
        ex = torch.exp2(x.double())
        r = (y.double() - ex) / ex
        rt = (torch.exp2(x).double() - ex) / ex     # torch's float32 exp2, for comparison
        ulp = 2.0 ** -23
        print(json.dumps({"range": [lo, hi], "v_exp_mean_rel": float(r.mean()), "v_exp_rms_rel": float(r.pow(2).mean().sqrt()),
                          "v_exp_max_ulp": float(r.abs().max()) / ulp, "torch_mean_rel": float(rt.mean()),
                          "torch_rms_rel": float(rt.pow(2).mean().sqrt())}), flush=True)


if __name__ == "__main__":
    main()
