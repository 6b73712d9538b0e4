"""Does the f32 MFMA pipe overlap VALU work on gfx950?  Times microbench.hip's
mfma_mix_probe: MFMA only, VALU only (24 FMA + 4 exp per iteration), both in one wave, and
split across the waves of a workgroup, at several workgroups per CU."""
import ctypes
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
mb = ctypes.CDLL(os.path.join(ROOT, "diff-icp_amd", "libdifficp_microbench.so"))
mb.dicp_mb_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]


def t(kind, blocks, iters):
    out = torch.zeros(256, device="cuda")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for _ in range(2):
        assert mb.dicp_mb_launch(kind, blocks, iters, ctypes.c_void_p(out.data_ptr()), st) == 0
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        mb.dicp_mb_launch(kind, blocks, iters, ctypes.c_void_p(out.data_ptr()), st)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / 5


for wg_per_cu in (2, 4, 8):
    blocks = 256 * wg_per_cu
    iters = 20000
    r = {k: t(k, blocks, iters) for k in (10, 11, 12, 13)}
    # cycles per iteration per wave, at a nominal 2.4 GHz, per SIMD (waves/SIMD = wg_per_cu)
    cyc = {k: v * 1e-3 * 2.4e9 / (iters * wg_per_cu) for k, v in r.items()}
    print(f"WG/CU {wg_per_cu}: ms mfma {r[10]:.3f} valu {r[11]:.3f} same-wave {r[12]:.3f} "
          f"cross-wave {r[13]:.3f} | SIMD cycles/iter/wave @2.4GHz: mfma {cyc[10]:.1f} valu {cyc[11]:.1f} "
          f"same {cyc[12]:.1f} cross {cyc[13]:.1f}", flush=True)

for wg_per_cu in (2, 4, 8):
    blocks = 256 * wg_per_cu
    iters = 20000
    r = {k: t(k, blocks, iters) for k in (20, 21, 22)}
    cyc = {k: v * 1e-3 * 2.4e9 / (iters * wg_per_cu) for k, v in r.items()}
    print(f"bf16 16x16x32 WG/CU {wg_per_cu}: ms mfma {r[20]:.3f} valu {r[21]:.3f} same-wave {r[22]:.3f} | "
          f"SIMD cycles/iter/wave @2.4GHz: mfma {cyc[20]:.1f} valu {cyc[21]:.1f} same {cyc[22]:.1f}", flush=True)
