// Peak-rate probes for the roofline of the pair kernels (diagnostic library, not the product):
// v_exp_f32 throughput, v_fma_f32 / v_pk_fma_f32 throughput.  Each thread runs ITER
// iterations of UNROLL independent chains so issue (not latency) bounds the loop.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int kChains = 8;

__global__ __launch_bounds__(256) void exp_probe(float* out, int iters, float seed) {
  float a[kChains];
#pragma unroll
  for (int k = 0; k < kChains; ++k) a[k] = seed * (threadIdx.x + k) * 1e-7f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < kChains; ++k) a[k] = __builtin_amdgcn_exp2f(a[k]) - 1.0f;
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < kChains; ++k) s += a[k];
  if (s == 12345.f) out[threadIdx.x] = s;  // keep live
}

__global__ __launch_bounds__(256) void fma_probe(float* out, int iters, float seed) {
  float a[kChains], b[kChains];
#pragma unroll
  for (int k = 0; k < kChains; ++k) {
    a[k] = seed * (threadIdx.x + k);
    b[k] = seed * 0.5f + k;
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < kChains; ++k) a[k] = fmaf(a[k], b[k], 0.999f);
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < kChains; ++k) s += a[k];
  if (s == 12345.f) out[threadIdx.x] = s;
}

typedef float float2v __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void pkfma_probe(float* out, int iters, float seed) {
  float2v a[kChains], b[kChains], c;
  c.x = 0.999f;
  c.y = 0.998f;
#pragma unroll
  for (int k = 0; k < kChains; ++k) {
    a[k].x = seed * (threadIdx.x + k);
    a[k].y = seed * (threadIdx.x + 2 * k);
    b[k].x = seed * 0.5f + k;
    b[k].y = seed * 0.25f + k;
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < kChains; ++k) a[k] = __builtin_elementwise_fma(a[k], b[k], c);
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < kChains; ++k) s += a[k].x + a[k].y;
  if (s == 12345.f) out[threadIdx.x] = s;
}

// DPP-add throughput: a[k] = dpp(a[k]) + b[k] on kChains independent chains
// (CTRL 0x134 = wave_rol:1, 0x121 = row_ror:1).
template <int CTRL>
__global__ __launch_bounds__(256) void dppadd_probe(float* out, int iters, float seed) {
  float a[kChains], b[kChains];
#pragma unroll
  for (int k = 0; k < kChains; ++k) {
    a[k] = seed * (threadIdx.x + k);
    b[k] = seed * 0.5f + k;
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < kChains; ++k)
      a[k] = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(a[k]), CTRL, 0xF, 0xF, false)) + b[k];
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < kChains; ++k) s += a[k];
  if (s == 12345.f) out[threadIdx.x] = s;
}

// Co-issue probe: per iteration kChains FMAs and ONE exp2 on an independent chain; compare
// its time with fma_probe (same FMAs, no exp) and exp_probe.
__global__ __launch_bounds__(256) void mix_probe(float* out, int iters, float seed) {
  float a[kChains], b[kChains];
  float e = seed * threadIdx.x * 1e-7f;
#pragma unroll
  for (int k = 0; k < kChains; ++k) {
    a[k] = seed * (threadIdx.x + k);
    b[k] = seed * 0.5f + k;
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < kChains; ++k) a[k] = fmaf(a[k], b[k], 0.999f);
    e = __builtin_amdgcn_exp2f(e) - 1.0f;
  }
  float s = e;
#pragma unroll
  for (int k = 0; k < kChains; ++k) s += a[k];
  if (s == 12345.f) out[threadIdx.x] = s;
}

typedef float f4v __attribute__((ext_vector_type(4)));

// MFMA / VALU overlap probes (the matrix-core forward's loop shape): per iteration
//   MODE 0: 4 independent v_mfma_f32_16x16x4_f32 (MFMA only)
//   MODE 1: 24 v_fma_f32 + 4 v_exp_f32 on independent chains (VALU only)
//   MODE 2: both in the same wave, interleaved (each MFMA's A operand = a fresh exp result)
//   MODE 3: waves 0,2 of the workgroup run MODE 0's body, waves 1,3 MODE 1's (cross-wave)
template <int MODE>
__global__ __launch_bounds__(256) void mfma_mix_probe(float* out, int iters, float seed) {
  const int wv = threadIdx.x >> 6;
  const bool do_m = MODE == 0 || MODE == 2 || (MODE == 3 && (wv & 1) == 0);
  const bool do_v = MODE == 1 || MODE == 2 || (MODE == 3 && (wv & 1) == 1);
  f4v acc[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) acc[k] = f4v{0.f, 0.f, 0.f, 0.f};
  float a[6], b = seed * 0.5f, e[4];
#pragma unroll
  for (int k = 0; k < 6; ++k) a[k] = seed * (threadIdx.x + k) * 1e-3f;
#pragma unroll
  for (int k = 0; k < 4; ++k) e[k] = seed * (threadIdx.x + k) * 1e-7f;
  const float bm = seed * 1e-3f * (threadIdx.x & 15);
  for (int it = 0; it < iters; ++it) {
    if (do_v) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int k = 0; k < 6; ++k) a[k] = fmaf(a[k], b, 0.999f);
        e[r] = __builtin_amdgcn_exp2f(-e[r] * e[r]);
        if (do_m) acc[r] = __builtin_amdgcn_mfma_f32_16x16x4f32(e[r], bm, acc[r], 0, 0, 0);
      }
    } else if (do_m) {
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[r] = __builtin_amdgcn_mfma_f32_16x16x4f32(e[r], bm, acc[r], 0, 0, 0);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 6; ++k) s += a[k];
#pragma unroll
  for (int r = 0; r < 4; ++r) s += e[r] + acc[r][0] + acc[r][1] + acc[r][2] + acc[r][3];
  if (s == 12345.f) out[threadIdx.x] = s;
}

typedef short bf8v __attribute__((ext_vector_type(8)));

// The same with v_mfma_f32_16x16x32_bf16 (16 cycles, 16x as many flops): per iteration
//   MODE 0: 4 MFMAs, MODE 1: 24 FMA + 4 exp, MODE 2: both in one wave (the A operand of each
//   MFMA takes bits of a fresh exp result)
template <int MODE>
__global__ __launch_bounds__(256) void bf16_mix_probe(float* out, int iters, float seed) {
  f4v acc[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) acc[k] = f4v{0.f, 0.f, 0.f, 0.f};
  float a[6], b = seed * 0.5f, e[4];
#pragma unroll
  for (int k = 0; k < 6; ++k) a[k] = seed * (threadIdx.x + k) * 1e-3f;
#pragma unroll
  for (int k = 0; k < 4; ++k) e[k] = seed * (threadIdx.x + k) * 1e-7f;
  bf8v bm;
#pragma unroll
  for (int k = 0; k < 8; ++k) bm[k] = (short)(0x3f80 + (threadIdx.x & 7) + k);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (MODE >= 1) {
#pragma unroll
        for (int k = 0; k < 6; ++k) a[k] = fmaf(a[k], b, 0.999f);
        e[r] = __builtin_amdgcn_exp2f(-e[r] * e[r]);
      }
      if (MODE != 1) {
        bf8v av = bm;
        if (MODE == 2) av[0] = (short)(__float_as_uint(e[r]) >> 16);
        acc[r] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bm, acc[r], 0, 0, 0);
      }
    }
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 6; ++k) s += a[k];
#pragma unroll
  for (int r = 0; r < 4; ++r) s += e[r] + acc[r][0] + acc[r][1] + acc[r][2] + acc[r][3];
  if (s == 12345.f) out[threadIdx.x] = s;
}

// FMA / transcendental co-issue probe: per iteration 16 independent FMA chains and NE v_exp_f32
// whose inputs are chain values and whose results are the next iteration's multipliers of NE
// chains (no extra instructions); compare the time per iteration across NE = 0, 2, 4, 8:
// + ~10 SIMD cycles per exp = the exps serialise with the FMAs, + ~2 = they overlap.
template <int NE, bool ILV = false>
__global__ __launch_bounds__(256) void coissue_probe(float* out, int iters, float seed) {
  float a[16], m[16];
  const float c = seed * 0.999f;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    a[k] = seed * (threadIdx.x + k) * 1e-3f;
    m[k] = seed * (0.5f + k * 1e-3f);
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 16; ++k) a[k] = fmaf(a[k], m[k], c);
#pragma unroll
    for (int r = 0; r < NE; ++r) m[r] = __builtin_amdgcn_exp2f(a[(r + 8) & 15]);
    if constexpr (ILV) {  // one transcendental, then 16 / NE FMAs, repeated (LLVM sched groups)
#pragma unroll
      for (int r = 0; r < NE; ++r) {
        __builtin_amdgcn_sched_group_barrier(0x0400, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x0002, 16 / NE, 0);
      }
    }
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < 16; ++k) s += a[k] + m[k];
  if (s == 12345.f) out[threadIdx.x] = s;
}

// Packed / scalar issue mix: per iteration NPK independent v_pk_fma_f32 chains and NSC scalar
// FMA chains (FMAC: accumulator form a = fma(m, c, a) -> v_fmac_f32 (VOP2); else a = fma(a, m, c)
// -> v_fma_f32 (VOP3)); DPP > 0: NSC of the scalar ops are v_add_f32 with a wave_rol:1 DPP
// source instead.  Answers whether scalar f32 ops keep their ~2.4-cycle issue cost among packed
// ones.
typedef float f2v __attribute__((ext_vector_type(2)));
template <int NPK, int NSC, bool FMAC, bool DPP = false>
__global__ __launch_bounds__(256) void pkmix_probe(float* out, int iters, float seed) {
  f2v ap[NPK > 0 ? NPK : 1], mp[NPK > 0 ? NPK : 1];
  float a[NSC > 0 ? NSC : 1], m[NSC > 0 ? NSC : 1];
  const float c = seed * 0.999f;
  const f2v cp = {c, c};
#pragma unroll
  for (int k = 0; k < NPK; ++k) {
    ap[k] = f2v{seed * (threadIdx.x + k), seed * (threadIdx.x - k)} * 1e-3f;
    mp[k] = f2v{seed * (0.5f + k * 1e-3f), seed * (0.5f - k * 1e-3f)};
  }
#pragma unroll
  for (int k = 0; k < NSC; ++k) {
    a[k] = seed * (threadIdx.x + 3 * k) * 1e-3f;
    m[k] = seed * (0.5f + 2e-3f * k);
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < NPK; ++k) ap[k] = __builtin_elementwise_fma(ap[k], mp[k], cp);
#pragma unroll
    for (int k = 0; k < NSC; ++k) {
      if constexpr (DPP)
        a[k] = a[k] + __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, m[k]), 0x134, 0xF, 0xF, false));
      else if constexpr (FMAC)
        a[k] = fmaf(m[k], c, a[k]);
      else
        a[k] = fmaf(a[k], m[k], c);
    }
  }
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NPK; ++k) s += ap[k].x + ap[k].y;
#pragma unroll
  for (int k = 0; k < NSC; ++k) s += a[k];
  if (s == 12345.f) out[threadIdx.x] = s;
}

template <int CTRL>
__global__ __launch_bounds__(64) void dpp_probe(int* out) {
  const int l = threadIdx.x;
  out[l] = __builtin_amdgcn_update_dpp(-1, l, CTRL, 0xF, 0xF, false);
}

__global__ __launch_bounds__(256) void exp2_eval(const float* __restrict__ x, float* __restrict__ y, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) y[i] = __builtin_amdgcn_exp2f(x[i]);
}

}  // namespace

// y[i] = v_exp_f32(x[i]) (the pair kernels' fast_exp2), for accuracy probes
// (tools/probes/exp2_bias.py)
extern "C" int dicp_mb_exp2_eval(const float* x, float* y, int64_t n, void* stream) {
  if (n <= 0) return 0;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  exp2_eval<<<dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st>>>(x, y, n);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// Lane map of a wave-wide DPP rotate: out[l] = source lane read by lane l
// (which = 0: wave_rol:1 (0x134), 1: wave_ror:1 (0x13C)); one wave64.
extern "C" int dicp_mb_dpp(int which, int* out, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (which == 0) dpp_probe<0x134><<<1, 64, 0, st>>>(out);
  else dpp_probe<0x13C><<<1, 64, 0, st>>>(out);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// kind: 0 = exp2, 1 = fma, 2 = pk_fma, 3 = dpp(wave_rol:1)+add, 4 = dpp(row_ror:1)+add,
// 5 = kChains fma + 1 exp2 per iteration, 10..13 = mfma_mix_probe<kind - 10>,
// 40..47 = pkmix_probe (packed / scalar / DPP issue mixes, see there),
// 30..33 = coissue_probe<0, 2, 4, 8> (16 fma + NE exp2 per iteration), 34 / 35 = NE 4 / 2
// interleaved one exp per 16 / NE fma.  Returns 0 on
// success.  ops per launch: blocks*256*iters*kChains (x2 lanes for pk_fma).
extern "C" int dicp_mb_launch(int kind, int blocks, int iters, float* out, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  dim3 g(blocks), b(256);
  if (kind == 0) exp_probe<<<g, b, 0, st>>>(out, iters, 1.0f);
  else if (kind == 1) fma_probe<<<g, b, 0, st>>>(out, iters, 1.0f);
  else if (kind == 2) pkfma_probe<<<g, b, 0, st>>>(out, iters, 1.0f);
  else if (kind == 3) dppadd_probe<0x134><<<g, b, 0, st>>>(out, iters, 1.0f);
  else if (kind == 4) dppadd_probe<0x121><<<g, b, 0, st>>>(out, iters, 1.0f);
  else if (kind == 5) mix_probe<<<g, b, 0, st>>>(out, iters, 1.0f);
  else if (kind == 10) mfma_mix_probe<0><<<g, b, 0, st>>>(out, iters, 1.0f);
  else if (kind == 11) mfma_mix_probe<1><<<g, b, 0, st>>>(out, iters, 1.0f);
  else if (kind == 12) mfma_mix_probe<2><<<g, b, 0, st>>>(out, iters, 1.0f);
  else if (kind == 13) mfma_mix_probe<3><<<g, b, 0, st>>>(out, iters, 1.0f);
  else if (kind == 30) coissue_probe<0><<<g, b, 0, st>>>(out, iters, 1.0f);
  else if (kind == 31) coissue_probe<2><<<g, b, 0, st>>>(out, iters, 1.0f);
  else if (kind == 32) coissue_probe<4><<<g, b, 0, st>>>(out, iters, 1.0f);
  else if (kind == 33) coissue_probe<8><<<g, b, 0, st>>>(out, iters, 1.0f);
  else if (kind == 34) coissue_probe<4, true><<<g, b, 0, st>>>(out, iters, 1.0f);
  else if (kind == 35) coissue_probe<2, true><<<g, b, 0, st>>>(out, iters, 1.0f);
  else if (kind == 40) pkmix_probe<0, 16, false><<<g, b, 0, st>>>(out, iters, 1.0f);
  else if (kind == 41) pkmix_probe<0, 16, true><<<g, b, 0, st>>>(out, iters, 1.0f);
  else if (kind == 42) pkmix_probe<8, 0, false><<<g, b, 0, st>>>(out, iters, 1.0f);
  else if (kind == 43) pkmix_probe<8, 8, false><<<g, b, 0, st>>>(out, iters, 1.0f);
  else if (kind == 44) pkmix_probe<8, 8, true><<<g, b, 0, st>>>(out, iters, 1.0f);
  else if (kind == 45) pkmix_probe<0, 16, false, true><<<g, b, 0, st>>>(out, iters, 1.0f);
  else if (kind == 46) pkmix_probe<8, 8, false, true><<<g, b, 0, st>>>(out, iters, 1.0f);
  else if (kind == 47) pkmix_probe<12, 4, true><<<g, b, 0, st>>>(out, iters, 1.0f);
  else if (kind == 20) bf16_mix_probe<0><<<g, b, 0, st>>>(out, iters, 1.0f);
  else if (kind == 21) bf16_mix_probe<1><<<g, b, 0, st>>>(out, iters, 1.0f);
  else if (kind == 22) bf16_mix_probe<2><<<g, b, 0, st>>>(out, iters, 1.0f);
  else return 1;
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

extern "C" int dicp_mb_chains(void) { return kChains; }
