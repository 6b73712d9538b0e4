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

template <int CTRL>
__global__ __launch_bounds__(64) void dpp_probe(int* out) {
  const int l = threadIdx.x;
  out[l] = __builtin_amdgcn_update_dpp(-1, l, CTRL, 0xF, 0xF, false);
}

}  // namespace

// Lane map of a wave-wide DPP rotate: out[l] = source lane read by lane l
// (which = 0: wave_rol:1 (0x134), 1: wave_ror:1 (0x13C)); one wave64.
extern "C" int dicp_mb_dpp(int which, int* out, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (which == 0) dpp_probe<0x134><<<1, 64, 0, st>>>(out);
  else dpp_probe<0x13C><<<1, 64, 0, st>>>(out);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// kind: 0 = exp2, 1 = fma, 2 = pk_fma, 3 = dpp(wave_rol:1)+add, 4 = dpp(row_ror:1)+add,
// 5 = kChains fma + 1 exp2 per iteration.  Returns 0 on success.  ops per launch:
// blocks*256*iters*kChains (x2 lanes for pk_fma).
extern "C" int dicp_mb_launch(int kind, int blocks, int iters, float* out, void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  dim3 g(blocks), b(256);
  if (kind == 0) exp_probe<<<g, b, 0, st>>>(out, iters, 1.0f);
  else if (kind == 1) fma_probe<<<g, b, 0, st>>>(out, iters, 1.0f);
  else if (kind == 2) pkfma_probe<<<g, b, 0, st>>>(out, iters, 1.0f);
  else if (kind == 3) dppadd_probe<0x134><<<g, b, 0, st>>>(out, iters, 1.0f);
  else if (kind == 4) dppadd_probe<0x121><<<g, b, 0, st>>>(out, iters, 1.0f);
  else mix_probe<<<g, b, 0, st>>>(out, iters, 1.0f);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

extern "C" int dicp_mb_chains(void) { return kChains; }
