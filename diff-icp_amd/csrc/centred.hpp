// Centred-expansion row reductions for the Gaussian-kernel sums whose pair term is linear in
// the column fields (KBase, KRedScal, KRed, GradKRed, the external-point ODE forward).
//
// The generic skeleton (common.hpp) spends 9-10 VALU + 1 exp per pair on KRed: 3 sub + 3 fma
// for r2 = |x - y|^2, a multiply by -log2(e)/(2 sigma^2), the exp and 3 fma.  Here the
// columns are visited in a spatial (Morton) order and grouped into sub-tiles of 64 (one
// wave's worth, built by one wave in the prep pass); each sub-tile t has a centre c_t, and in
// scaled coordinates (X = alpha (x - c_t), Y = alpha (y - c_t), alpha = sqrt(log2 e / (2 sigma^2)))
//     K = exp2(-|X - Y|^2) = exp2(m - |X|^2) * exp2(2 X.Y - |Y|^2 - m)
// where 2Y and -|Y|^2 - m are stored in the column record and the row factor
// F = exp2(m - |X|^2) is formed once per (row, sub-tile) and applied to the sub-tile's partial
// sums: the exponent costs 3 fma, the whole KRed pair 6 VALU + 1 exp (the generic skeleton:
// 10).  Terms linear in z = x - y are summed as X sum K - sum K Y (per sub-tile, then folded
// into the row's totals), so GradKRed costs 7 VALU + exp and the external-point forward 7-11.
// Range (m = 16, sub-tile radius rho <= 4): 2 X.Y - |Y|^2 - m <= 2 rho |X| - m stays finite
// for |X| <= 14, and rows farther than 14 scaled units from a sub-tile (F = 0 in float32) are
// clamped to |X| = 14 -- their contributions from it are below 2^-140 and vanish either way;
// F itself underflows (below 2^-126) only for rows more than ~12 scaled units (~14 sigma)
// from the sub-tile, whose contributions are below 2^-(12 - rho)^2.
//
// Accuracy: X and Y are formed from RAW differences (x - c_t, y - c_t, then scaled), so their
// rounding is relative to the distance from the sub-tile centre, not to the coordinates'
// magnitude; the cancellation error of the expanded exponent is ~eps (|X|^2 + |Y|^2), small
// where K matters (|X - Y| = O(1) and |Y| <= rho_t, the sub-tile radius).  A sub-tile whose
// radius exceeds rho_max (cx_rho_x100 / 100 scaled units, default 1.5) is summed in the
// difference form on the raw coordinates, z = alpha (x - y) (the record also carries y), with
// the z-linear terms accumulated directly -- the generic skeleton's arithmetic.  Checked
// against float64 in tests/test_gpu_centred.py (compact, wide and offset clouds).
// Deterministic: the sort is a stable radix sort of Morton codes, summation order fixed.
#pragma once
#include "launch.hpp"
#include "lddmm_ops.hpp"
#include "packed.hpp"

namespace dicp {

// The compact pair terms are written once for a scalar row (T = float) and for two rows
// packed in one VGPR pair (T = f2: every fma is one v_pk_fma_f32, the column field broadcast
// into both halves), so the packed loop is bitwise the scalar one.
template <class T> __device__ __forceinline__ T bc(float x);
template <> __device__ __forceinline__ float bc<float>(float x) { return x; }
template <> __device__ __forceinline__ f2 bc<f2>(float x) { return splat(x); }
__device__ __forceinline__ float vfma(float a, float b, float c) { return fmaf(a, b, c); }
__device__ __forceinline__ f2 vfma(f2 a, f2 b, f2 c) { return pk_fma(a, b, c); }

constexpr int kSub = 64;  // columns per centred sub-tile (one wave64 in the prep pass)
constexpr float kCxShift = 16.f;     // m: exponent shift between the row factor and the pair term
constexpr float kCxClamp = 14.f;     // |X| clamp (see above); needs rho <= kCxRhoCap
constexpr float kCxRhoCap = 4.f;     // largest sub-tile radius the expanded form accepts
#ifndef DICP_CX_PK
#define DICP_CX_PK 1
#endif
constexpr bool kCxPk = DICP_CX_PK != 0;  // packed compact loop (two rows per v_pk_fma_f32)

// ---- ops: record = [2Y_0, 2Y_1 | c, c | 2Y_2 (D = 3) | fields... | y (D, raw)] -------------
// c = -|Y|^2 - m, stored twice: the packed loop takes the aligned pair (rec[2], rec[3]) as the
// exponent's initial value for both rows without a register copy, and a D = 3 KRed record's
// compact part is two whole float4s (ds_read_b128: 4 LDS cycles per wave; a 3-float tail
// would be a ds_read_b96, 8 cycles, MI355X_MICROARCH.md LDS table).
constexpr int kCxC = 2;                                            // c, c at rec[2], rec[3]
template <int D> constexpr int cx_f = D + 2;                       // first field
__host__ __device__ constexpr int cx_y(int d) { return d < 2 ? d : d + 2; }   // 2Y_d
// pair(K, e, rec, acc): compact sub-tiles (K without the row factor F, e its exponent);
// pair_z(K, e, z, rec, acc): wide sub-tiles, z = alpha (x - y) from raw coordinates, the
// z-linear sums accumulated directly in the slots the compact form uses for its Y sums;
// fold(X, acc, tot, compact, F, Es) adds a sub-tile's partial sums into the row's totals
// (compact: times F = exp2(Es), with the X terms; wide: as they are).
template <int D>
struct CxBase {
  static constexpr int kPre = D + 1;
};

// KBase: sum_j K                                                     kernel.py:131 / :178
template <int D>
struct CxKBase : CxBase<D> {
  static constexpr int kRaw = cx_f<D>;
  static constexpr int RW4 = cw4(kRaw + D), NACC = 1, NTOT = 1, kNOut = 1;
  static constexpr int kOutW[4] = {1, 0, 0, 0};
  __device__ static void build(const Args&, int64_t, const float*, float*) {}
  template <class T>
  __device__ static void pair(T K, T, const float*, T* acc) { acc[0] += K; }
  __device__ static void pair_z(float K, float e, const float*, const float* rec, float* acc) { pair(K, e, rec, acc); }
  __device__ static void fold(const float*, const float* acc, float* tot, bool c, float F, float) {
    tot[0] = fmaf(c ? F : 1.f, acc[0], tot[0]);
  }
  __device__ static void store(const Scal&, float, const float* t, float* v) { v[0] = t[0]; }
};

// KRedScal: sum_j K d_j                                              kernel.py:135 / :182
template <int D>
struct CxKRedScal : CxBase<D> {
  static constexpr int kRaw = cx_f<D> + 1;
  static constexpr int RW4 = cw4(kRaw + D), NACC = 1, NTOT = 1, kNOut = 1;
  static constexpr int kOutW[4] = {1, 0, 0, 0};
  __device__ static void build(const Args& a, int64_t o, const float*, float* rec) { rec[cx_f<D>] = a.c1[o]; }
  template <class T>
  __device__ static void pair(T K, T, const float* rec, T* acc) { acc[0] = vfma(K, bc<T>(rec[cx_f<D>]), acc[0]); }
  __device__ static void pair_z(float K, float e, const float*, const float* rec, float* acc) { pair(K, e, rec, acc); }
  __device__ static void fold(const float*, const float* acc, float* tot, bool c, float F, float) {
    tot[0] = fmaf(c ? F : 1.f, acc[0], tot[0]);
  }
  __device__ static void store(const Scal&, float, const float* t, float* v) { v[0] = t[0]; }
};

// KRed: sum_j K b_j  (the velocity field, LDDMM.py:114)             kernel.py:138 / :186
template <int D>
struct CxKRed : CxBase<D> {
  static constexpr int kRaw = cx_f<D> + D;
  static constexpr int RW4 = cw4(kRaw + D), NACC = D, NTOT = D, kNOut = 1;
  static constexpr int kOutW[4] = {D, 0, 0, 0};
  __device__ static void build(const Args& a, int64_t o, const float*, float* rec) {
#pragma unroll
    for (int d = 0; d < D; ++d) rec[cx_f<D> + d] = a.c1[o * D + d];
  }
  template <class T>
  __device__ static void pair(T K, T, const float* rec, T* acc) {
#pragma unroll
    for (int d = 0; d < D; ++d) acc[d] = vfma(K, bc<T>(rec[cx_f<D> + d]), acc[d]);
  }
  __device__ static void pair_z(float K, float e, const float*, const float* rec, float* acc) { pair(K, e, rec, acc); }
  __device__ static void fold(const float*, const float* acc, float* tot, bool c, float F, float) {
    const float f = c ? F : 1.f;
#pragma unroll
    for (int d = 0; d < D; ++d) tot[d] = fmaf(f, acc[d], tot[d]);
  }
  __device__ static void store(const Scal&, float, const float* t, float* v) {
#pragma unroll
    for (int d = 0; d < D; ++d) v[d] = t[d];
  }
};

// GradKRed: -s sum_j K z = -(s/alpha) (X sum K - sum K Y)           kernel.py:142 / :190
// (wide sub-tiles: -(s/alpha) sum K z' accumulated directly)
template <int D>
struct CxGradK : CxBase<D> {
  static constexpr int kRaw = cx_f<D>;
  static constexpr int RW4 = cw4(kRaw + D), NACC = D + 1, NTOT = D, kNOut = 1;
  static constexpr int kOutW[4] = {D, 0, 0, 0};
  __device__ static void build(const Args&, int64_t, const float*, float*) {}
  template <class T>
  __device__ static void pair(T K, T, const float* rec, T* acc) {
    acc[0] += K;
#pragma unroll
    for (int d = 0; d < D; ++d) acc[1 + d] = vfma(K, bc<T>(rec[cx_y(d)]), acc[1 + d]);  // sum K 2Y
  }
  __device__ static void pair_z(float K, float, const float* z, const float*, float* acc) {
#pragma unroll
    for (int d = 0; d < D; ++d) acc[1 + d] = fmaf(K, z[d], acc[1 + d]);    // sum K z
  }
  __device__ static void fold(const float* X, const float* acc, float* tot, bool compact, float F, float) {
#pragma unroll
    for (int d = 0; d < D; ++d)
      tot[d] += compact ? F * fmaf(X[d], acc[0], -0.5f * acc[1 + d]) : acc[1 + d];
  }
  __device__ static void store(const Scal& sc, float sa, const float* t, float* v) {
#pragma unroll
    for (int d = 0; d < D; ++d) v[d] = -sa * t[d];
  }
};

// External points x carried by the flow (LDDMM.py:219-227), rows x, columns (q, p):
//   vx = sum K p_j + eta s sum K z,   gx = s sum K (z.p_j) + eta s sum K (s r2 - D)
// with z = (X - Y) / alpha, s r2 = kS2 r2' = -kS2 e (e = the computed exponent):
//   sum K (z.p_j) = (X.sum K p - sum K (Y.p_j)) / alpha  (w_j = Y.p_j in the record).
template <int D, bool ETA, bool DIV>
struct CxExtFwd : CxBase<D> {
  static constexpr int kP = cx_f<D>;                         // p_j slots
  static constexpr int kW = kP + D;                          // w_j slot
  static constexpr int kRaw = kP + D + (DIV ? 1 : 0);
  static constexpr int RW4 = cw4(kRaw + D);
  // acc: V (D) | W | K, K2Y (D), Ke  (wide sub-tiles: W <- sum K (z.p), K2Y <- sum K z)
  static constexpr int oW = D, oK = D + (DIV ? 1 : 0);
  static constexpr int NACC = oK + (ETA ? D + 2 : 0);
  // tot: V (D) | G | Z (D), L
  static constexpr int tG = D, tZ = D + (DIV ? 1 : 0);
  static constexpr int NTOT = tZ + (ETA ? D + 1 : 0);
  static constexpr int kNOut = 2;
  static constexpr int kOutW[4] = {D, 1, 0, 0};
  __device__ static void build(const Args& a, int64_t o, const float* Yc, float* rec) {
    float w = 0.f;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const float pd = a.c1[o * D + d];
      rec[kP + d] = pd;
      w = fmaf(Yc[d], pd, w);
    }
    if (DIV) rec[kW] = w;
  }
  template <class T>
  __device__ static void pair(T K, T e, const float* rec, T* acc) {
#pragma unroll
    for (int d = 0; d < D; ++d) acc[d] = vfma(K, bc<T>(rec[kP + d]), acc[d]);
    if (DIV) acc[oW] = vfma(K, bc<T>(rec[kW]), acc[oW]);
    if (ETA) {
      acc[oK] += K;
#pragma unroll
      for (int d = 0; d < D; ++d) acc[oK + 1 + d] = vfma(K, bc<T>(rec[cx_y(d)]), acc[oK + 1 + d]);
      acc[oK + 1 + D] = vfma(K, e, acc[oK + 1 + D]);
    }
  }
  __device__ static void pair_z(float K, float e, const float* z, const float* rec, float* acc) {
#pragma unroll
    for (int d = 0; d < D; ++d) acc[d] = fmaf(K, rec[kP + d], acc[d]);
    if (DIV) acc[oW] = fmaf(K, dot<D>(z, rec + kP), acc[oW]);
    if (ETA) {
      acc[oK] += K;
#pragma unroll
      for (int d = 0; d < D; ++d) acc[oK + 1 + d] = fmaf(K, z[d], acc[oK + 1 + d]);
      acc[oK + 1 + D] = fmaf(K, e, acc[oK + 1 + D]);
    }
  }
  __device__ static void fold(const float* X, const float* acc, float* tot, bool compact, float F, float Es) {
    const float f = compact ? F : 1.f;
#pragma unroll
    for (int d = 0; d < D; ++d) tot[d] = fmaf(f, acc[d], tot[d]);
    if (DIV) {
      float g = compact ? -acc[oW] : acc[oW];
      if (compact) {
#pragma unroll
        for (int d = 0; d < D; ++d) g = fmaf(X[d], acc[d], g);
      }
      tot[tG] = fmaf(f, g, tot[tG]);
    }
    if (ETA) {
#pragma unroll
      for (int d = 0; d < D; ++d)
        tot[tZ + d] += compact ? F * fmaf(X[d], acc[oK], -0.5f * acc[oK + 1 + d]) : acc[oK + 1 + d];
      // sum K e over the true exponents: compact pairs carry e - Es
      const float Ke = compact ? fmaf(Es, acc[oK], acc[oK + 1 + D]) : acc[oK + 1 + D];
      tot[tZ + D] += f * fmaf(-kS2, Ke, -(float)D * acc[oK]);
    }
  }
  __device__ static void store(const Scal& sc, float sa, const float* t, float* v) {
    const float s = sc.s, eta = sc.eta;
#pragma unroll
    for (int d = 0; d < D; ++d) v[d] = ETA ? fmaf(eta * sa, t[tZ + d], t[d]) : t[d];
    float g = DIV ? sa * t[tG] : 0.f;
    if (ETA && DIV) g = fmaf(eta * s, t[tZ + D], g);
    v[D] = g;
  }
};

// ---- prep pass ----------------------------------------------------------------------------
// bounding box of the columns, stage 1: each workgroup reduces a grid-strided share of the
// columns to (lo[D], hi[D]) in part[blockIdx.x]; the codes kernel reduces the parts (stage 2)
constexpr int kBoxBlocks = 256;
template <int D>
__global__ __launch_bounds__(256) void cx_bbox_kernel(const float* __restrict__ y, int64_t N, float* part) {
  __shared__ float red[2 * D][4];
  float lo[D], hi[D];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    lo[d] = __builtin_huge_valf();
    hi[d] = -__builtin_huge_valf();
  }
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < N; j += (int64_t)gridDim.x * blockDim.x) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const float v = y[j * D + d];
      lo[d] = fminf(lo[d], v);
      hi[d] = fmaxf(hi[d], v);
    }
  }
#pragma unroll
  for (int d = 0; d < D; ++d) {
    for (int off = 32; off > 0; off >>= 1) {
      lo[d] = fminf(lo[d], __shfl_xor(lo[d], off, 64));
      hi[d] = fmaxf(hi[d], __shfl_xor(hi[d], off, 64));
    }
  }
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      red[d][w] = lo[d];
      red[D + d][w] = hi[d];
    }
  }
  __syncthreads();
  if (threadIdx.x < 2 * D) {
    const int k = threadIdx.x;
    float v = red[k][0];
    for (int i = 1; i < 4; ++i) v = k < D ? fminf(v, red[k][i]) : fmaxf(v, red[k][i]);
    part[blockIdx.x * 2 * D + k] = v;
  }
}

__device__ __forceinline__ uint32_t spread3(uint32_t c) {  // 10 bits -> every third bit
  c = (c | (c << 16)) & 0x030000FFu;
  c = (c | (c << 8)) & 0x0300F00Fu;
  c = (c | (c << 4)) & 0x030C30C3u;
  c = (c | (c << 2)) & 0x09249249u;
  return c;
}
__device__ __forceinline__ uint32_t spread2(uint32_t c) {  // 15 bits -> every second bit
  c &= 0x7FFFu;
  c = (c | (c << 8)) & 0x00FF00FFu;
  c = (c | (c << 4)) & 0x0F0F0F0Fu;
  c = (c | (c << 2)) & 0x33333333u;
  c = (c | (c << 1)) & 0x55555555u;
  return c;
}

// Morton code of each column over the bounding box (30 bits), value = column index; every
// workgroup first reduces the nparts bounding-box parts of cx_bbox_kernel (first wave)
template <int D>
__global__ __launch_bounds__(256) void cx_codes_kernel(const float* __restrict__ y, int64_t N,
                                                       const float* __restrict__ part, int nparts,
                                                       uint32_t* keys, int32_t* vals) {
  __shared__ float box[2 * D];
  if (threadIdx.x < 64) {
    float lo[D], hi[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
      lo[d] = __builtin_huge_valf();
      hi[d] = -__builtin_huge_valf();
    }
    for (int b = threadIdx.x; b < nparts; b += 64) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        lo[d] = fminf(lo[d], part[b * 2 * D + d]);
        hi[d] = fmaxf(hi[d], part[b * 2 * D + D + d]);
      }
    }
#pragma unroll
    for (int d = 0; d < D; ++d)
      for (int off = 32; off > 0; off >>= 1) {
        lo[d] = fminf(lo[d], __shfl_xor(lo[d], off, 64));
        hi[d] = fmaxf(hi[d], __shfl_xor(hi[d], off, 64));
      }
    if (threadIdx.x == 0) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        box[d] = lo[d];
        box[D + d] = hi[d];
      }
    }
  }
  __syncthreads();
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= N) return;
  constexpr uint32_t kMax = D == 3 ? 1023u : 32767u;
  uint32_t code = 0;
#pragma unroll
  for (int d = 0; d < D; ++d) {
    const float lo = box[d], ext = box[D + d] - lo;
    float t = ext > 0.f ? (y[j * D + d] - lo) / ext : 0.f;
    t = fminf(fmaxf(t, 0.f), 1.f);
    const uint32_t c = (uint32_t)(t * (float)kMax);
    code |= (D == 3 ? spread3(c) : spread2(c)) << d;
  }
  keys[j] = code;
  vals[j] = (int32_t)j;
}

// One wave per sub-tile of 64 sorted columns: the sub-tile centre (mid-range of its scaled
// coordinates), its radius, and the column records (layout above) relative to it.
// meta[t] = (raw centre (D), 1 if the sub-tile is compact (scaled radius^2 <= rho2max) else 0).
template <int D, class Op>
__global__ __launch_bounds__(256) void cx_build_kernel(Args a, int64_t N, float alpha, float rho2max,
                                                       const int32_t* __restrict__ order, float4* recs,
                                                       float4* meta) {
  const int lane = threadIdx.x & 63;
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t nsub = (N + kSub - 1) / kSub;
  if (t >= nsub) return;  // whole wave leaves together
  const int64_t j = t * kSub + lane;
  const bool valid = j < N;
  const int64_t o = valid ? order[j] : 0;
  float y[D], lo[D], hi[D];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    y[d] = a.c0[o * D + d];
    lo[d] = valid ? y[d] : __builtin_huge_valf();
    hi[d] = valid ? y[d] : -__builtin_huge_valf();
  }
#pragma unroll
  for (int d = 0; d < D; ++d)
    for (int off = 32; off > 0; off >>= 1) {
      lo[d] = fminf(lo[d], __shfl_xor(lo[d], off, 64));
      hi[d] = fmaxf(hi[d], __shfl_xor(hi[d], off, 64));
    }
  float c[D], Yc[D], r2 = 0.f;
#pragma unroll
  for (int d = 0; d < D; ++d) {
    c[d] = 0.5f * (lo[d] + hi[d]);          // raw centre of the sub-tile
    Yc[d] = alpha * (y[d] - c[d]);          // scaled, relative to it
    r2 = fmaf(Yc[d], Yc[d], r2);
  }
  float rmax = valid ? r2 : 0.f;
  for (int off = 32; off > 0; off >>= 1) rmax = fmaxf(rmax, __shfl_xor(rmax, off, 64));
  if (valid) {
    float rec[Op::RW4 * 4];
#pragma unroll
    for (int k = 0; k < Op::RW4 * 4; ++k) rec[k] = 0.f;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      rec[cx_y(d)] = 2.f * Yc[d];
      rec[Op::kRaw + d] = y[d];
    }
    rec[kCxC] = rec[kCxC + 1] = -r2 - kCxShift;
    Op::build(a, o, Yc, rec);
#pragma unroll
    for (int k = 0; k < Op::RW4; ++k)
      recs[j * Op::RW4 + k] = make_float4(rec[4 * k], rec[4 * k + 1], rec[4 * k + 2], rec[4 * k + 3]);
  }
  if (lane == 0) {
    float m[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int d = 0; d < D; ++d) m[d] = c[d];
    m[3] = rmax <= rho2max ? 1.f : 0.f;
    meta[t] = make_float4(m[0], m[1], m[2], m[3]);
  }
}

// ---- main pass ----------------------------------------------------------------------------
template <class Op, int D, int R>
__global__ __launch_bounds__(kBlock) void cx_kernel(const float* __restrict__ x, int64_t M, float alpha,
                                                    const float4* __restrict__ recs,
                                                    const float4* __restrict__ meta, int64_t N, int64_t chunk,
                                                    Scal sc, Outs outs) {
  constexpr int RW4 = Op::RW4;
  constexpr int NSUB = kTile / kSub;
  __shared__ float4 lds[2][kTile * RW4];
  __shared__ float4 lmeta[2][NSUB];
  const int tid = threadIdx.x;
  const int64_t ibase = (int64_t)blockIdx.x * (kBlock * R) + tid;
  float xs[R][D];  // raw coordinates of the thread's rows
#pragma unroll
  for (int r = 0; r < R; ++r) {
    int64_t i = ibase + (int64_t)r * kBlock;
    if (i >= M) i = M - 1;
#pragma unroll
    for (int d = 0; d < D; ++d) xs[r][d] = x[i * D + d];
  }
  float tot[R][Op::NTOT];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int k = 0; k < Op::NTOT; ++k) tot[r][k] = 0.f;

  const int64_t j0 = (int64_t)blockIdx.y * chunk;  // chunk: a multiple of kTile
  int64_t j1 = j0 + chunk;
  if (j1 > N) j1 = N;
  int cnt = (int)((j1 - j0) < kTile ? (j1 - j0) : kTile);
  if (cnt > 0) {
    if (tid < cnt) {
#pragma unroll
      for (int k = 0; k < RW4; ++k) lds[0][tid * RW4 + k] = recs[(j0 + tid) * RW4 + k];
    }
    if (tid < NSUB && tid * kSub < cnt) lmeta[0][tid] = meta[j0 / kSub + tid];
  }
  __syncthreads();
  int buf = 0;
  for (int64_t jt = j0; jt < j1; jt += kTile) {
    const int64_t jn = jt + kTile;
    const int cntn = jn < j1 ? (int)((j1 - jn) < kTile ? (j1 - jn) : kTile) : 0;
    if (tid < cntn) {
#pragma unroll
      for (int k = 0; k < RW4; ++k) lds[buf ^ 1][tid * RW4 + k] = recs[(jn + tid) * RW4 + k];
    }
    if (tid < NSUB && tid * kSub < cntn) lmeta[buf ^ 1][tid] = meta[jn / kSub + tid];
#pragma unroll 1
    for (int sb = 0; sb < NSUB; ++sb) {
      const int b0 = sb * kSub;
      if (b0 >= cnt) break;
      const int n = (cnt - b0) < kSub ? (cnt - b0) : kSub;
      const float4 m = lmeta[buf][sb];
      const float cm[3] = {m.x, m.y, m.z};
      const bool compact = m.w != 0.f;
      float X[R][D], F[R], Es[R], acc[R][Op::NACC];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        float a2 = 0.f;
#pragma unroll
        for (int d = 0; d < D; ++d) {
          X[r][d] = alpha * (xs[r][d] - cm[d]);
          a2 = fmaf(X[r][d], X[r][d], a2);
        }
        Es[r] = kCxShift - a2;                 // row factor F = exp2(m - |X|^2)
        F[r] = fast_exp2(Es[r]);
        if (a2 > kCxClamp * kCxClamp) {        // F = 0: keep the pair exponents finite
          const float f = kCxClamp * __builtin_amdgcn_rsqf(a2);
#pragma unroll
          for (int d = 0; d < D; ++d) X[r][d] *= f;
        }
#pragma unroll
        for (int k = 0; k < Op::NACC; ++k) acc[r][k] = 0.f;
      }
      const float4* tile = lds[buf] + b0 * RW4;
      if (compact && kCxPk && R % 2 == 0) {  // compact, rows packed in pairs (v_pk_fma_f32)
        constexpr int H = R / 2;
        f2 Xp[H][D], ap[H][Op::NACC];
#pragma unroll
        for (int h = 0; h < H; ++h) {
#pragma unroll
          for (int d = 0; d < D; ++d) Xp[h][d] = f2{X[2 * h][d], X[2 * h + 1][d]};
#pragma unroll
          for (int k = 0; k < Op::NACC; ++k) ap[h][k] = splat(0.f);
        }
        constexpr int CW = (Op::kRaw + 3) / 4;  // float4s of the record the compact terms read
#pragma unroll 2
        for (int t = 0; t < n; ++t) {
          float rec[RW4 * 4];
#pragma unroll
          for (int k = 0; k < CW; ++k) {
            const float4 q = tile[t * RW4 + k];
            rec[4 * k] = q.x; rec[4 * k + 1] = q.y; rec[4 * k + 2] = q.z; rec[4 * k + 3] = q.w;
          }
#pragma unroll
          for (int h = 0; h < H; ++h) {
            f2 e = f2{rec[kCxC], rec[kCxC + 1]};
#pragma unroll
            for (int d = 0; d < D; ++d) e = pk_fma(Xp[h][d], splat(rec[cx_y(d)]), e);
            Op::pair(f2{fast_exp2(e.x), fast_exp2(e.y)}, e, rec, ap[h]);
          }
        }
#pragma unroll
        for (int h = 0; h < H; ++h)
#pragma unroll
          for (int k = 0; k < Op::NACC; ++k) {
            acc[2 * h][k] = ap[h][k].x;
            acc[2 * h + 1][k] = ap[h][k].y;
          }
      } else if (compact) {  // compact sub-tile: expanded exponent, D fma
#pragma unroll 2
        for (int t = 0; t < n; ++t) {
          float rec[RW4 * 4];
#pragma unroll
          for (int k = 0; k < RW4; ++k) {
            const float4 q = tile[t * RW4 + k];
            rec[4 * k] = q.x; rec[4 * k + 1] = q.y; rec[4 * k + 2] = q.z; rec[4 * k + 3] = q.w;
          }
#pragma unroll
          for (int r = 0; r < R; ++r) {
            float e = rec[kCxC];
#pragma unroll
            for (int d = 0; d < D; ++d) e = fmaf(X[r][d], rec[cx_y(d)], e);
            Op::pair(fast_exp2(e), e, rec, acc[r]);
          }
        }
      } else {  // wide sub-tile: difference form on the raw coordinates (the generic arithmetic)
#pragma unroll 2
        for (int t = 0; t < n; ++t) {
          float rec[RW4 * 4];
#pragma unroll
          for (int k = 0; k < RW4; ++k) {
            const float4 q = tile[t * RW4 + k];
            rec[4 * k] = q.x; rec[4 * k + 1] = q.y; rec[4 * k + 2] = q.z; rec[4 * k + 3] = q.w;
          }
#pragma unroll
          for (int r = 0; r < R; ++r) {
            float z[D], e = 0.f;
#pragma unroll
            for (int d = 0; d < D; ++d) {
              z[d] = alpha * (xs[r][d] - rec[Op::kRaw + d]);
              e = fmaf(-z[d], z[d], e);
            }
            Op::pair_z(fast_exp2(e), e, z, rec, acc[r]);
          }
        }
      }
#pragma unroll
      for (int r = 0; r < R; ++r) Op::fold(X[r], acc[r], tot[r], compact, F[r], Es[r]);
    }
    __syncthreads();
    buf ^= 1;
    cnt = cntn;
  }

  const bool split = gridDim.y > 1;
  const float sa = sc.aux1;  // s / alpha
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t i = ibase + (int64_t)r * kBlock;
    if (i >= M) continue;
    float vals[Op::kOutW[0] + Op::kOutW[1] + Op::kOutW[2] + Op::kOutW[3]];
    Op::store(sc, sa, tot[r], vals);
    int off = 0;
#pragma unroll
    for (int k = 0; k < Op::kNOut; ++k) {
      const int w = Op::kOutW[k];
      float* base = outs.ptr[k];
      if (base != nullptr) {
        if (split) {
          float* dst = base + (int64_t)blockIdx.y * M * w + i * w;
#pragma unroll
          for (int e = 0; e < w; ++e) dst[e] = vals[off + e];
        } else {
#pragma unroll
          for (int e = 0; e < w; ++e) base[i * w + e] = epilogue(outs, k, i * w + e, vals[off + e]);
        }
      }
      off += w;
    }
  }
}

}  // namespace dicp
