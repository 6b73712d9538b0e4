// Pair operators of the Gaussian-kernel reductions and of the fused LDDMM ODE, plugged
// into dicp::rowred_kernel (common.hpp).  Each struct states the reference formula it
// computes (diffICP/tools/kernel.py, diffICP/core/LDDMM.py) and its per-pair algorithmic
// cost (FMA = 2 flop, exp2 = 1 transcendental) used by the roofline accounting.
//
// Row i carries x_i (and row weights), column j carries y_j (and column weights);
// z = x_i - y_j, r2 = |z|^2, K = exp2(nc r2) = exp(-r2/(2 sigma^2)), s = 1/sigma^2.
#pragma once
#include "common.hpp"

namespace dicp {

template <int D>
__device__ __forceinline__ float diff_sq(const float* __restrict__ x, const float* __restrict__ y,
                                         float* __restrict__ z) {
  float r2 = 0.f;
#pragma unroll
  for (int d = 0; d < D; ++d) {
    z[d] = x[d] - y[d];
    r2 = fmaf(z[d], z[d], r2);
  }
  return r2;
}

template <int D>
__device__ __forceinline__ float dot(const float* __restrict__ a, const float* __restrict__ b) {
  float r = 0.f;
#pragma unroll
  for (int d = 0; d < D; ++d) r = fmaf(a[d], b[d], r);
  return r;
}

template <int W>
__device__ __forceinline__ void ld(const float* __restrict__ p, int64_t i, float* dst) {
#pragma unroll
  for (int d = 0; d < W; ++d) dst[d] = p[i * W + d];
}

constexpr int cw4(int floats) { return (floats + 3) / 4; }

// -------------------------------------------------------------------------------------
// The ten GenKernel reductions (kernel.py:127-168 KeOps, :177-215/:259-292 torch).
// -------------------------------------------------------------------------------------

// KBase: X_i = sum_j K(x_i - y_j)                         kernel.py:131 / :178-179
template <int D>
struct OpKBase {
  static constexpr int CW4 = cw4(D), NACC = 1, kNOut = 1;
  static constexpr int kOutW[4] = {1, 0, 0, 0};
  static constexpr bool kMin = false;
  struct Row { float x[D]; };
  __device__ static void load_row(const Args& a, int64_t i, Row& r) { ld<D>(a.r0, i, r.x); }
  __device__ static void load_col(const Args& a, int64_t j, float* rec) { ld<D>(a.c0, j, rec); }
  __device__ static void pair(const Scal& sc, const Row& r, const float* rec, float* acc) {
    float z[D];
    const float r2 = diff_sq<D>(r.x, rec, z);
    acc[0] += fast_exp2(sc.nc * r2);
  }
  __device__ static void store(const Scal&, const Row&, const float* t, float* v) { v[0] = t[0]; }
};

// KRedScal: X_i = sum_j K d_j                              kernel.py:135 / :182-183
template <int D>
struct OpKRedScal {
  static constexpr int CW4 = cw4(D + 1), NACC = 1, kNOut = 1;
  static constexpr int kOutW[4] = {1, 0, 0, 0};
  static constexpr bool kMin = false;
  struct Row { float x[D]; };
  __device__ static void load_row(const Args& a, int64_t i, Row& r) { ld<D>(a.r0, i, r.x); }
  __device__ static void load_col(const Args& a, int64_t j, float* rec) {
    ld<D>(a.c0, j, rec);
    rec[D] = a.c1[j];
  }
  __device__ static void pair(const Scal& sc, const Row& r, const float* rec, float* acc) {
    float z[D];
    const float r2 = diff_sq<D>(r.x, rec, z);
    acc[0] = fmaf(fast_exp2(sc.nc * r2), rec[D], acc[0]);
  }
  __device__ static void store(const Scal&, const Row&, const float* t, float* v) { v[0] = t[0]; }
};

// KRed: X_i = sum_j K b_j  (the velocity field v, LDDMM.py:114/116)   kernel.py:138 / :186-187
// 3D cost: 3 sub + 3 fma (r2) + 1 mul + 1 exp + 3 fma = 15 flop + 1 T
template <int D>
struct OpKRed {
  static constexpr int CW4 = cw4(2 * D), NACC = D, kNOut = 1;
  static constexpr int kOutW[4] = {D, 0, 0, 0};
  static constexpr bool kMin = false;
  struct Row { float x[D]; };
  __device__ static void load_row(const Args& a, int64_t i, Row& r) { ld<D>(a.r0, i, r.x); }
  __device__ static void load_col(const Args& a, int64_t j, float* rec) {
    ld<D>(a.c0, j, rec);
    ld<D>(a.c1, j, rec + D);
  }
  __device__ static void pair(const Scal& sc, const Row& r, const float* rec, float* acc) {
    float z[D];
    const float K = fast_exp2(sc.nc * diff_sq<D>(r.x, rec, z));
#pragma unroll
    for (int d = 0; d < D; ++d) acc[d] = fmaf(K, rec[D + d], acc[d]);
  }
  __device__ static void store(const Scal&, const Row&, const float* t, float* v) {
#pragma unroll
    for (int d = 0; d < D; ++d) v[d] = t[d];
  }
};

// GradKRed: X_i = sum_j (grad K)(x_i - y_j) = -s sum_j z K    kernel.py:142 / :190-191, :262-263
template <int D>
struct OpGradK {
  static constexpr int CW4 = cw4(D), NACC = D, kNOut = 1;
  static constexpr int kOutW[4] = {D, 0, 0, 0};
  static constexpr bool kMin = false;
  struct Row { float x[D]; };
  __device__ static void load_row(const Args& a, int64_t i, Row& r) { ld<D>(a.r0, i, r.x); }
  __device__ static void load_col(const Args& a, int64_t j, float* rec) { ld<D>(a.c0, j, rec); }
  __device__ static void pair(const Scal& sc, const Row& r, const float* rec, float* acc) {
    float z[D];
    const float K = fast_exp2(sc.nc * diff_sq<D>(r.x, rec, z));
#pragma unroll
    for (int d = 0; d < D; ++d) acc[d] = fmaf(K, z[d], acc[d]);
  }
  __device__ static void store(const Scal& sc, const Row&, const float* t, float* v) {
#pragma unroll
    for (int d = 0; d < D; ++d) v[d] = -sc.s * t[d];
  }
};

// GradKScal: X_i = sum_j -s z K d_j  (gradient of KBase / KRedScal w.r.t. x)
template <int D>
struct OpGradKScal {
  static constexpr int CW4 = cw4(D + 1), NACC = D, kNOut = 1;
  static constexpr int kOutW[4] = {D, 0, 0, 0};
  static constexpr bool kMin = false;
  struct Row { float x[D]; };
  __device__ static void load_row(const Args& a, int64_t i, Row& r) { ld<D>(a.r0, i, r.x); }
  __device__ static void load_col(const Args& a, int64_t j, float* rec) {
    ld<D>(a.c0, j, rec);
    rec[D] = a.c1[j];
  }
  __device__ static void pair(const Scal& sc, const Row& r, const float* rec, float* acc) {
    float z[D];
    const float Kd = fast_exp2(sc.nc * diff_sq<D>(r.x, rec, z)) * rec[D];
#pragma unroll
    for (int d = 0; d < D; ++d) acc[d] = fmaf(Kd, z[d], acc[d]);
  }
  __device__ static void store(const Scal& sc, const Row&, const float* t, float* v) {
#pragma unroll
    for (int d = 0; d < D; ++d) v[d] = -sc.s * t[d];
  }
};

// GradKRed_rev (column reduction, kernel.py:147 / :194-195) evaluated as a row reduction
// over the former columns: Y_j = sum_i gradK(x_i - y_j).d_i = sum_i s ((y_j - x_i).d_i) K.
// Called with rows = y, cols = (x, d):  X_i = s sum_j (z . b_j) K.
template <int D>
struct OpZDotB {
  static constexpr int CW4 = cw4(2 * D), NACC = 1, kNOut = 1;
  static constexpr int kOutW[4] = {1, 0, 0, 0};
  static constexpr bool kMin = false;
  struct Row { float x[D]; };
  __device__ static void load_row(const Args& a, int64_t i, Row& r) { ld<D>(a.r0, i, r.x); }
  __device__ static void load_col(const Args& a, int64_t j, float* rec) {
    ld<D>(a.c0, j, rec);
    ld<D>(a.c1, j, rec + D);
  }
  __device__ static void pair(const Scal& sc, const Row& r, const float* rec, float* acc) {
    float z[D];
    const float K = fast_exp2(sc.nc * diff_sq<D>(r.x, rec, z));
    acc[0] = fmaf(K, dot<D>(z, rec + D), acc[0]);
  }
  __device__ static void store(const Scal& sc, const Row&, const float* t, float* v) {
    v[0] = sc.s * t[0];
  }
};

// DDKRed: X_i^d = sum_j -s z^d K b_j^d                  kernel.py:151 / :198-199
template <int D>
struct OpDDK {
  static constexpr int CW4 = cw4(2 * D), NACC = D, kNOut = 1;
  static constexpr int kOutW[4] = {D, 0, 0, 0};
  static constexpr bool kMin = false;
  struct Row { float x[D]; };
  __device__ static void load_row(const Args& a, int64_t i, Row& r) { ld<D>(a.r0, i, r.x); }
  __device__ static void load_col(const Args& a, int64_t j, float* rec) {
    ld<D>(a.c0, j, rec);
    ld<D>(a.c1, j, rec + D);
  }
  __device__ static void pair(const Scal& sc, const Row& r, const float* rec, float* acc) {
    float z[D];
    const float K = fast_exp2(sc.nc * diff_sq<D>(r.x, rec, z));
#pragma unroll
    for (int d = 0; d < D; ++d) acc[d] = fmaf(K * z[d], rec[D + d], acc[d]);
  }
  __device__ static void store(const Scal& sc, const Row&, const float* t, float* v) {
#pragma unroll
    for (int d = 0; d < D; ++d) v[d] = -sc.s * t[d];
  }
};

// GenDKRed: X_i = sum_j -s z K (c_i . b_j)   (momentum update Gq, LDDMM.py:199)
// kernel.py:155 / :202-203.  3D cost ~21 flop + 1 T.
template <int D>
struct OpGenDK {
  static constexpr int CW4 = cw4(2 * D), NACC = D, kNOut = 1;
  static constexpr int kOutW[4] = {D, 0, 0, 0};
  static constexpr bool kMin = false;
  struct Row { float x[D]; float c[D]; };
  __device__ static void load_row(const Args& a, int64_t i, Row& r) {
    ld<D>(a.r0, i, r.x);
    ld<D>(a.r1, i, r.c);
  }
  __device__ static void load_col(const Args& a, int64_t j, float* rec) {
    ld<D>(a.c0, j, rec);
    ld<D>(a.c1, j, rec + D);
  }
  __device__ static void pair(const Scal& sc, const Row& r, const float* rec, float* acc) {
    float z[D];
    const float K = fast_exp2(sc.nc * diff_sq<D>(r.x, rec, z));
    const float w = K * dot<D>(r.c, rec + D);
#pragma unroll
    for (int d = 0; d < D; ++d) acc[d] = fmaf(w, z[d], acc[d]);
  }
  __device__ static void store(const Scal& sc, const Row&, const float* t, float* v) {
#pragma unroll
    for (int d = 0; d < D; ++d) v[d] = -sc.s * t[d];
  }
};

// HessKRed: X_i = sum_j [s^2 (z.u) z - s u] K,  u = c_i - b_j     kernel.py:160 / :284-286
template <int D>
struct OpHessK {
  static constexpr int CW4 = cw4(2 * D), NACC = D, kNOut = 1;
  static constexpr int kOutW[4] = {D, 0, 0, 0};
  static constexpr bool kMin = false;
  struct Row { float x[D]; float c[D]; };
  __device__ static void load_row(const Args& a, int64_t i, Row& r) {
    ld<D>(a.r0, i, r.x);
    ld<D>(a.r1, i, r.c);
  }
  __device__ static void load_col(const Args& a, int64_t j, float* rec) {
    ld<D>(a.c0, j, rec);
    ld<D>(a.c1, j, rec + D);
  }
  __device__ static void pair(const Scal& sc, const Row& r, const float* rec, float* acc) {
    float z[D], u[D];
    const float K = fast_exp2(sc.nc * diff_sq<D>(r.x, rec, z));
#pragma unroll
    for (int d = 0; d < D; ++d) u[d] = r.c[d] - rec[D + d];
    const float zu = sc.s * dot<D>(z, u);
#pragma unroll
    for (int d = 0; d < D; ++d) acc[d] = fmaf(K, fmaf(zu, z[d], -u[d]), acc[d]);
  }
  __device__ static void store(const Scal& sc, const Row&, const float* t, float* v) {
#pragma unroll
    for (int d = 0; d < D; ++d) v[d] = sc.s * t[d];
  }
};

// LapKRed: X_i = sum_j (s^2 r2 - D s) K                 kernel.py:164 / :206-207, :265-267
template <int D>
struct OpLapK {
  static constexpr int CW4 = cw4(D), NACC = 1, kNOut = 1;
  static constexpr int kOutW[4] = {1, 0, 0, 0};
  static constexpr bool kMin = false;
  struct Row { float x[D]; };
  __device__ static void load_row(const Args& a, int64_t i, Row& r) { ld<D>(a.r0, i, r.x); }
  __device__ static void load_col(const Args& a, int64_t j, float* rec) { ld<D>(a.c0, j, rec); }
  __device__ static void pair(const Scal& sc, const Row& r, const float* rec, float* acc) {
    float z[D];
    const float r2 = diff_sq<D>(r.x, rec, z);
    const float K = fast_exp2(sc.nc * r2);
    acc[0] = fmaf(K, fmaf(sc.s, r2, -(float)D), acc[0]);
  }
  __device__ static void store(const Scal& sc, const Row&, const float* t, float* v) {
    v[0] = sc.s * t[0];
  }
};

// GradLapKRed: X_i = sum_j -z (s^3 r2 - (D+2) s^2) K     kernel.py:168 / :289-292
// (aux0 = 1: plain; GradLapKScal multiplies by a column weight d_j)
template <int D, bool SCAL>
struct OpGradLapK {
  static constexpr int CW4 = cw4(D + (SCAL ? 1 : 0)), NACC = D, kNOut = 1;
  static constexpr int kOutW[4] = {D, 0, 0, 0};
  static constexpr bool kMin = false;
  struct Row { float x[D]; };
  __device__ static void load_row(const Args& a, int64_t i, Row& r) { ld<D>(a.r0, i, r.x); }
  __device__ static void load_col(const Args& a, int64_t j, float* rec) {
    ld<D>(a.c0, j, rec);
    if (SCAL) rec[D] = a.c1[j];
  }
  __device__ static void pair(const Scal& sc, const Row& r, const float* rec, float* acc) {
    float z[D];
    const float r2 = diff_sq<D>(r.x, rec, z);
    float w = fast_exp2(sc.nc * r2) * fmaf(sc.s, r2, -(float)(D + 2));
    if (SCAL) w *= rec[D];
#pragma unroll
    for (int d = 0; d < D; ++d) acc[d] = fmaf(w, z[d], acc[d]);
  }
  __device__ static void store(const Scal& sc, const Row&, const float* t, float* v) {
    const float s2 = sc.s * sc.s;
#pragma unroll
    for (int d = 0; d < D; ++d) v[d] = -s2 * t[d];
  }
};

// Squared distance with the exact arithmetic of the reference's torch expression
// ((x_i - x_j)**2).sum(-1) on the CPU: products rounded, summed left to right, no FMA
// contraction (so comparisons against a radius give bit-identical decisions).  The empty
// asm makes each rounded product opaque: -ffp-contract=fast would otherwise fuse it into
// the following add in the backend (a source-level contract pragma does not prevent that).
template <int D>
__device__ __forceinline__ float exact_sq(const float* __restrict__ x, const float* __restrict__ y) {
  float s = 0.f;
#pragma unroll
  for (int d = 0; d < D; ++d) {
    const float z = x[d] - y[d];
    float zz = z * z;
    asm("" : "+v"(zz));
    s = (d == 0) ? zz : s + zz;
  }
  return s;
}

// out_i = min_j |x_i - y_j|^2   (check_coverage, kernel.py:324-329)
template <int D>
struct OpMinSqDist {
  static constexpr int CW4 = cw4(D), NACC = 1, kNOut = 1;
  static constexpr int kOutW[4] = {1, 0, 0, 0};
  static constexpr bool kMin = true;
  struct Row { float x[D]; };
  __device__ static void load_row(const Args& a, int64_t i, Row& r) { ld<D>(a.r0, i, r.x); }
  __device__ static void load_col(const Args& a, int64_t j, float* rec) { ld<D>(a.c0, j, rec); }
  __device__ static void pair(const Scal&, const Row& r, const float* rec, float* acc) {
    acc[0] = fminf(acc[0], exact_sq<D>(r.x, rec));
  }
  __device__ static void store(const Scal&, const Row&, const float* t, float* v) { v[0] = t[0]; }
};

// out_i = min_{j != i} |x_i - x_j|^2 over the same point set (rows = columns): the second
// smallest entry of row i of the distance matrix, D_ij.Kmin(2)[:, 1] of intrinsic_scale
// (point_sets.py:13-26).  Indices travel as raw int bits in a float slot.
template <int D>
struct OpMinSqDistOther {
  static constexpr int CW4 = cw4(D + 1), NACC = 1, kNOut = 1;
  static constexpr int kOutW[4] = {1, 0, 0, 0};
  static constexpr bool kMin = true;
  struct Row { float x[D]; int i; };
  __device__ static void load_row(const Args& a, int64_t i, Row& r) {
    ld<D>(a.r0, i, r.x);
    r.i = (int)i;
  }
  __device__ static void load_col(const Args& a, int64_t j, float* rec) {
    ld<D>(a.c0, j, rec);
    rec[D] = __int_as_float((int)j);
  }
  __device__ static void pair(const Scal&, const Row& r, const float* rec, float* acc) {
    const float d2 = exact_sq<D>(r.x, rec);
    acc[0] = (__float_as_int(rec[D]) != r.i) ? fminf(acc[0], d2) : acc[0];
  }
  __device__ static void store(const Scal&, const Row&, const float* t, float* v) { v[0] = t[0]; }
};

// out_i = #{j : |x_i - y_j|^2 <= R2}  (float-valued, exact below 2^24)   decimate,
// point_sets.py:114-116 (D <= R**2 with the torch arithmetic of exact_sq); R2 in sc.aux0.
template <int D>
struct OpRadiusCount {
  static constexpr int CW4 = cw4(D), NACC = 1, kNOut = 1;
  static constexpr int kOutW[4] = {1, 0, 0, 0};
  static constexpr bool kMin = false;
  struct Row { float x[D]; };
  __device__ static void load_row(const Args& a, int64_t i, Row& r) { ld<D>(a.r0, i, r.x); }
  __device__ static void load_col(const Args& a, int64_t j, float* rec) { ld<D>(a.c0, j, rec); }
  __device__ static void pair(const Scal& sc, const Row& r, const float* rec, float* acc) {
    acc[0] += (exact_sq<D>(r.x, rec) <= sc.aux0) ? 1.f : 0.f;
  }
  __device__ static void store(const Scal&, const Row&, const float* t, float* v) { v[0] = t[0]; }
};

// -------------------------------------------------------------------------------------
// Fused LDDMM ODE right-hand side on the support points (LDDMMModel.ODE, LDDMM.py:176-227).
// Rows and columns are both (q, p).  One exp per pair feeds every term.
//
// Scaled coordinates: q' = alpha q, alpha = sqrt(log2(e)/(2 sigma^2)) (Args::scale), so
// z' = alpha z and K = exp2(-|z'|^2) with no per-pair multiply; s2 = s / alpha^2 = 2 ln 2.
// ETA=false (classic / hybrid, eta = 0):
//   V = sum K p_j,  Z' = sum K z',  Gs' = sum K z' (p_i.p_j)
//   v = V ; mG = -GenDKRed = (s/alpha) Gs' ; g = p_i.GradKRed_i = -(s/alpha) p_i.Z' ;
//   h = 1/2 p_i.V
// ETA=true (logdet, eta = 1/lambda), additionally with u = p_i - p_j:
//   Hs = sum K [s2 (z'.u) z' - u]        (HessKRed = s Hs),
//   GL' = sum K z' (s2 r2' - (D+2))       (GradLapKRed = -(s^2/alpha) GL'),
//   L = sum K (s2 r2' - D)                (LapKRed = s L)
//   v  = V + eta (s/alpha) Z'                                     (LDDMM.py:114)
//   mG = (s/alpha) Gs' + eta s Hs - eta^2 (s^2/alpha) GL'         (LDDMM.py:201-203)
//   g  = -(s/alpha) p_i.Z' + eta s L                              (LDDMM.py:135)
//   h  = 1/2 p_i.V + eta (s/alpha) p_i.Z' - 1/2 eta^2 s L         (LDDMM.py:151-153)
// 3D cost (ETA=false, DIV=true): 33 flop + 1 T per pair.
// -------------------------------------------------------------------------------------
constexpr float kS2 = 1.3862943611198906f;  // s / alpha^2 = 2 ln 2

template <int D>
__device__ __forceinline__ void ld_scaled(const float* __restrict__ p, int64_t i, float a, float* dst) {
#pragma unroll
  for (int d = 0; d < D; ++d) dst[d] = a * p[i * D + d];
}

template <int D, bool ETA, bool DIV>
struct OpOdeSelfFwd {
  static constexpr int CW4 = cw4(2 * D);
  static constexpr int NACC = ETA ? (5 * D + 1) : (DIV ? 3 * D : 2 * D);
  static constexpr int kNOut = 4;
  static constexpr int kOutW[4] = {D, D, 1, 1};
  static constexpr bool kMin = false;
  struct Row { float q[D]; float p[D]; };
  __device__ static void load_row(const Args& a, int64_t i, Row& r) {
    ld_coord<D>(a, a.r0, i, r.q);
    ld<D>(a.r1, i, r.p);
  }
  __device__ static void load_col(const Args& a, int64_t j, float* rec) {
    ld_coord<D>(a, a.c0, j, rec);
    ld<D>(a.c1, j, rec + D);
  }
  __device__ static void pair(const Scal& sc, const Row& r, const float* rec, float* acc) {
    float z[D];
    const float r2 = diff_sq<D>(r.q, rec, z);
    const float K = fast_exp2(-r2);
    const float* pj = rec + D;
    const float Kpp = K * dot<D>(r.p, pj);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      acc[d] = fmaf(K, pj[d], acc[d]);           // V
      acc[D + d] = fmaf(Kpp, z[d], acc[D + d]);  // Gs'
    }
    if (ETA || DIV) {
#pragma unroll
      for (int d = 0; d < D; ++d) acc[2 * D + d] = fmaf(K, z[d], acc[2 * D + d]);  // Z'
    }
    if (ETA) {
      float u[D];
#pragma unroll
      for (int d = 0; d < D; ++d) u[d] = r.p[d] - pj[d];
      const float szu = kS2 * dot<D>(z, u);
      const float sr2 = kS2 * r2;
      const float KGL = K * (sr2 - (float)(D + 2));
#pragma unroll
      for (int d = 0; d < D; ++d) {
        acc[3 * D + d] = fmaf(K, fmaf(szu, z[d], -u[d]), acc[3 * D + d]);  // Hs
        acc[4 * D + d] = fmaf(KGL, z[d], acc[4 * D + d]);                   // GL'
      }
      acc[5 * D] = fmaf(K, sr2 - (float)D, acc[5 * D]);  // L
    }
  }
  __device__ static void store(const Scal& sc, const Row& r, const float* t, float* v) {
    const float s = sc.s, eta = sc.eta, sa = sc.aux1;  // aux1 = s / alpha
    const float* V = t;
    const float* Gs = t + D;
    const float* Z = t + 2 * D;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      if (ETA) {
        v[d] = fmaf(eta * sa, Z[d], V[d]);
        v[D + d] = sa * Gs[d] + eta * s * t[3 * D + d] - eta * eta * s * sa * t[4 * D + d];
      } else {
        v[d] = V[d];
        v[D + d] = sa * Gs[d];
      }
    }
    const float pV = dot<D>(r.p, V);
    if (ETA) {
      const float pZ = dot<D>(r.p, Z);
      const float L = t[5 * D];
      v[2 * D] = -sa * pZ + eta * s * L;
      v[2 * D + 1] = 0.5f * pV + eta * sa * pZ - 0.5f * eta * eta * s * L;
    } else {
      v[2 * D] = DIV ? -sa * dot<D>(r.p, Z) : 0.f;
      v[2 * D + 1] = 0.5f * pV;
    }
  }
};

// OpOdeSelfFwd<D, false, true> whose fourth output is the row's divergence vector in original
// units, zs_i = sum_j K_ij (q_i - q_j) = Z'_i / alpha (= -sigma^2 GradKRed(q,q)_i), instead of
// the Hamiltonian row h_i: the per-row sum through which the cotangent of sum_i g_i enters
// dL/dp of the VJP (gp_i gets -gdiv s zs_i), so the VJP need not re-sum it pair by pair.
template <int D>
struct OpOdeSelfFwdZs : OpOdeSelfFwd<D, false, true> {
  using P = OpOdeSelfFwd<D, false, true>;
  static constexpr int kOutW[4] = {D, D, 1, D};
  __device__ static void store(const Scal& sc, const typename P::Row& r, const float* t, float* v) {
    P::store(sc, r, t, v);
    const float ia = sc.aux1 / sc.s;  // 1 / alpha
#pragma unroll
    for (int d = 0; d < D; ++d) v[2 * D + 1 + d] = ia * t[2 * D + d];
  }
};

// -------------------------------------------------------------------------------------
// VJP of OpOdeSelfFwd (eta = 0): cotangents a = dL/dv, bm = dL/dmG, gam = dL/d(sum g).
// Row m, column j, z = q_m - q_j (derivation in DESIGN.md; checked against torch autograd
// of the oracle in tests/test_gpu_kernels.py::test_ode_self_bwd):
//   gp_m = sum_j K [ a_j + s ((bm_m - bm_j).z) p_j - s gam z ]
//   gq_m = s sum_j K [ (p_m.p_j)(bm_m - bm_j) - gam (p_m - p_j)
//                      + z ( s (gam (p_m-p_j).z - (p_m.p_j)(bm_m-bm_j).z) - (a_m.p_j + a_j.p_m) ) ]
// In scaled coordinates (z' = alpha z, s1 = s/alpha, s2 = s/alpha^2, ia = 1/alpha):
//   gp_m = sum_j K [ a_j + s1 (db.z') p_j - s1 gam z' ]
//   gq_m = s sum_j K [ pp db - gam dp + z' (s2 (gam dp.z' - pp db.z') - ia ap) ]
// 3D cost: 89 flop + 1 T per pair.
// -------------------------------------------------------------------------------------
template <int D>
struct OpOdeSelfBwd {
  static constexpr int64_t kRoundRows = 5000, kMaxRounds = 24;  // launch.hpp rounds_for
  static constexpr int CW4 = cw4(4 * D);
  static constexpr int NACC = 2 * D;
  static constexpr int kNOut = 2;
  static constexpr int kOutW[4] = {D, D, 0, 0};
  static constexpr bool kMin = false;
  // ap is evaluated with the row's a, p pre-multiplied by 1/alpha (ia_a, ia_p)
  struct Row { float q[D]; float p[D]; float b[D]; float ia_a[D]; float ia_p[D]; };
  __device__ static void load_row(const Args& a, int64_t i, Row& r) {
    ld_coord<D>(a, a.r0, i, r.q);
    ld<D>(a.r1, i, r.p);
    ld<D>(a.r3, i, r.b);
    const float ia = 1.0f / a.scale;
    ld_scaled<D>(a.r2, i, ia, r.ia_a);
#pragma unroll
    for (int d = 0; d < D; ++d) r.ia_p[d] = ia * r.p[d];
  }
  __device__ static void load_col(const Args& a, int64_t j, float* rec) {
    ld_coord<D>(a, a.c0, j, rec);
    ld<D>(a.c1, j, rec + D);
    ld<D>(a.c2, j, rec + 2 * D);
    ld<D>(a.c3, j, rec + 3 * D);
  }
  __device__ static void pair(const Scal& sc, const Row& r, const float* rec, float* acc) {
    const float s1 = sc.aux1, gam = sc.aux0;
    float z[D], db[D], dp[D];
    const float K = fast_exp2(-diff_sq<D>(r.q, rec, z));
    const float* pj = rec + D;
    const float* aj = rec + 2 * D;
    const float* bj = rec + 3 * D;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      db[d] = r.b[d] - bj[d];
      dp[d] = r.p[d] - pj[d];
    }
    const float pp = dot<D>(r.p, pj);
    const float iap = dot<D>(r.ia_a, pj) + dot<D>(aj, r.ia_p);
    const float zb = dot<D>(z, db);
    const float zp = dot<D>(z, dp);
    const float Ks1 = K * s1;
    const float t1 = Ks1 * zb;
    const float t2 = Ks1 * gam;
    const float w = fmaf(kS2, fmaf(-pp, zb, gam * zp), -iap);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      acc[d] = fmaf(K, aj[d], fmaf(t1, pj[d], fmaf(-t2, z[d], acc[d])));            // gp
      const float e = fmaf(pp, db[d], fmaf(-gam, dp[d], w * z[d]));
      acc[D + d] = fmaf(K, e, acc[D + d]);                                           // gq / s
    }
  }
  __device__ static void store(const Scal& sc, const Row&, const float* t, float* v) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      v[d] = sc.s * t[D + d];  // gq
      v[D + d] = t[d];         // gp
    }
  }
};

// Same VJP as OpOdeSelfBwd with the per-pair algebra regrouped to 48 VALU ops (D = 3)
// instead of 55:
//   u   = gam (p_i - p_j) - pp (b_i - b_j)     (gam p_j staged once per column in LDS)
//   w   = kS2 z'.u - iap,   e = w z' - u       (= pp db - gam dp + w z')
//   gp  = s1 sum_j [ K (a'_j - gam z') + K zb p_j ],   a'_j = a_j / s1 (staged in LDS)
//   gq  = s  sum_j K e
template <int D>
struct OpOdeSelfBwd2 {
  static constexpr int64_t kRoundRows = 5000, kMaxRounds = 24;  // launch.hpp rounds_for
  static constexpr int CW4 = cw4(5 * D);
  static constexpr int NACC = 2 * D;
  static constexpr int kNOut = 2;
  static constexpr int kOutW[4] = {D, D, 0, 0};
  static constexpr bool kMin = false;
  struct Row { float q[D]; float p[D]; float b[D]; float ia_a[D]; float sia_p[D]; float gp[D]; float ngam; };
  __device__ static void load_row_s(const Args& a, const Scal& sc, int64_t i, Row& r) {
    ld_coord<D>(a, a.r0, i, r.q);
    ld<D>(a.r1, i, r.p);
    ld<D>(a.r3, i, r.b);
    const float ia = 1.0f / a.scale;
    ld_scaled<D>(a.r2, i, ia, r.ia_a);
    const float sia = sc.aux1 * ia, gam = sc.aux0;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      r.sia_p[d] = sia * r.p[d];
      r.gp[d] = gam * r.p[d];
    }
    r.ngam = -gam;
  }
  __device__ static void load_col_s(const Args& a, const Scal& sc, int64_t j, float* rec) {
    ld_coord<D>(a, a.c0, j, rec);
    ld<D>(a.c1, j, rec + D);
    ld_scaled<D>(a.c2, j, 1.0f / sc.aux1, rec + 2 * D);
    ld<D>(a.c3, j, rec + 3 * D);
    const float gam = sc.aux0;
#pragma unroll
    for (int d = 0; d < D; ++d) rec[4 * D + d] = gam * rec[D + d];
#pragma unroll
    for (int k = 5 * D; k < 4 * CW4; ++k) rec[k] = 0.f;
  }
  __device__ static void pair(const Scal&, const Row& r, const float* rec, float* acc) {
    float z[D], db[D], u[D];
    const float K = fast_exp2(-diff_sq<D>(r.q, rec, z));
    const float* pj = rec + D;
    const float* aj = rec + 2 * D;
    const float* bj = rec + 3 * D;
    const float* gpj = rec + 4 * D;
    const float pp = dot<D>(r.p, pj);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      db[d] = r.b[d] - bj[d];
      u[d] = fmaf(-pp, db[d], r.gp[d] - gpj[d]);
    }
    const float zu = dot<D>(z, u);
    const float zb = dot<D>(z, db);
    const float iap = dot<D>(r.ia_a, pj) + dot<D>(aj, r.sia_p);
    const float w = fmaf(kS2, zu, -iap);
    const float Kzb = K * zb;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      acc[d] = fmaf(Kzb, pj[d], fmaf(K, fmaf(r.ngam, z[d], aj[d]), acc[d]));  // gp / s1
      acc[D + d] = fmaf(K, fmaf(w, z[d], -u[d]), acc[D + d]);                   // gq / s
    }
  }
  __device__ static void store(const Scal& sc, const Row&, const float* t, float* v) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      v[d] = sc.s * t[D + d];    // gq
      v[D + d] = sc.aux1 * t[d];  // gp
    }
  }
};

// -------------------------------------------------------------------------------------
// External points x carried by the flow (LDDMM.py:219-227): rows x_i, columns (q_j, p_j).
//   vx = sum K p_j + eta s sum K z                           (v(x,q,p), LDDMM.py:114)
//   gx = s sum K (z.p_j) + eta s sum K (s r2 - D)            (row form of mdivsum(x,q,p),
//        LDDMM.py:135: sum_j p_j.sum_k gradK(q_j - x_k) = sum_k sum_j s ((x_k-q_j).p_j) K)
// -------------------------------------------------------------------------------------
template <int D, bool ETA, bool DIV>
struct OpOdeExtFwd {
  static constexpr int CW4 = cw4(2 * D);
  static constexpr int NACC = D + (DIV ? 1 : 0) + (ETA ? D + 1 : 0);
  static constexpr int kNOut = 2;
  static constexpr int kOutW[4] = {D, 1, 0, 0};
  static constexpr bool kMin = false;
  struct Row { float x[D]; };
  __device__ static void load_row(const Args& a, int64_t i, Row& r) { ld<D>(a.r0, i, r.x); }
  __device__ static void load_col(const Args& a, int64_t j, float* rec) {
    ld<D>(a.c0, j, rec);
    ld<D>(a.c1, j, rec + D);
  }
  __device__ static void pair(const Scal& sc, const Row& r, const float* rec, float* acc) {
    float z[D];
    const float r2 = diff_sq<D>(r.x, rec, z);
    const float K = fast_exp2(sc.nc * r2);
    const float* pj = rec + D;
#pragma unroll
    for (int d = 0; d < D; ++d) acc[d] = fmaf(K, pj[d], acc[d]);
    if (DIV) acc[D] = fmaf(K, dot<D>(z, pj), acc[D]);
    if (ETA) {
      constexpr int o = D + (DIV ? 1 : 0);
#pragma unroll
      for (int d = 0; d < D; ++d) acc[o + d] = fmaf(K, z[d], acc[o + d]);
      acc[o + D] = fmaf(K, fmaf(sc.s, r2, -(float)D), acc[o + D]);
    }
  }
  __device__ static void store(const Scal& sc, const Row&, const float* t, float* v) {
    const float s = sc.s, eta = sc.eta;
    constexpr int o = D + (DIV ? 1 : 0);
#pragma unroll
    for (int d = 0; d < D; ++d) v[d] = ETA ? fmaf(eta * s, t[o + d], t[d]) : t[d];
    float g = DIV ? s * t[D] : 0.f;
    if (ETA && DIV) g += eta * s * t[o + D];
    v[D] = g;
  }
};

// VJP of OpOdeExtFwd w.r.t. x (eta = 0): rows x_i (+ cotangent a_i), columns (q_j, p_j).
//   gx_i = s sum_j K [ gam p_j - z ( a_i.p_j + s gam (z.p_j) ) ]
template <int D>
struct OpOdeExtBwdX {
  static constexpr int CW4 = cw4(2 * D);
  static constexpr int NACC = D;
  static constexpr int kNOut = 1;
  static constexpr int kOutW[4] = {D, 0, 0, 0};
  static constexpr bool kMin = false;
  struct Row { float x[D]; float a[D]; };
  __device__ static void load_row(const Args& a, int64_t i, Row& r) {
    ld<D>(a.r0, i, r.x);
    ld<D>(a.r1, i, r.a);
  }
  __device__ static void load_col(const Args& a, int64_t j, float* rec) {
    ld<D>(a.c0, j, rec);
    ld<D>(a.c1, j, rec + D);
  }
  __device__ static void pair(const Scal& sc, const Row& r, const float* rec, float* acc) {
    const float gam = sc.aux0;
    float z[D];
    const float K = fast_exp2(sc.nc * diff_sq<D>(r.x, rec, z));
    const float* pj = rec + D;
    const float w = dot<D>(r.a, pj) + sc.s * gam * dot<D>(z, pj);
#pragma unroll
    for (int d = 0; d < D; ++d) acc[d] = fmaf(K, fmaf(gam, pj[d], -w * z[d]), acc[d]);
  }
  __device__ static void store(const Scal& sc, const Row&, const float* t, float* v) {
#pragma unroll
    for (int d = 0; d < D; ++d) v[d] = sc.s * t[d];
  }
};

// VJP of OpOdeExtFwd w.r.t. (q, p) (eta = 0), as a row reduction over the support rows
// q_j (+ p_j) against columns (x_i, a_i); z' = q_j - x_i:
//   gp_j = sum_i K [ a_i - s gam z' ]
//   gq_j = -s sum_i K [ z' (a_i.p_j - s gam (z'.p_j)) + gam p_j ]
template <int D>
struct OpOdeExtBwdQ {
  static constexpr int CW4 = cw4(2 * D);
  static constexpr int NACC = 2 * D;
  static constexpr int kNOut = 2;
  static constexpr int kOutW[4] = {D, D, 0, 0};
  static constexpr bool kMin = false;
  struct Row { float q[D]; float p[D]; };
  __device__ static void load_row(const Args& a, int64_t i, Row& r) {
    ld<D>(a.r0, i, r.q);
    ld<D>(a.r1, i, r.p);
  }
  __device__ static void load_col(const Args& a, int64_t j, float* rec) {
    ld<D>(a.c0, j, rec);
    ld<D>(a.c1, j, rec + D);
  }
  __device__ static void pair(const Scal& sc, const Row& r, const float* rec, float* acc) {
    const float s = sc.s, gam = sc.aux0;
    float z[D];
    const float K = fast_exp2(sc.nc * diff_sq<D>(r.q, rec, z));
    const float* ai = rec + D;
    const float sg = s * gam;
    const float w = dot<D>(ai, r.p) - sg * dot<D>(z, r.p);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      acc[d] = fmaf(K, fmaf(-sg, z[d], ai[d]), acc[d]);                 // gp
      acc[D + d] = fmaf(K, fmaf(w, z[d], gam * r.p[d]), acc[D + d]);    // -gq/s
    }
  }
  __device__ static void store(const Scal& sc, const Row&, const float* t, float* v) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      v[d] = -sc.s * t[D + d];  // gq
      v[D + d] = t[d];          // gp
    }
  }
};

// -------------------------------------------------------------------------------------
// VJP of the fused self ODE with gradcomponent (eta = 1/lambda != 0, "logdet" model,
// LDDMM.py:198-203 + :133-135).  Row m, column j, z = q_m - q_j, d* = *_m - *_j:
//   gp_m = sum_j K [ a_j + s zb p_j + eta s (s zb z - db) - gam s z ]
//   gq_m = sum_j K [ eta s da + s pp db + eta s^2 (zb dp + zp db)
//                    - eta^2 s^2 ((s r2 - D - 2) db + 2 s zb z) - gam s dp + 4 gam eta s^2 z
//                    - s Phi z ]
//   Phi = ap + eta s za + s pp zb + eta s (s zp zb - db.dp) - eta^2 s^2 zb (s r2 - D - 2)
//         - gam s zp + 2 gam eta s (s r2 - D)
// with zb = db.z, zp = dp.z, za = da.z, pp = p_m.p_j, ap = a_m.p_j + a_j.p_m
// (checked against torch autograd of the oracle, tests/test_gpu_kernels.py).
// -------------------------------------------------------------------------------------
template <int D>
struct OpOdeSelfBwdEta {
  static constexpr int64_t kRoundRows = 5000, kMaxRounds = 24;  // launch.hpp rounds_for
  static constexpr int CW4 = cw4(4 * D);
  static constexpr int NACC = 2 * D;
  static constexpr int kNOut = 2;
  static constexpr int kOutW[4] = {D, D, 0, 0};
  static constexpr bool kMin = false;
  struct Row { float q[D]; float p[D]; float a[D]; float b[D]; };
  __device__ static void load_row(const Args& a, int64_t i, Row& r) {
    ld<D>(a.r0, i, r.q);
    ld<D>(a.r1, i, r.p);
    ld<D>(a.r2, i, r.a);
    ld<D>(a.r3, i, r.b);
  }
  __device__ static void load_col(const Args& a, int64_t j, float* rec) {
    ld<D>(a.c0, j, rec);
    ld<D>(a.c1, j, rec + D);
    ld<D>(a.c2, j, rec + 2 * D);
    ld<D>(a.c3, j, rec + 3 * D);
  }
  __device__ static void pair(const Scal& sc, const Row& r, const float* rec, float* acc) {
    const float s = sc.s, eta = sc.eta, gam = sc.aux0;
    float z[D], da[D], db[D], dp[D];
    const float r2 = diff_sq<D>(r.q, rec, z);
    const float K = fast_exp2(sc.nc * r2);
    const float* pj = rec + D;
    const float* aj = rec + 2 * D;
    const float* bj = rec + 3 * D;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      da[d] = r.a[d] - aj[d];
      db[d] = r.b[d] - bj[d];
      dp[d] = r.p[d] - pj[d];
    }
    const float pp = dot<D>(r.p, pj);
    const float ap = dot<D>(r.a, pj) + dot<D>(aj, r.p);
    const float zb = dot<D>(z, db), zp = dot<D>(z, dp), za = dot<D>(z, da), bp = dot<D>(db, dp);
    const float es = eta * s, es2 = es * s, e2s2 = eta * es2, gs = gam * s;
    const float sr2 = s * r2;
    const float Phi = ap + es * za + s * pp * zb + es * (s * zp * zb - bp) -
                      e2s2 * zb * (sr2 - (float)(D + 2)) - gs * zp + 2.f * gam * es * (sr2 - (float)D);
    const float cz_p = s * zb * es - gs;                      // gp: coefficient of z
    const float cz_q = -2.f * e2s2 * s * zb + 4.f * gam * es2 - s * Phi;  // gq: coefficient of z
    const float cdb = s * pp + es2 * zp - e2s2 * (sr2 - (float)(D + 2));
#pragma unroll
    for (int d = 0; d < D; ++d) {
      acc[d] = fmaf(K, aj[d] + s * zb * pj[d] - es * db[d] + cz_p * z[d], acc[d]);           // gp
      acc[D + d] = fmaf(K, es * da[d] + cdb * db[d] + es2 * zb * dp[d] - gs * dp[d] + cz_q * z[d],
                        acc[D + d]);                                                        // gq
    }
  }
  __device__ static void store(const Scal&, const Row&, const float* t, float* v) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      v[d] = t[D + d];  // gq
      v[D + d] = t[d];  // gp
    }
  }
};

// VJP of the external-point ODE terms with gradcomponent (eta != 0), rows x_i (+ a_i):
//   dF/dz = K [ eta s a_i + gam s p_j + 2 gam eta s^2 z - s Phi z ],
//   Phi = a_i.p_j + eta s (a_i.z) + gam s (z.p_j) + gam eta s (s r2 - D);   gx_i = sum_j dF/dz
template <int D>
struct OpOdeExtBwdXEta {
  static constexpr int CW4 = cw4(2 * D);
  static constexpr int NACC = D;
  static constexpr int kNOut = 1;
  static constexpr int kOutW[4] = {D, 0, 0, 0};
  static constexpr bool kMin = false;
  struct Row { float x[D]; float a[D]; };
  __device__ static void load_row(const Args& a, int64_t i, Row& r) {
    ld<D>(a.r0, i, r.x);
    ld<D>(a.r1, i, r.a);
  }
  __device__ static void load_col(const Args& a, int64_t j, float* rec) {
    ld<D>(a.c0, j, rec);
    ld<D>(a.c1, j, rec + D);
  }
  __device__ static void pair(const Scal& sc, const Row& r, const float* rec, float* acc) {
    const float s = sc.s, eta = sc.eta, gam = sc.aux0;
    float z[D];
    const float r2 = diff_sq<D>(r.x, rec, z);
    const float K = fast_exp2(sc.nc * r2);
    const float* pj = rec + D;
    const float es = eta * s, gs = gam * s;
    const float Phi = dot<D>(r.a, pj) + es * dot<D>(r.a, z) + gs * dot<D>(z, pj) +
                      gam * es * (s * r2 - (float)D);
    const float cz = 2.f * gam * es * s - s * Phi;
#pragma unroll
    for (int d = 0; d < D; ++d) acc[d] = fmaf(K, es * r.a[d] + gs * pj[d] + cz * z[d], acc[d]);
  }
  __device__ static void store(const Scal&, const Row&, const float* t, float* v) {
#pragma unroll
    for (int d = 0; d < D; ++d) v[d] = t[d];
  }
};

// ... and w.r.t. (q_j, p_j) as a row reduction over supports (z' = q_j - x_i = -z):
//   gq_j = -sum_i K [ eta s a_i + gam s p_j - 2 gam eta s^2 z' + s Phi' z' ],
//   Phi' = a_i.p_j - eta s (a_i.z') - gam s (z'.p_j) + gam eta s (s r2 - D);
//   gp_j = sum_i K [ a_i - gam s z' ]
template <int D>
struct OpOdeExtBwdQEta {
  static constexpr int CW4 = cw4(2 * D);
  static constexpr int NACC = 2 * D;
  static constexpr int kNOut = 2;
  static constexpr int kOutW[4] = {D, D, 0, 0};
  static constexpr bool kMin = false;
  struct Row { float q[D]; float p[D]; };
  __device__ static void load_row(const Args& a, int64_t i, Row& r) {
    ld<D>(a.r0, i, r.q);
    ld<D>(a.r1, i, r.p);
  }
  __device__ static void load_col(const Args& a, int64_t j, float* rec) {
    ld<D>(a.c0, j, rec);
    ld<D>(a.c1, j, rec + D);
  }
  __device__ static void pair(const Scal& sc, const Row& r, const float* rec, float* acc) {
    const float s = sc.s, eta = sc.eta, gam = sc.aux0;
    float z[D];
    const float r2 = diff_sq<D>(r.q, rec, z);
    const float K = fast_exp2(sc.nc * r2);
    const float* ai = rec + D;
    const float es = eta * s, gs = gam * s;
    const float Phi = dot<D>(ai, r.p) - es * dot<D>(ai, z) - gs * dot<D>(z, r.p) +
                      gam * es * (s * r2 - (float)D);
    const float cz = -2.f * gam * es * s + s * Phi;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      acc[d] = fmaf(K, fmaf(-gs, z[d], ai[d]), acc[d]);                             // gp
      acc[D + d] = fmaf(K, es * ai[d] + gs * r.p[d] + cz * z[d], acc[D + d]);      // -gq
    }
  }
  __device__ static void store(const Scal&, const Row&, const float* t, float* v) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      v[d] = -t[D + d];  // gq
      v[D + d] = t[d];   // gp
    }
  }
};

}  // namespace dicp
