// Pair operators of the BACKWARD passes of the Gaussian-kernel reductions that have no
// fused-kernel gradient (GenDKRed, HessKRed, GradLapKRed, DDKRed, GradKRed_rev).  The
// reference differentiates them through KeOps' / torch's autodiff (kernel.py:147-168,
// :194-207, :284-292); here each gradient is one more row reduction of the same tiled
// skeleton (common.hpp rowred_kernel), with the pair formula derived by hand
// ("Gradients of the reductions"; checked against float64 autograd of
// the oracle in tests/test_gpu_kernel_grads.py).
//
// One generic record layout: rows carry x_i and two optional D-vectors R1_i, R2_i; columns
// carry y_j, two optional D-vectors C1_j, C2_j and an optional scalar cw_j.  A NULL pointer
// reads as zeros (for R2/C2: both NULL reads as the weight 1).  z = x_i - y_j, r2 = |z|^2,
// K = exp(-s r2 / 2), s = 1 / sigma^2.
//
//   HESSW   X_i = sum_j cw_j (R2_i.C2_j) [s^2 (z.u) z - s u] K,  u = R1_i - C1_j
//   HESSWP  X_i = sum_j [s^2 (z.u) z - s u] K,                   u = R1_i (*) C1_j (elementwise)
//   ZDOTV   X_i = sum_j -s (z.a) K C2_j,                         a = R1_i + C1_j
//   HESS3   X_i = sum_j K ( s^2 [(z.g) u + (z.u) g] - s z [s^2 (z.u)(z.g) - s (u.g)] ),
//                                                                u = R1_i - C1_j, g = R2_i + C2_j
//           (the z-gradient of g . HessKRed's pair term: third kernel derivative)
//   GRADLAP3 X_i = sum_j -K [ phi g + s^3 (D + 4 - s r2)(g.z) z ],
//                  phi = s^3 r2 - (D+2) s^2,                     g = R1_i + C1_j
//           (the z-gradient of g . GradLapKRed's pair term)
#pragma once
#include "lddmm_ops.hpp"

namespace dicp {

enum GradKind { kHessW = 0, kHessWP = 1, kZDotV = 2, kHess3 = 3, kGradLap3 = 4 };

template <int W>
__device__ __forceinline__ void ld_or(const float* __restrict__ p, int64_t i, float* dst, float fill = 0.f) {
#pragma unroll
  for (int d = 0; d < W; ++d) dst[d] = p ? p[i * W + d] : fill;
}

template <int D, int KIND>
struct OpGrad {
  // column record: y | C1 | C2 | cw  (only what the kind reads)
  static constexpr int kC1 = D;
  static constexpr int kC2 = 2 * D;
  static constexpr int kCW = 3 * D;
  static constexpr int kRecFloats = KIND == kHessW ? 3 * D + 1 : (KIND == kZDotV || KIND == kHess3) ? 3 * D : 2 * D;
  static constexpr int CW4 = cw4(kRecFloats), NACC = D, kNOut = 1;
  static constexpr int kOutW[4] = {D, 0, 0, 0};
  static constexpr bool kMin = false;
  struct Row { float x[D]; float r1[D]; float r2[D]; };
  __device__ static void load_row(const Args& a, int64_t i, Row& r) {
    ld<D>(a.r0, i, r.x);
    ld_or<D>(a.r1, i, r.r1);
    if (KIND == kHessW && a.r2 == nullptr && a.c2 == nullptr) {
#pragma unroll
      for (int d = 0; d < D; ++d) r.r2[d] = d == 0 ? 1.f : 0.f;   // weight R2.C2 = 1
    } else {
      ld_or<D>(a.r2, i, r.r2);
    }
  }
  __device__ static void load_col(const Args& a, int64_t j, float* rec) {
    ld<D>(a.c0, j, rec);
    ld_or<D>(a.c1, j, rec + kC1);
    if (KIND == kHessW || KIND == kZDotV || KIND == kHess3) {
      if (KIND == kHessW && a.r2 == nullptr && a.c2 == nullptr) {
#pragma unroll
        for (int d = 0; d < D; ++d) rec[kC2 + d] = d == 0 ? 1.f : 0.f;
      } else {
        ld_or<D>(a.c2, j, rec + kC2);
      }
    }
    if (KIND == kHessW) rec[kCW] = a.c3 ? a.c3[j] : 1.f;
  }
  __device__ static void pair(const Scal& sc, const Row& r, const float* rec, float* acc) {
    float z[D];
    const float r2 = diff_sq<D>(r.x, rec, z);
    const float K = fast_exp2(sc.nc * r2);
    const float s = sc.s;
    if constexpr (KIND == kHessW || KIND == kHessWP) {
      float u[D];
#pragma unroll
      for (int d = 0; d < D; ++d) u[d] = KIND == kHessW ? r.r1[d] - rec[kC1 + d] : r.r1[d] * rec[kC1 + d];
      float w = K;
      if (KIND == kHessW) w *= rec[kCW] * dot<D>(r.r2, rec + kC2);
      const float szu = s * dot<D>(z, u);
#pragma unroll
      for (int d = 0; d < D; ++d) acc[d] = fmaf(w, fmaf(szu, z[d], -u[d]), acc[d]);
    } else if constexpr (KIND == kZDotV) {
      float za = 0.f;
#pragma unroll
      for (int d = 0; d < D; ++d) za = fmaf(z[d], r.r1[d] + rec[kC1 + d], za);
      const float w = K * za;
#pragma unroll
      for (int d = 0; d < D; ++d) acc[d] = fmaf(w, rec[kC2 + d], acc[d]);
    } else if constexpr (KIND == kHess3) {
      float u[D], g[D];
#pragma unroll
      for (int d = 0; d < D; ++d) {
        u[d] = r.r1[d] - rec[kC1 + d];
        g[d] = r.r2[d] + rec[kC2 + d];
      }
      const float zg = dot<D>(z, g), zu = dot<D>(z, u), ug = dot<D>(u, g);
      const float c = fmaf(s * zu, zg, -ug);   // s (z.u)(z.g) - (u.g)
#pragma unroll
      for (int d = 0; d < D; ++d) acc[d] = fmaf(K, fmaf(zg, u[d], fmaf(zu, g[d], -c * z[d])), acc[d]);
    } else {  // kGradLap3
      float g[D];
#pragma unroll
      for (int d = 0; d < D; ++d) g[d] = r.r1[d] + rec[kC1 + d];
      const float a = fmaf(s, r2, -(float)(D + 2));               // s r2 - D - 2
      const float b = s * dot<D>(g, z) * ((float)(D + 4) - s * r2); // s (g.z)(D + 4 - s r2)
#pragma unroll
      for (int d = 0; d < D; ++d) acc[d] = fmaf(K, fmaf(a, g[d], b * z[d]), acc[d]);
    }
  }
  __device__ static void store(const Scal& sc, const Row&, const float* t, float* v) {
    const float s = sc.s;
    const float f = (KIND == kHessW || KIND == kHessWP) ? s
                  : KIND == kZDotV ? -s
                  : KIND == kHess3 ? s * s
                  : -s * s;
#pragma unroll
    for (int d = 0; d < D; ++d) v[d] = f * t[d];
  }
};

}  // namespace dicp
