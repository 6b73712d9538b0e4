// External-point passes (points x carried by the flow of the support (q, p): LDDMM.py:219-227
// forward, and its VJP) and KRed on the packed-FP32 row skeleton (packed.hpp rowred_pk_kernel):
// a thread's two rows as float2, the per-pair algebra as v_pk_*_f32.  These serve the sizes the
// centred reductions (centred.hpp) do not take (tools/cx_ab.py: below ~2e9 pairs): apply,
// custom / decimated / grid support, the C1 and Chui paths, v(x).
//
// Coordinates stay in original units: z = x_i - q_j is exact for nearby points (Sterbenz), so
// the kernel values keep the accuracy of the reference's fp32 arithmetic at any cloud extent
// and offset; K = exp2(nc |z|^2) costs one packed multiply per two pairs more than the
// scaled-coordinate form of the self kernels.  With s = 1/sigma^2 and gam the divergence
// cotangent (device scalar, Scal::aux0):
//
//   forward  (rows x, columns (q, p)):  V = sum K p,  ZP = sum K (z.p),  [Z = sum K z,
//            L = sum K (s r2 - D)]      v = V [+ eta s Z],  g = s ZP [+ eta s L]
//   VJP, x   (rows (x, a), columns (q, p, gam p)):
//            gx = s sum K [gam p - z (a.p + s gam (z.p))]
//   VJP, q/p (rows (q, p), columns (x, a)), z = q - x:  t = a - s gam z,
//            gp = sum K t,  gq = -s sum K (t.p) z - s gam p sum K
// (the sums of OpOdeExtFwd / OpOdeExtBwdX / OpOdeExtBwdQ of lddmm_ops.hpp; parity:
// tests/test_gpu_ext_pk.py, golden and full-size suites).
#pragma once
#include "packed.hpp"

namespace dicp {

// ------------------------------------------------------------------------------------------
// forward
template <int D, bool ETA, bool DIV>
struct OpExtFwdS {
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
  __device__ static void store(const Scal& sc, const Row&, const float* t, float* v) {
    const float s = sc.s;
    constexpr int o = D + (DIV ? 1 : 0);
#pragma unroll
    for (int d = 0; d < D; ++d) v[d] = ETA ? fmaf(sc.eta * s, t[o + d], t[d]) : t[d];
    float g = DIV ? s * t[D] : 0.f;
    if (ETA && DIV) g = fmaf(sc.eta * sc.s, t[o + D], g);
    v[D] = g;
  }
};

template <int D, bool ETA, bool DIV>
struct OpExtFwdPk {
  using Base = OpExtFwdS<D, ETA, DIV>;
  static constexpr int kRP = 2;            // 4 rows per thread on large passes (packed.hpp pk_rp)
  static constexpr int CW4 = Base::CW4;
  static constexpr int NACC = Base::NACC;
  static constexpr int kNOut = Base::kNOut;
  static constexpr bool kMin = false;
  struct Row2 { f2 x[D]; f2 nc, s; };
  __device__ static void load_rows_s(const Args& a, const Scal& sc, int64_t i0, int64_t i1, Row2& r,
                                     typename Base::Row& b0, typename Base::Row& b1) {
    Base::load_row(a, i0, b0);
    Base::load_row(a, i1, b1);
#pragma unroll
    for (int d = 0; d < D; ++d) r.x[d] = f2{b0.x[d], b1.x[d]};
    r.nc = splat(sc.nc);
    r.s = splat(sc.s);
  }
  __device__ static void pair2(const Row2& r, const float* rec, f2* acc) {
    f2 z[D];
    f2 r2 = splat(0.f);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      z[d] = r.x[d] - splat(rec[d]);
      r2 = pk_fma(z[d], z[d], r2);
    }
    const f2 e = r.nc * r2;
    const f2 K = f2{fast_exp2(e.x), fast_exp2(e.y)};
    const float* pj = rec + D;
#pragma unroll
    for (int d = 0; d < D; ++d) acc[d] = pk_fma(K, splat(pj[d]), acc[d]);
    if constexpr (DIV) {
      f2 zp = z[0] * splat(pj[0]);
#pragma unroll
      for (int d = 1; d < D; ++d) zp = pk_fma(z[d], splat(pj[d]), zp);
      acc[D] = pk_fma(K, zp, acc[D]);
    }
    if constexpr (ETA) {
      constexpr int o = D + (DIV ? 1 : 0);
#pragma unroll
      for (int d = 0; d < D; ++d) acc[o + d] = pk_fma(K, z[d], acc[o + d]);
      acc[o + D] = pk_fma(K, pk_fma(r.s, r2, splat(-(float)D)), acc[o + D]);
    }
  }
};

// ------------------------------------------------------------------------------------------
// VJP w.r.t. the carried points x (eta = 0)
template <int D>
struct OpExtBwdXS {
  static constexpr int CW4 = cw4(3 * D);
  static constexpr int NACC = D;
  static constexpr int kNOut = 1;
  static constexpr int kOutW[4] = {D, 0, 0, 0};
  static constexpr bool kMin = false;
  struct Row { float x[D]; float a[D]; };
  __device__ static void load_row(const Args& a, int64_t i, Row& r) {
    ld<D>(a.r0, i, r.x);
    ld<D>(a.r1, i, r.a);
  }
  // column record: q | p | gam p   (staged once per column)
  __device__ static void load_col_s(const Args& a, const Scal& sc, int64_t j, float* rec) {
    ld<D>(a.c0, j, rec);
    ld<D>(a.c1, j, rec + D);
#pragma unroll
    for (int d = 0; d < D; ++d) rec[2 * D + d] = sc.aux0 * rec[D + d];
  }
  __device__ static void store(const Scal& sc, const Row&, const float* t, float* v) {
#pragma unroll
    for (int d = 0; d < D; ++d) v[d] = sc.s * t[d];
  }
};

template <int D>
struct OpExtBwdXPk {
  using Base = OpExtBwdXS<D>;
  static constexpr int kRP = 2;            // 4 rows per thread on large passes (packed.hpp pk_rp)
  static constexpr int CW4 = Base::CW4;
  static constexpr int NACC = D;
  static constexpr int kNOut = 1;
  static constexpr bool kMin = false;
  struct Row2 { f2 x[D], a[D]; f2 g2, nc; };
  __device__ static void load_rows_s(const Args& a, const Scal& sc, int64_t i0, int64_t i1, Row2& r,
                                     typename Base::Row& b0, typename Base::Row& b1) {
    Base::load_row(a, i0, b0);
    Base::load_row(a, i1, b1);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      r.x[d] = f2{b0.x[d], b1.x[d]};
      r.a[d] = f2{b0.a[d], b1.a[d]};
    }
    r.g2 = splat(sc.s * sc.aux0);   // s gam
    r.nc = splat(sc.nc);
  }
  __device__ static void pair2(const Row2& r, const float* rec, f2* acc) {
    f2 z[D];
    f2 r2 = splat(0.f);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      z[d] = r.x[d] - splat(rec[d]);
      r2 = pk_fma(z[d], z[d], r2);
    }
    const f2 e = r.nc * r2;
    const f2 K = f2{fast_exp2(e.x), fast_exp2(e.y)};
    const float* pj = rec + D;
    const float* gp = rec + 2 * D;
    f2 ap = r.a[0] * splat(pj[0]);
    f2 zp = z[0] * splat(pj[0]);
#pragma unroll
    for (int d = 1; d < D; ++d) {
      ap = pk_fma(r.a[d], splat(pj[d]), ap);
      zp = pk_fma(z[d], splat(pj[d]), zp);
    }
    const f2 w = pk_fma(r.g2, zp, ap);
#pragma unroll
    for (int d = 0; d < D; ++d) acc[d] = pk_fma(K, pk_fma(-w, z[d], splat(gp[d])), acc[d]);
  }
};

// ------------------------------------------------------------------------------------------
// VJP w.r.t. the support (q, p) (eta = 0): rows (q, p), columns (x, a); accumulated into gq/gp
template <int D>
struct OpExtBwdQS {
  static constexpr int CW4 = cw4(2 * D);
  static constexpr int NACC = 2 * D + 1;
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
  // t = [gp (D) | sum K (t.p) z (D) | sum K]
  __device__ static void store(const Scal& sc, const Row& r, const float* t, float* v) {
    const float s = sc.s, sg = sc.s * sc.aux0;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      v[d] = -fmaf(s, t[D + d], sg * r.p[d] * t[2 * D]);  // gq
      v[D + d] = t[d];                                     // gp
    }
  }
};

template <int D>
struct OpExtBwdQPk {
  using Base = OpExtBwdQS<D>;
  static constexpr int kRP = 2;            // 4 rows per thread on large passes (packed.hpp pk_rp)
  static constexpr int CW4 = Base::CW4;
  static constexpr int NACC = Base::NACC;
  static constexpr int kNOut = 2;
  static constexpr bool kMin = false;
  struct Row2 { f2 q[D], p[D]; f2 ng2, nc; };
  __device__ static void load_rows_s(const Args& a, const Scal& sc, int64_t i0, int64_t i1, Row2& r,
                                     typename Base::Row& b0, typename Base::Row& b1) {
    Base::load_row(a, i0, b0);
    Base::load_row(a, i1, b1);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      r.q[d] = f2{b0.q[d], b1.q[d]};
      r.p[d] = f2{b0.p[d], b1.p[d]};
    }
    r.ng2 = splat(-sc.s * sc.aux0);   // -s gam
    r.nc = splat(sc.nc);
  }
  __device__ static void pair2(const Row2& r, const float* rec, f2* acc) {
    f2 z[D];
    f2 r2 = splat(0.f);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      z[d] = r.q[d] - splat(rec[d]);
      r2 = pk_fma(z[d], z[d], r2);
    }
    const f2 e = r.nc * r2;
    const f2 K = f2{fast_exp2(e.x), fast_exp2(e.y)};
    const float* ai = rec + D;
    f2 t[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
      t[d] = pk_fma(r.ng2, z[d], splat(ai[d]));   // a - s gam z
      acc[d] = pk_fma(K, t[d], acc[d]);
    }
    f2 tp = t[0] * r.p[0];
#pragma unroll
    for (int d = 1; d < D; ++d) tp = pk_fma(t[d], r.p[d], tp);
    const f2 Kw = K * tp;
#pragma unroll
    for (int d = 0; d < D; ++d) acc[D + d] = pk_fma(Kw, z[d], acc[D + d]);
    acc[2 * D] = acc[2 * D] + K;
  }
};

}  // namespace dicp
