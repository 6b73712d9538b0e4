// Packed-FP32 variant of the symmetric pair-once VJP (lddmm_sym.hpp sym_bwd_kernel, eta = 0):
// the two rows a lane owns are held as float2 vectors, so the pair algebra of SymBwd<D> runs
// as v_pk_*_f32 instructions over both rows (the column record is broadcast into both halves);
// the column-side contributions of the two rows are added once per step (one scalar add per
// accumulator) before the DPP rotation.  Work decomposition, slots and merge are those of
// sym_bwd_kernel, so results differ only by fp32 contraction order.
#pragma once
#include "lddmm_sym.hpp"
#include "packed.hpp"

namespace dicp {

// GQ = false: the gp half only (dL/dp of the VJP), for the last adjoint step of a shooting
// whose start points need no gradient (the support points in Reg_opt): the pair scalars
// pp, u, zu, iap, w and every gq accumulation drop out -- 32 of the 60 packed instructions
// per step remain.
// B0 = true: the cotangent b on mG is zero (the first adjoint step: the loss does not depend
// on the final momenta), so db, zb, pp and every cKzb term drop out -- 40 of 60 remain.
// GT = false: the pair loop leaves out the divergence cotangent's gp terms -gt K z' (row side)
// and +gt K z' (column side): gam = 0 (no cost cotangent), or their row sums are the forward's
// divergence rows zs, which the merge adds once per row (sym_merge_kernel) -- 6 of the 60
// packed instructions per step drop; the column contributions of the lane's two rows are then
// summed by scalar FMAs (DICP_SYMBWD_SCALAR_CT), 6 more packed instructions become 4 scalar
// ones each.
#ifndef DICP_SYMBWD_SCALAR_CT
#define DICP_SYMBWD_SCALAR_CT 1
#endif
// RAW = true: coordinates in original units (Args::scale = 1, no shift, Scal::aux1 = s): z is
// exact for nearby points whatever the cloud's extent; K = exp2(nc r2) costs one packed
// multiply more per step (coord_raw).
template <int D, bool GQ = true, bool B0 = false, bool GT = true, bool RAW = false>
struct SymBwdPk {
  using S = SymBwd<D>;
  static constexpr int W = GQ ? 2 * D : D;
  static constexpr int kMaxWaves = 4;
  // LDS record layout (rec_layout): D = 3 puts each D-vector of the record (q', p, a, b, gam p)
  // in a plane of its own, components x y z, so no broadcast operand sits in a .w slot
#ifndef DICP_SYMBWD_PK_REC3
#define DICP_SYMBWD_PK_REC3 1
#endif
  static constexpr bool kRec3 = DICP_SYMBWD_PK_REC3 && D == 3;
  static constexpr int kPlanes = kRec3 ? 5 : S::CW;
  static constexpr bool kDupW = kRec3;
  __host__ __device__ static constexpr int slot(int i) { return kRec3 ? (i / 3) * 4 + i % 3 : i; }
  // the record's floats as broadcast pairs for the packed algebra; with kDupW the z component
  // of each D-vector is the pair (.z, .w) of its plane -- two registers of one ds_read_b128 --
  // instead of a splat of .z, which the register allocator materialises with a v_mov
  __device__ static void colvec(const float* rec, f2* cv) {
#pragma unroll
    for (int i = 0; i < 5 * D; ++i) cv[i] = splat(rec[i]);
    if constexpr (kDupW) {
#pragma unroll
      for (int m = 0; m < 5; ++m) cv[3 * m + 2] = f2{rec[3 * m + 2], rec[4 * S::CW + m]};
    }
  }
  struct Prm {
    float gt, c;  // gam s1 / alpha, s1 / alpha (SymBwd::Prm)
    float nc, s2; // exponent multiplier (RAW), s / alpha^2 (kS2 scaled, s raw)
  };
  __device__ static Prm params(const Args& a, const Scal& sc) {
    const float cs = sc.aux1 / a.scale;
    return Prm{sc.aux0 * cs, cs, sc.nc, RAW ? sc.s : kS2};
  }
  struct Row2 {
    f2 q[D], p[D], b[D], ia_a[D], gp[D];
  };
  __device__ static void pack(const typename S::Row& r0, const typename S::Row& r1, Row2& r) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      r.q[d] = f2{r0.q[d], r1.q[d]};
      r.p[d] = f2{r0.p[d], r1.p[d]};
      r.b[d] = f2{r0.b[d], r1.b[d]};
      r.ia_a[d] = f2{r0.ia_a[d], r1.ia_a[d]};
      r.gp[d] = f2{r0.gp[d], r1.gp[d]};
    }
  }
  struct Shared {
    f2 z[D], u[D];
    f2 K, w, cKzb;
  };
  __device__ static void shared_terms(const Prm& prm, const Row2& r, const f2* cv, Shared& t) {
    const float c = prm.c;
    const f2* qj = cv;
    const f2* pj = cv + D;
    const f2* aj = cv + 2 * D;
    const f2* bj = cv + 3 * D;
    const f2* gpj = cv + 4 * D;
    f2 r2 = splat(0.f);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      t.z[d] = r.q[d] - qj[d];
      r2 = pk_fma(t.z[d], t.z[d], r2);
    }
    if constexpr (RAW) {
      const f2 e = splat(prm.nc) * r2;
      t.K = f2{fast_exp2(e.x), fast_exp2(e.y)};
    } else {
      t.K = f2{fast_exp2(-r2.x), fast_exp2(-r2.y)};
    }
    if constexpr (B0) {
      // b = 0: u = gam (p_i - p_j), zb = 0
      if constexpr (GQ) {
#pragma unroll
        for (int d = 0; d < D; ++d) t.u[d] = r.gp[d] - gpj[d];
        f2 zu = t.z[0] * t.u[0];
        f2 iap = pk_fma(r.ia_a[0], pj[0], r.p[0] * aj[0]);
#pragma unroll
        for (int d = 1; d < D; ++d) {
          zu = pk_fma(t.z[d], t.u[d], zu);
          iap = pk_fma(r.ia_a[d], pj[d], pk_fma(r.p[d], aj[d], iap));
        }
        t.w = pk_fma(splat(prm.s2), zu, -iap);
      }
      (void)bj;
      (void)c;
    } else if constexpr (GQ) {
      f2 pp = r.p[0] * pj[0];
#pragma unroll
      for (int d = 1; d < D; ++d) pp = pk_fma(r.p[d], pj[d], pp);
      f2 db[D];
#pragma unroll
      for (int d = 0; d < D; ++d) {
        db[d] = r.b[d] - bj[d];
        t.u[d] = pk_fma(-pp, db[d], r.gp[d] - gpj[d]);
      }
      f2 zu = t.z[0] * t.u[0], zb = t.z[0] * db[0];
      f2 iap = pk_fma(r.ia_a[0], pj[0], r.p[0] * aj[0]);
#pragma unroll
      for (int d = 1; d < D; ++d) {
        zu = pk_fma(t.z[d], t.u[d], zu);
        zb = pk_fma(t.z[d], db[d], zb);
        iap = pk_fma(r.ia_a[d], pj[d], pk_fma(r.p[d], aj[d], iap));
      }
      t.w = pk_fma(splat(prm.s2), zu, -iap);
      t.cKzb = (splat(c) * zb) * t.K;
    } else {
      f2 zb = t.z[0] * (r.b[0] - bj[0]);
#pragma unroll
      for (int d = 1; d < D; ++d) zb = pk_fma(t.z[d], r.b[d] - bj[d], zb);
      t.cKzb = (splat(c) * zb) * t.K;
    }
  }
  // ordered pairs (i, j) of both rows, row side only (diag blocks)
  __device__ static void pair_row(const Prm& prm, const Row2& r, const float* rec, f2* acc) {
    const float gt = prm.gt;
    f2 cv[5 * D];
    colvec(rec, cv);
    Shared t;
    shared_terms(prm, r, cv, t);
    const f2* pj = cv + D;
    const f2* aj = cv + 2 * D;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const f2 ka = GT ? pk_fma(splat(-gt), t.z[d], aj[d]) : aj[d];
      if constexpr (B0)
        acc[d] = pk_fma(t.K, ka, acc[d]);
      else
        acc[d] = pk_fma(t.cKzb, pj[d], pk_fma(t.K, ka, acc[d]));
      if constexpr (GQ) acc[D + d] = pk_fma(t.K, pk_fma(t.w, t.z[d], -t.u[d]), acc[D + d]);
    }
  }
  // unordered pairs {i, j} of both rows: row side into acc, the column's total (both rows)
  // into ct (scalars)
  __device__ static void pair_sym(const Prm& prm, const Row2& r, const float* rec, f2* acc, float* ct) {
    const float gt = prm.gt;
    f2 cv[5 * D];
    colvec(rec, cv);
    Shared t;
    shared_terms(prm, r, cv, t);
    const f2* pj = cv + D;
    const f2* aj = cv + 2 * D;
    if constexpr (!GT) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        if constexpr (B0)
          acc[d] = pk_fma(t.K, aj[d], acc[d]);
        else
          acc[d] = pk_fma(t.cKzb, pj[d], pk_fma(t.K, aj[d], acc[d]));
#if DICP_SYMBWD_SCALAR_CT
        float cg = fmaf(t.K.x, r.ia_a[d].x, t.K.y * r.ia_a[d].y);
        if constexpr (!B0) cg = fmaf(t.cKzb.x, r.p[d].x, fmaf(t.cKzb.y, r.p[d].y, cg));
        ct[d] = cg;
#else
        const f2 cg = B0 ? t.K * r.ia_a[d] : pk_fma(t.cKzb, r.p[d], t.K * r.ia_a[d]);
        ct[d] = cg.x + cg.y;
#endif
        if constexpr (GQ) {
          const f2 e = pk_fma(t.w, t.z[d], -t.u[d]);
#if DICP_SYMBWD_SCALAR_CT
          acc[D + d] = pk_fma(t.K, e, acc[D + d]);
          ct[D + d] = -fmaf(t.K.x, e.x, t.K.y * e.y);
#else
          const f2 Ke = t.K * e;
          acc[D + d] = acc[D + d] + Ke;
          ct[D + d] = -(Ke.x + Ke.y);
#endif
        }
      }
      return;
    }
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const f2 tt = pk_fma(splat(gt), t.z[d], r.ia_a[d]);
      if constexpr (B0) {
        acc[d] = pk_fma(t.K, pk_fma(splat(-gt), t.z[d], aj[d]), acc[d]);
        const f2 cg = t.K * tt;
        ct[d] = cg.x + cg.y;
      } else {
        acc[d] = pk_fma(t.cKzb, pj[d], pk_fma(t.K, pk_fma(splat(-gt), t.z[d], aj[d]), acc[d]));
        const f2 cg = pk_fma(t.cKzb, r.p[d], t.K * tt);
        ct[d] = cg.x + cg.y;
      }
      if constexpr (GQ) {
        const f2 e = pk_fma(t.w, t.z[d], -t.u[d]);
        const f2 Ke = t.K * e;
        acc[D + d] = acc[D + d] + Ke;
        ct[D + d] = -(Ke.x + Ke.y);
      }
    }
  }
  // 4 rows per lane (sym_pk4_body): unordered pairs {i, j} of both row pairs r0, r1 against one
  // column record.  The column's total over the 4 rows is formed with packed products -- the
  // two row pairs' terms are chained into one float2 and only its two halves are added as
  // scalars -- instead of two scalar FMAs per row and accumulator (4 rows: per D-component
  // 4-5 v_pk + 1 scalar add instead of 8-10 scalar FMAs + 2 adds).
  __device__ static void pair_sym4(const Prm& prm, const Row2& r0, const Row2& r1, const float* rec,
                                   f2* acc0, f2* acc1, float* ct) {
    const float gt = prm.gt;
    f2 cv[5 * D];
    colvec(rec, cv);
    Shared t0, t1;
    shared_terms(prm, r0, cv, t0);
    shared_terms(prm, r1, cv, t1);
    const f2* pj = cv + D;
    const f2* aj = cv + 2 * D;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const f2 ka0 = GT ? pk_fma(splat(-gt), t0.z[d], aj[d]) : aj[d];
      const f2 ka1 = GT ? pk_fma(splat(-gt), t1.z[d], aj[d]) : aj[d];
      const f2 tt0 = GT ? pk_fma(splat(gt), t0.z[d], r0.ia_a[d]) : r0.ia_a[d];
      const f2 tt1 = GT ? pk_fma(splat(gt), t1.z[d], r1.ia_a[d]) : r1.ia_a[d];
      f2 cg;
      if constexpr (B0) {
        acc0[d] = pk_fma(t0.K, ka0, acc0[d]);
        acc1[d] = pk_fma(t1.K, ka1, acc1[d]);
        cg = pk_fma(t1.K, tt1, t0.K * tt0);
      } else {
        acc0[d] = pk_fma(t0.cKzb, pj[d], pk_fma(t0.K, ka0, acc0[d]));
        acc1[d] = pk_fma(t1.cKzb, pj[d], pk_fma(t1.K, ka1, acc1[d]));
        cg = pk_fma(t1.cKzb, r1.p[d], pk_fma(t1.K, tt1, pk_fma(t0.cKzb, r0.p[d], t0.K * tt0)));
      }
      ct[d] = cg.x + cg.y;
      if constexpr (GQ) {
        const f2 e0 = pk_fma(t0.w, t0.z[d], -t0.u[d]);
        const f2 e1 = pk_fma(t1.w, t1.z[d], -t1.u[d]);
        const f2 Ke0 = t0.K * e0;
        acc0[D + d] = acc0[D + d] + Ke0;
        acc1[D + d] = pk_fma(t1.K, e1, acc1[D + d]);
        const f2 cs = pk_fma(t1.K, e1, Ke0);
        ct[D + d] = -(cs.x + cs.y);
      }
    }
  }
};

// LDS layout of the column records in sym_pk_body: record float i lives in plane
// rec_slot<P>(i) / 4, component rec_slot<P>(i) % 4.  Default: the scalar struct's contiguous
// float4 planes (S::CW of them); an op may define kPlanes / slot(i) to place its broadcast
// operands where the packed algebra's op_sel can pick them without a v_mov.
// kDupW: every plane's .w repeats its .z and is read back as rec[4 S::CW + plane] (see
// SymBwdPk::colvec).
template <class P, class = void>
struct rec_layout {
  static constexpr int kPlanes = P::S::CW;
  static constexpr bool kDupW = false;
  __host__ __device__ static constexpr int slot(int i) { return i; }
};
template <class P>
struct rec_layout<P, std::void_t<decltype(P::kPlanes)>> {
  static constexpr int kPlanes = P::kPlanes;
  static constexpr bool kDupW = P::kDupW;
  __host__ __device__ static constexpr int slot(int i) { return P::slot(i); }
};
// live components of plane m (1 + the highest used component, 0 if none)
template <class P>
__host__ __device__ constexpr int plane_width(int m) {
  if (rec_layout<P>::kDupW) return 4;
  int w = 0;
  for (int i = 0; i < P::S::kUsed; ++i)
    if (rec_layout<P>::slot(i) / 4 == m && rec_layout<P>::slot(i) % 4 + 1 > w) w = rec_layout<P>::slot(i) % 4 + 1;
  return w;
}

#ifndef DICP_SYMBWD_PK_WMIN
#define DICP_SYMBWD_PK_WMIN 1
#endif
#ifndef DICP_SYMBWD_PK_WMAX
#define DICP_SYMBWD_PK_WMAX 4
#endif
#ifndef DICP_SYMBWD_PK_PREFETCH
#define DICP_SYMBWD_PK_PREFETCH 0
#endif
#ifndef DICP_SYMBWD_PK_UNROLL
#define DICP_SYMBWD_PK_UNROLL 2
#endif
// The kernel body, shared by the eta = 0 (SymBwdPk) and eta != 0 (SymBwdEtaPk) VJPs.  P supplies
// S (the scalar struct: CW, W, kUsed, Row, load_row, load_col), Row2 / pack, Prm / params and
// the packed pair_sym / pair_row.
template <class P>
__device__ __forceinline__ void sym_pk_body(Args a, Scal sc, int64_t M, int nG, int L,
                                            float* __restrict__ slab, int64_t slot_stride, int qoff,
                                            int qstride, unsigned bx, unsigned by) {
  using S = typename P::S;
  using LY = rec_layout<P>;
  constexpr int CW = S::CW, NP = LY::kPlanes, W = P::W;
  __shared__ float4 planes[2][NP][kSymG];
  __shared__ float colacc[kSymQ][kSymG][W];
  if (sc.dev0 != nullptr) sc.aux0 = sc.dev0[0];
  const typename P::Prm prm = P::params(a, sc);

  const int Q = qoff + qstride * (int)by, kc = (int)bx;
  const int B0 = kSymQ * Q + kc * L;
  if (B0 >= nG) return;  // uniform for the whole workgroup, before any barrier
  const int B1 = min(B0 + L, nG);
  const int tid = threadIdx.x, wv = tid >> 6, l = tid & 63;
  const int A = kSymQ * Q + wv;

  typename P::Row2 row;
  int64_t ri[2];
  bool rv[2];
  {
    typename S::Row r2[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      ri[r] = (int64_t)A * kSymG + r * 64 + l;
      rv[r] = A < nG && ri[r] < M;
      S::load_row(a, sc, rv[r] ? ri[r] : 0, rv[r], r2[r]);
    }
    P::pack(r2[0], r2[1], row);
  }
  f2 racc[W];
#pragma unroll
  for (int k = 0; k < W; ++k) racc[k] = splat(0.f);

  auto stage = [&](int B, int buf) {
    if (tid < kSymG) {
      const int64_t j = (int64_t)B * kSymG + tid;
      float rec[4 * CW], ph[4 * NP];
      S::load_col(a, sc, j < M ? j : 0, j < M, rec);
#pragma unroll
      for (int k = 0; k < 4 * NP; ++k) ph[k] = 0.f;
#pragma unroll
      for (int i = 0; i < S::kUsed; ++i) ph[LY::slot(i)] = rec[i];
      if constexpr (LY::kDupW) {
#pragma unroll
        for (int m = 0; m < NP; ++m) ph[4 * m + 3] = ph[4 * m + 2];
      }
#pragma unroll
      for (int m = 0; m < NP; ++m)
        planes[buf][m][tid] = make_float4(ph[4 * m], ph[4 * m + 1], ph[4 * m + 2], ph[4 * m + 3]);
    }
  };

  int buf = 0;
  // read a column record: only the S::kUsed live floats (as sym_kernel's ldrec)
  auto ldrec = [&](int col, float* rec) {
    float ph[4 * NP];
#pragma unroll
    for (int m = 0; m < NP; ++m) {
      const int w = plane_width<P>(m);   // compile-time after unrolling
      const float* src = reinterpret_cast<const float*>(&planes[buf][m][col]);
      if (w == 4) {
        const float4 v = *reinterpret_cast<const float4*>(src);
        ph[4 * m] = v.x, ph[4 * m + 1] = v.y, ph[4 * m + 2] = v.z, ph[4 * m + 3] = v.w;
      } else if (w == 3) {
        const float3 v = *reinterpret_cast<const float3*>(src);
        ph[4 * m] = v.x, ph[4 * m + 1] = v.y, ph[4 * m + 2] = v.z, ph[4 * m + 3] = 0.f;
      } else if (w == 2) {
        const float2 v = *reinterpret_cast<const float2*>(src);
        ph[4 * m] = v.x, ph[4 * m + 1] = v.y, ph[4 * m + 2] = ph[4 * m + 3] = 0.f;
      } else {
        ph[4 * m] = src[0], ph[4 * m + 1] = ph[4 * m + 2] = ph[4 * m + 3] = 0.f;
      }
    }
#pragma unroll
    for (int i = 0; i < 4 * CW; ++i) rec[i] = i < S::kUsed ? ph[LY::slot(i)] : 0.f;
#pragma unroll
    for (int m = 0; m < NP; ++m) rec[4 * CW + m] = LY::kDupW ? ph[4 * m + 3] : 0.f;
  };
  stage(B0, 0);
  __syncthreads();
  for (int B = B0; B < B1; ++B) {
    if (B + 1 < B1) stage(B + 1, buf ^ 1);
    const bool sym = A < B;          // wave-uniform
    const bool diag = A == B;
#pragma unroll 1
    for (int h = 0; h < 2; ++h) {
      float cacc[W];
#pragma unroll
      for (int k = 0; k < W; ++k) cacc[k] = 0.f;
      if (sym) {
#if DICP_SYMBWD_PK_PREFETCH
        // register double-buffer of the column record (as sym_kernel): step k2 + 1's LDS
        // reads are issued before step k2's algebra, so their latency is not exposed
        float rec[4 * CW + NP];
        ldrec(h * 64 + (l & 63), rec);
#pragma unroll DICP_SYMBWD_PK_UNROLL
        for (int k2 = 0; k2 < 64; ++k2) {
          float nxt[4 * CW + NP];
          __builtin_amdgcn_s_waitcnt(kLgkm0);
          ldrec(h * 64 + ((l + k2 + 1) & 63), nxt);  // k2 = 63 wraps to column l: harmless
          __builtin_amdgcn_sched_barrier(0);
          float ct[W];
          P::pair_sym(prm, row, rec, racc, ct);
#pragma unroll
          for (int k = 0; k < W; ++k) cacc[k] = rol1(cacc[k]) + ct[k];
#pragma unroll
          for (int k = 0; k < 4 * CW + NP; ++k) rec[k] = nxt[k];
        }
#else
#pragma unroll DICP_SYMBWD_PK_UNROLL
        for (int k2 = 0; k2 < 64; ++k2) {
          const int col = h * 64 + ((l + k2) & 63);
          float rec[4 * CW + NP];
          ldrec(col, rec);
          float ct[W];
          P::pair_sym(prm, row, rec, racc, ct);
#pragma unroll
          for (int k = 0; k < W; ++k) cacc[k] = rol1(cacc[k]) + ct[k];
        }
#endif
#pragma unroll
        for (int k = 0; k < W; ++k) cacc[k] = rol1(cacc[k]);
      } else if (diag) {
#pragma unroll 2
        for (int k2 = 0; k2 < 64; ++k2) {
          const int col = h * 64 + ((l + k2) & 63);
          float rec[4 * CW + NP];
          ldrec(col, rec);
          P::pair_row(prm, row, rec, racc);
        }
      }
#pragma unroll
      for (int k = 0; k < W; ++k) colacc[wv][h * 64 + l][k] = cacc[k];
    }
    __syncthreads();
    if (tid < kSymG) {
      const int64_t j = (int64_t)B * kSymG + tid;
      if (j < M) {
        float* dst = slab + (int64_t)Q * slot_stride + j * W;
#pragma unroll
        for (int k = 0; k < W; ++k)
          dst[k] = ((colacc[0][tid][k] + colacc[1][tid][k]) + colacc[2][tid][k]) + colacc[3][tid][k];
      }
    }
    __syncthreads();
    buf ^= 1;
  }
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    if (!rv[r]) continue;
    float* dst = slab + (int64_t)(Q + 1 + kc) * slot_stride + ri[r] * W;
#pragma unroll
    for (int k = 0; k < W; ++k) dst[k] = r == 0 ? racc[k].x : racc[k].y;
  }
}

// 4 rows per lane (dicp_set_option "sym_rp", automatic from ~90k points): sym_pk_body with 256-point
// groups -- a wave's lane holds rows r*64 + l (r = 0..3) of its group as two float2 row pairs,
// the column record and the DPP rotation of the column sums are shared by the 4 rows, and a
// column group is staged as 256 records (four 64-column quarters).  Slots and merge are those
// of the 128 form with G = 256 (sym_merge_kernel<..., kSymG4>).
#ifndef DICP_SYMBWD4_UNROLL
#define DICP_SYMBWD4_UNROLL 2
#endif
#ifndef DICP_SYMBWD4_WMIN
#define DICP_SYMBWD4_WMIN 1
#endif
template <class P>
__device__ __forceinline__ void sym_pk4_body(Args a, Scal sc, int64_t M, int nG, int L,
                                             float* __restrict__ slab, int64_t slot_stride, int qoff,
                                             int qstride, unsigned bx, unsigned by) {
  using S = typename P::S;
  using LY = rec_layout<P>;
  constexpr int G = kSymG4;
  constexpr int CW = S::CW, NP = LY::kPlanes, W = P::W;
  __shared__ float4 planes[2][NP][G];
  __shared__ float colacc[kSymQ][G][W];
  if (sc.dev0 != nullptr) sc.aux0 = sc.dev0[0];
  const typename P::Prm prm = P::params(a, sc);

  const int Q = qoff + qstride * (int)by, kc = (int)bx;
  const int B0 = kSymQ * Q + kc * L;
  if (B0 >= nG) return;  // uniform for the whole workgroup, before any barrier
  const int B1 = min(B0 + L, nG);
  const int tid = threadIdx.x, wv = tid >> 6, l = tid & 63;
  const int A = kSymQ * Q + wv;

  typename P::Row2 row[2];
  int64_t ri[4];
  bool rv[4];
  {
    typename S::Row r4[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      ri[r] = (int64_t)A * G + r * 64 + l;
      rv[r] = A < nG && ri[r] < M;
      S::load_row(a, sc, rv[r] ? ri[r] : 0, rv[r], r4[r]);
    }
    P::pack(r4[0], r4[1], row[0]);
    P::pack(r4[2], r4[3], row[1]);
  }
  f2 racc[2][W];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int k = 0; k < W; ++k) racc[h][k] = splat(0.f);

  auto stage = [&](int B, int buf) {
    const int64_t j = (int64_t)B * G + tid;   // 256 threads: one record each
    float rec[4 * CW], ph[4 * NP];
    S::load_col(a, sc, j < M ? j : 0, j < M, rec);
#pragma unroll
    for (int k = 0; k < 4 * NP; ++k) ph[k] = 0.f;
#pragma unroll
    for (int i = 0; i < S::kUsed; ++i) ph[LY::slot(i)] = rec[i];
    if constexpr (LY::kDupW) {
#pragma unroll
      for (int m = 0; m < NP; ++m) ph[4 * m + 3] = ph[4 * m + 2];
    }
#pragma unroll
    for (int m = 0; m < NP; ++m)
      planes[buf][m][tid] = make_float4(ph[4 * m], ph[4 * m + 1], ph[4 * m + 2], ph[4 * m + 3]);
  };

  int buf = 0;
  auto ldrec = [&](int col, float* rec) {
    float ph[4 * NP];
#pragma unroll
    for (int m = 0; m < NP; ++m) {
      const int w = plane_width<P>(m);
      const float* src = reinterpret_cast<const float*>(&planes[buf][m][col]);
      if (w == 4) {
        const float4 v = *reinterpret_cast<const float4*>(src);
        ph[4 * m] = v.x, ph[4 * m + 1] = v.y, ph[4 * m + 2] = v.z, ph[4 * m + 3] = v.w;
      } else if (w == 3) {
        const float3 v = *reinterpret_cast<const float3*>(src);
        ph[4 * m] = v.x, ph[4 * m + 1] = v.y, ph[4 * m + 2] = v.z, ph[4 * m + 3] = 0.f;
      } else if (w == 2) {
        const float2 v = *reinterpret_cast<const float2*>(src);
        ph[4 * m] = v.x, ph[4 * m + 1] = v.y, ph[4 * m + 2] = ph[4 * m + 3] = 0.f;
      } else {
        ph[4 * m] = src[0], ph[4 * m + 1] = ph[4 * m + 2] = ph[4 * m + 3] = 0.f;
      }
    }
#pragma unroll
    for (int i = 0; i < 4 * CW; ++i) rec[i] = i < S::kUsed ? ph[LY::slot(i)] : 0.f;
#pragma unroll
    for (int m = 0; m < NP; ++m) rec[4 * CW + m] = LY::kDupW ? ph[4 * m + 3] : 0.f;
  };
  stage(B0, 0);
  __syncthreads();
  for (int B = B0; B < B1; ++B) {
    if (B + 1 < B1) stage(B + 1, buf ^ 1);
    const bool sym = A < B;          // wave-uniform
    const bool diag = A == B;
#pragma unroll 1
    for (int h = 0; h < G / 64; ++h) {
      float cacc[W];
#pragma unroll
      for (int k = 0; k < W; ++k) cacc[k] = 0.f;
      if (sym) {
#pragma unroll DICP_SYMBWD4_UNROLL
        for (int k2 = 0; k2 < 64; ++k2) {
          const int col = h * 64 + ((l + k2) & 63);
          float rec[4 * CW + NP];
          ldrec(col, rec);
          float ct[W];
          P::pair_sym4(prm, row[0], row[1], rec, racc[0], racc[1], ct);
#pragma unroll
          for (int k = 0; k < W; ++k) cacc[k] = rol1(cacc[k]) + ct[k];
        }
#pragma unroll
        for (int k = 0; k < W; ++k) cacc[k] = rol1(cacc[k]);
      } else if (diag) {
#pragma unroll 2
        for (int k2 = 0; k2 < 64; ++k2) {
          const int col = h * 64 + ((l + k2) & 63);
          float rec[4 * CW + NP];
          ldrec(col, rec);
          P::pair_row(prm, row[0], rec, racc[0]);
          P::pair_row(prm, row[1], rec, racc[1]);
        }
      }
#pragma unroll
      for (int k = 0; k < W; ++k) colacc[wv][h * 64 + l][k] = cacc[k];
    }
    __syncthreads();
    {
      const int64_t j = (int64_t)B * G + tid;
      if (j < M) {
        float* dst = slab + (int64_t)Q * slot_stride + j * W;
#pragma unroll
        for (int k = 0; k < W; ++k)
          dst[k] = ((colacc[0][tid][k] + colacc[1][tid][k]) + colacc[2][tid][k]) + colacc[3][tid][k];
      }
    }
    __syncthreads();
    buf ^= 1;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (!rv[r]) continue;
    float* dst = slab + (int64_t)(Q + 1 + kc) * slot_stride + ri[r] * W;
    const f2* ra = racc[r >> 1];
#pragma unroll
    for (int k = 0; k < W; ++k) dst[k] = (r & 1) == 0 ? ra[k].x : ra[k].y;
  }
}

template <int D, bool GQ, bool B0, bool GT, bool RAW>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(DICP_SYMBWD4_WMIN, 4))) void sym_bwd_pk4_kernel(
    Args a, Scal sc, int64_t M, int nG, int L, float* __restrict__ slab, int64_t slot_stride, int qoff,
    int qstride) {
  sym_pk4_body<SymBwdPk<D, GQ, B0, GT, RAW>>(a, sc, M, nG, L, slab, slot_stride, qoff, qstride, blockIdx.x,
                                             blockIdx.y);
}

template <int D, bool GQ, bool B0, bool GT, bool RAW>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(DICP_SYMBWD_PK_WMIN, DICP_SYMBWD_PK_WMAX))) void sym_bwd_pk_kernel(
    Args a, Scal sc, int64_t M, int nG, int L, float* __restrict__ slab, int64_t slot_stride, int qoff,
    int qstride) {
  sym_pk_body<SymBwdPk<D, GQ, B0, GT, RAW>>(a, sc, M, nG, L, slab, slot_stride, qoff, qstride, blockIdx.x,
                                            blockIdx.y);
}

// batched forms (batch.hpp): blockIdx.z = the recorded call (SymEntry, lddmm_sym.hpp)
template <int D, bool GQ, bool B0, bool GT, bool RAW>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(DICP_SYMBWD_PK_WMIN, DICP_SYMBWD_PK_WMAX))) void sym_bwd_pk_batch_kernel(
    BatchTab<SymEntry> t) {
  const SymEntry& e = t.e[blockIdx.z];
  if (blockIdx.x >= e.gx || blockIdx.y >= e.gy) return;
  sym_pk_body<SymBwdPk<D, GQ, B0, GT, RAW>>(e.a, e.sc, e.M, e.nG, e.L, e.slab, e.slot_stride, e.qoff, e.qstride,
                                            blockIdx.x, blockIdx.y);
}
template <int D, bool GQ, bool B0, bool GT, bool RAW>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(DICP_SYMBWD4_WMIN, 4))) void sym_bwd_pk4_batch_kernel(
    BatchTab<SymEntry> t) {
  const SymEntry& e = t.e[blockIdx.z];
  if (blockIdx.x >= e.gx || blockIdx.y >= e.gy) return;
  sym_pk4_body<SymBwdPk<D, GQ, B0, GT, RAW>>(e.a, e.sc, e.M, e.nG, e.L, e.slab, e.slot_stride, e.qoff, e.qstride,
                                             blockIdx.x, blockIdx.y);
}
template <int D, bool GQ, bool B0, bool GT, bool RAW>
int sym_bwd_pk_batch_flush(const std::vector<const void*>& es, hipStream_t st) {
  return batch_launch<SymEntry>(sym_bwd_pk_batch_kernel<D, GQ, B0, GT, RAW>, es, st, "sym_bwd_pk");
}
template <int D, bool GQ, bool B0, bool GT, bool RAW>
int sym_bwd_pk4_batch_flush(const std::vector<const void*>& es, hipStream_t st) {
  return batch_launch<SymEntry>(sym_bwd_pk4_batch_kernel<D, GQ, B0, GT, RAW>, es, st, "sym_bwd_pk4");
}

// Packed-FP32 rows of the eta != 0 symmetric VJP (lddmm_sym.hpp SymBwdEta, the logdet /
// gradcomponent model): the same per-pair algebra on float2 rows, column side summed over the
// lane's two rows before the rotation (the scalar kernel's ct = cgp(row 0) + cgp(row 1)).
// GQ = false: the gp half only (the last adjoint step when q0 needs no gradient): the pair
// scalars pp, ap, zp, za, bp, Phi, czq, cdb, cdp and the G terms drop out.
// B0 = true: the cotangent b on mG is zero (the first adjoint step): db, zb, bp, pp and szbK
// drop out, Tv = -gs z.
template <int D, bool GQ = true, bool B0 = false>
struct SymBwdEtaPk {
  using S = SymBwdEta<D>;
  using Prm = typename S::Prm;
  static constexpr int W = GQ ? S::W : D;
  __device__ static Prm params(const Args& a, const Scal& sc) { return S::params(a, sc); }
  struct Row2 {
    f2 q[D], p[D], a[D], b[D];
  };
  __device__ static void pack(const typename S::Row& r0, const typename S::Row& r1, Row2& r) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      r.q[d] = f2{r0.q[d], r1.q[d]};
      r.p[d] = f2{r0.p[d], r1.p[d]};
      r.a[d] = f2{r0.a[d], r1.a[d]};
      r.b[d] = f2{r0.b[d], r1.b[d]};
    }
  }
  struct Shared {
    f2 z[D], db[D], da[D], dp[D];
    f2 K, szbK, czp, cdb, cdp, czq;
  };
  __device__ static void shared_terms(const Prm& P, const Row2& r, const float* rec, Shared& t) {
    const float* pj = rec + D;
    const float* aj = rec + 2 * D;
    const float* bj = rec + 3 * D;
    f2 r2 = splat(0.f);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      t.z[d] = r.q[d] - splat(rec[d]);
      r2 = pk_fma(t.z[d], t.z[d], r2);
      if constexpr (GQ) {
        t.da[d] = r.a[d] - splat(aj[d]);
        t.dp[d] = r.p[d] - splat(pj[d]);
      }
      if constexpr (!B0) t.db[d] = r.b[d] - splat(bj[d]);
    }
    t.K = f2{fast_exp2(P.nc * r2.x), fast_exp2(P.nc * r2.y)};
    if constexpr (!GQ) {
      if constexpr (!B0) {
        f2 zb = t.z[0] * t.db[0];
#pragma unroll
        for (int d = 1; d < D; ++d) zb = pk_fma(t.z[d], t.db[d], zb);
        t.czp = splat(P.s) * zb * splat(P.es) - splat(P.gs);
        t.szbK = splat(P.s) * zb * t.K;
      }
    } else if constexpr (B0) {
      f2 ap = pk_fma(r.a[0], splat(pj[0]), r.p[0] * splat(aj[0]));
      f2 zp = t.z[0] * t.dp[0], za = t.z[0] * t.da[0];
#pragma unroll
      for (int d = 1; d < D; ++d) {
        ap = pk_fma(r.a[d], splat(pj[d]), pk_fma(r.p[d], splat(aj[d]), ap));
        zp = pk_fma(t.z[d], t.dp[d], zp);
        za = pk_fma(t.z[d], t.da[d], za);
      }
      const f2 sr2 = splat(P.s) * r2;
      const f2 Phi = ap + splat(P.es) * za - splat(P.gs) * zp +
                     splat(2.f * P.gam * P.es) * (sr2 - splat((float)D));
      t.czq = splat(4.f * P.gam * P.es2) - splat(P.s) * Phi;
    } else {
      f2 pp = r.p[0] * splat(pj[0]);
      f2 ap = pk_fma(r.a[0], splat(pj[0]), r.p[0] * splat(aj[0]));
      f2 zb = t.z[0] * t.db[0], zp = t.z[0] * t.dp[0], za = t.z[0] * t.da[0], bp = t.db[0] * t.dp[0];
#pragma unroll
      for (int d = 1; d < D; ++d) {
        pp = pk_fma(r.p[d], splat(pj[d]), pp);
        ap = pk_fma(r.a[d], splat(pj[d]), pk_fma(r.p[d], splat(aj[d]), ap));
        zb = pk_fma(t.z[d], t.db[d], zb);
        zp = pk_fma(t.z[d], t.dp[d], zp);
        za = pk_fma(t.z[d], t.da[d], za);
        bp = pk_fma(t.db[d], t.dp[d], bp);
      }
      const f2 sr2 = splat(P.s) * r2;
      const f2 sr2D2 = sr2 - splat((float)(D + 2));
      const f2 Phi = ap + splat(P.es) * za + splat(P.s) * pp * zb +
                     splat(P.es) * (splat(P.s) * zp * zb - bp) - splat(P.e2s2) * zb * sr2D2 -
                     splat(P.gs) * zp + splat(2.f * P.gam * P.es) * (sr2 - splat((float)D));
      t.czp = splat(P.s) * zb * splat(P.es) - splat(P.gs);
      t.czq = splat(-2.f * P.e2s2 * P.s) * zb + splat(4.f * P.gam * P.es2) - splat(P.s) * Phi;
      t.cdb = splat(P.s) * pp + splat(P.es2) * zp - splat(P.e2s2) * sr2D2;
      t.cdp = splat(P.es2) * zb - splat(P.gs);
      t.szbK = splat(P.s) * zb * t.K;
    }
  }
  // Tv_d = czp z_d - es db_d (B0: czp = -gs, db = 0)
  __device__ static f2 tv(const Prm& P, const Shared& t, int d) {
    if constexpr (B0)
      return splat(-P.gs) * t.z[d];
    else
      return pk_fma(t.czp, t.z[d], splat(-P.es) * t.db[d]);
  }
  // G_d (before the factor K) = es da_d + cdb db_d + cdp dp_d + czq z_d (B0: cdb db = 0, cdp = -gs)
  __device__ static f2 gterm(const Prm& P, const Shared& t, int d) {
    if constexpr (B0)
      return pk_fma(splat(P.es), t.da[d], pk_fma(splat(-P.gs), t.dp[d], t.czq * t.z[d]));
    else
      return pk_fma(splat(P.es), t.da[d], pk_fma(t.cdb, t.db[d], pk_fma(t.cdp, t.dp[d], t.czq * t.z[d])));
  }
  // ordered pairs of both rows, row side only (diag blocks)
  __device__ static void pair_row(const Prm& P, const Row2& r, const float* rec, f2* acc) {
    Shared t;
    shared_terms(P, r, rec, t);
    const float* pj = rec + D;
    const float* aj = rec + 2 * D;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const f2 Tv = tv(P, t, d);
      if constexpr (B0)
        acc[d] = pk_fma(t.K, splat(aj[d]) + Tv, acc[d]);
      else
        acc[d] = pk_fma(t.K, splat(aj[d]) + Tv, pk_fma(t.szbK, splat(pj[d]), acc[d]));
      if constexpr (GQ) acc[D + d] = pk_fma(t.K, gterm(P, t, d), acc[D + d]);
    }
  }
  // unordered pairs of both rows: row side into acc, the column's total (both rows) into ct
  __device__ static void pair_sym(const Prm& P, const Row2& r, const float* rec, f2* acc, float* ct) {
    Shared t;
    shared_terms(P, r, rec, t);
    const float* pj = rec + D;
    const float* aj = rec + 2 * D;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const f2 Tv = tv(P, t, d);
      f2 cgp;
      if constexpr (B0) {
        acc[d] = pk_fma(t.K, splat(aj[d]) + Tv, acc[d]);
        cgp = t.K * (r.a[d] - Tv);
      } else {
        acc[d] = pk_fma(t.K, splat(aj[d]) + Tv, pk_fma(t.szbK, splat(pj[d]), acc[d]));
        cgp = pk_fma(t.K, r.a[d] - Tv, t.szbK * r.p[d]);
      }
      ct[d] = cgp.x + cgp.y;
      if constexpr (GQ) {
        const f2 G = t.K * gterm(P, t, d);
        acc[D + d] = acc[D + d] + G;
        ct[D + d] = -G.x - G.y;
      }
    }
  }
};

template <int D, bool GQ, bool B0>
__global__ __launch_bounds__(256) void sym_bwd_eta_pk_kernel(Args a, Scal sc, int64_t M, int nG, int L,
                                                             float* __restrict__ slab, int64_t slot_stride,
                                                             int qoff, int qstride) {
  sym_pk_body<SymBwdEtaPk<D, GQ, B0>>(a, sc, M, nG, L, slab, slot_stride, qoff, qstride, blockIdx.x, blockIdx.y);
}

// Packed-FP32 rows of the symmetric (pair-once) eta = 0 forward (lddmm_sym.hpp SymFwd): the
// lane's two rows as float2; per unordered pair the row side (V, Gs', Z') is packed and the
// column side (K p_i, -Kpp z, -K z) is summed over the two rows in scalar form before the
// DPP rotation.  Same slots and merge as sym_kernel<SymFwd>.
template <int D, bool DIV>
struct SymFwdPk {
  using S = SymFwd<D, DIV>;
  static constexpr int W = S::W;
  struct Prm {};
  __device__ static Prm params(const Args&, const Scal&) { return Prm{}; }
  struct Row2 {
    f2 q[D], p[D];
  };
  __device__ static void pack(const typename S::Row& r0, const typename S::Row& r1, Row2& r) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      r.q[d] = f2{r0.q[d], r1.q[d]};
      r.p[d] = f2{r0.p[d], r1.p[d]};
    }
  }
  __device__ static void pair_row(const Prm&, const Row2& r, const float* rec, f2* acc) {
    f2 z[D];
    f2 r2 = splat(0.f);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      z[d] = r.q[d] - splat(rec[d]);
      r2 = pk_fma(z[d], z[d], r2);
    }
    const f2 K = f2{fast_exp2(-r2.x), fast_exp2(-r2.y)};
    const float* pj = rec + D;
    f2 pp = r.p[0] * splat(pj[0]);
#pragma unroll
    for (int d = 1; d < D; ++d) pp = pk_fma(r.p[d], splat(pj[d]), pp);
    const f2 Kpp = K * pp;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      acc[d] = pk_fma(K, splat(pj[d]), acc[d]);
      acc[D + d] = pk_fma(Kpp, z[d], acc[D + d]);
      if (DIV) acc[2 * D + d] = pk_fma(K, z[d], acc[2 * D + d]);
    }
  }
  __device__ static void pair_sym(const Prm&, const Row2& r, const float* rec, f2* acc, float* ct) {
    f2 z[D];
    f2 r2 = splat(0.f);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      z[d] = r.q[d] - splat(rec[d]);
      r2 = pk_fma(z[d], z[d], r2);
    }
    const f2 K = f2{fast_exp2(-r2.x), fast_exp2(-r2.y)};
    const float* pj = rec + D;
    f2 pp = r.p[0] * splat(pj[0]);
#pragma unroll
    for (int d = 1; d < D; ++d) pp = pk_fma(r.p[d], splat(pj[d]), pp);
    const f2 Kpp = K * pp;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      acc[d] = pk_fma(K, splat(pj[d]), acc[d]);
      acc[D + d] = pk_fma(Kpp, z[d], acc[D + d]);
      if (DIV) acc[2 * D + d] = pk_fma(K, z[d], acc[2 * D + d]);
      // column j's side: sum over the lane's two rows, (i, j) -> (j, i) flips z
      ct[d] = fmaf(K.x, r.p[d].x, K.y * r.p[d].y);
      ct[D + d] = -fmaf(Kpp.x, z[d].x, Kpp.y * z[d].y);
      if (DIV) ct[2 * D + d] = -fmaf(K.x, z[d].x, K.y * z[d].y);
    }
  }
};

// The symmetric eta = 0 forward with 4 rows per lane (sym_pk4_body; fwd_alg 5): per unordered
// pair the row side of each row pair as SymFwdPk, and the column side of the 4 rows (K p_i,
// -Kpp z, -K z) chained over the two row pairs in packed form, so that only one scalar add per
// accumulator (and one DPP rotation, shared by the 4 rows) remains per column: per step 56 v_pk
// + 9 adds + 9 DPP + 4 exp for 8 ordered pair-equivalents, against 76 v_pk + 8 exp of the
// ordered 4-row forward.  D = 3 records as planes [q (3) | q_z] [p (3) | p_z] (z components as
// aligned register pairs, as SymBwdPk).
template <int D, bool DIV>
struct SymFwdPk4 {
  using S = SymFwd<D, DIV>;
  static constexpr int W = S::W;
  static constexpr bool kRec3 = D == 3;
  static constexpr int kPlanes = kRec3 ? 2 : S::CW;
  static constexpr bool kDupW = kRec3;
  __host__ __device__ static constexpr int slot(int i) { return kRec3 ? (i / 3) * 4 + i % 3 : i; }
  struct Prm {};
  __device__ static Prm params(const Args&, const Scal&) { return Prm{}; }
  using Row2 = typename SymFwdPk<D, DIV>::Row2;
  __device__ static void pack(const typename S::Row& r0, const typename S::Row& r1, Row2& r) {
    SymFwdPk<D, DIV>::pack(r0, r1, r);
  }
  __device__ static void colvec(const float* rec, f2* cv) {
#pragma unroll
    for (int i = 0; i < 2 * D; ++i) cv[i] = splat(rec[i]);
    if constexpr (kDupW) {
#pragma unroll
      for (int m = 0; m < 2; ++m) cv[3 * m + 2] = f2{rec[3 * m + 2], rec[4 * S::CW + m]};
    }
  }
  struct Sh {
    f2 z[D];
    f2 K, Kpp;
  };
  __device__ static void shared(const Row2& r, const f2* cv, Sh& t) {
    f2 r2 = splat(0.f);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      t.z[d] = r.q[d] - cv[d];
      r2 = pk_fma(t.z[d], t.z[d], r2);
    }
    t.K = f2{fast_exp2(-r2.x), fast_exp2(-r2.y)};
    f2 pp = r.p[0] * cv[D];
#pragma unroll
    for (int d = 1; d < D; ++d) pp = pk_fma(r.p[d], cv[D + d], pp);
    t.Kpp = t.K * pp;
  }
  __device__ static void row_side(const Sh& t, const f2* cv, f2* acc) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      acc[d] = pk_fma(t.K, cv[D + d], acc[d]);
      acc[D + d] = pk_fma(t.Kpp, t.z[d], acc[D + d]);
      if (DIV) acc[2 * D + d] = pk_fma(t.K, t.z[d], acc[2 * D + d]);
    }
  }
  __device__ static void pair_row(const Prm&, const Row2& r, const float* rec, f2* acc) {
    f2 cv[2 * D];
    colvec(rec, cv);
    Sh t;
    shared(r, cv, t);
    row_side(t, cv, acc);
  }
  __device__ static void pair_sym4(const Prm&, const Row2& r0, const Row2& r1, const float* rec, f2* acc0,
                                   f2* acc1, float* ct) {
    f2 cv[2 * D];
    colvec(rec, cv);
    Sh t0, t1;
    shared(r0, cv, t0);
    shared(r1, cv, t1);
    row_side(t0, cv, acc0);
    row_side(t1, cv, acc1);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      // column j's side over the 4 rows, (i, j) -> (j, i) flips z
      const f2 cV = pk_fma(t1.K, r1.p[d], t0.K * r0.p[d]);
      ct[d] = cV.x + cV.y;
      const f2 cG = pk_fma(t1.Kpp, t1.z[d], t0.Kpp * t0.z[d]);
      ct[D + d] = -(cG.x + cG.y);
      if (DIV) {
        const f2 cZ = pk_fma(t1.K, t1.z[d], t0.K * t0.z[d]);
        ct[2 * D + d] = -(cZ.x + cZ.y);
      }
    }
  }
};

// ---- the symmetric eta = 0 forward with 2 NRP rows per lane (NRP = 4: 8 rows, 512-point
// groups, fwd from DICP_SYM_FWD8_MIN_M points; NRP = 3: 6 rows, 384-point groups; dicp_set_option
// "sym_fwd_rows" 4 / 6 / 8 forces) -- a lane holds rows r * 64 + l (r < 2 NRP) of its group as
// NRP float2 row pairs, so each column's record, its LDS reads, and the column side's one scalar
// add + DPP rotation per accumulator serve 2 NRP rows instead of 4 (~19% of the
// 4-row loop's issue went to that column side).  8 rows per step: 76 v_pk (row side) + 36 v_pk
// + 9 adds + 9 DPP (column side) + 8 exp for 16 ordered pair-equivalents, against 2 x (56 v_pk +
// 9 + 9 + 4 exp) for the 4-row form.  Own body (the 4-row sym_pk4_body also runs the tuned
// VJP, whose schedule must not move); slots and merge as the 4-row form with G = 128 NRP.
// 8 rows need 208 VGPRs (2 waves / SIMD, 2 workgroups per CU); 6 rows fit 3 waves / SIMD.
template <int NRP>
constexpr int sym_fwd_group() { return 128 * NRP; }
constexpr int kSymG8 = 512;
template <int D, bool DIV, int NRP>
struct SymFwdPkN {
  using P4 = SymFwdPk4<D, DIV>;
  using S = typename P4::S;
  static constexpr int W = S::W;
  using Row2 = typename P4::Row2;
  using Sh = typename P4::Sh;
  __device__ static void pair_sym(const Row2* r, const float* rec, f2 (*acc)[W], float* ct) {
    f2 cv[2 * D];
    P4::colvec(rec, cv);
    // per row pair: its shared terms, row side, and its share of the column side chained into
    // the column partials in row-pair order
    f2 cV[D], cG[D], cZ[D];
#pragma unroll
    for (int h = 0; h < NRP; ++h) {
      Sh t;
      P4::shared(r[h], cv, t);
      P4::row_side(t, cv, acc[h]);
#pragma unroll
      for (int d = 0; d < D; ++d) {
        // column j's side over the 2 NRP rows; (i, j) -> (j, i) flips z
        cV[d] = h == 0 ? t.K * r[h].p[d] : pk_fma(t.K, r[h].p[d], cV[d]);
        cG[d] = h == 0 ? t.Kpp * t.z[d] : pk_fma(t.Kpp, t.z[d], cG[d]);
        if (DIV) cZ[d] = h == 0 ? t.K * t.z[d] : pk_fma(t.K, t.z[d], cZ[d]);
      }
    }
#pragma unroll
    for (int d = 0; d < D; ++d) {
      ct[d] = cV[d].x + cV[d].y;
      ct[D + d] = -(cG[d].x + cG[d].y);
      if (DIV) ct[2 * D + d] = -(cZ[d].x + cZ[d].y);
    }
  }
  __device__ static void pair_row(const Row2& r, const float* rec, f2* acc) {
    P4::pair_row(typename P4::Prm{}, r, rec, acc);
  }
};

#ifndef DICP_SYMFWD8_WPE
#define DICP_SYMFWD8_WPE 1
#endif
template <int D, bool DIV, int NRP>
__device__ __forceinline__ void sym_fwd_pkn_body(const Args& a, const Scal& sc, int64_t M, int nG, int L,
                                                 float* __restrict__ slab, int64_t slot_stride, unsigned bx,
                                                 unsigned by) {
  using P = SymFwdPkN<D, DIV, NRP>;
  using P4 = SymFwdPk4<D, DIV>;
  using S = typename P::S;
  using LY = rec_layout<P4>;
  constexpr int G = sym_fwd_group<NRP>(), NR = 2 * NRP;
  constexpr int CW = S::CW, NP = LY::kPlanes, W = P::W;
  __shared__ float4 planes[2][NP][G];
  __shared__ float colacc[kSymQ][64][W];    // one 64-column slice of a group at a time

  const int Q = (int)by, kc = (int)bx;
  const int B0 = kSymQ * Q + kc * L;
  if (B0 >= nG) return;  // uniform for the whole workgroup, before any barrier
  const int B1 = min(B0 + L, nG);
  const int tid = threadIdx.x, wv = tid >> 6, l = tid & 63;
  const int A = kSymQ * Q + wv;

  typename P::Row2 row[NRP];
  // row r of the lane: A * G + r * 64 + l (recomputed at the stores: no index registers live
  // across the pair loop)
  const int64_t rbase = (int64_t)A * G + l;
  {
    typename S::Row rr[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int64_t ri = rbase + r * 64;
      const bool rv = A < nG && ri < M;
      S::load_row(a, sc, rv ? ri : 0, rv, rr[r]);
    }
#pragma unroll
    for (int h = 0; h < NRP; ++h) P4::pack(rr[2 * h], rr[2 * h + 1], row[h]);
  }
  f2 racc[NRP][W];
#pragma unroll
  for (int h = 0; h < NRP; ++h)
#pragma unroll
    for (int k = 0; k < W; ++k) racc[h][k] = splat(0.f);

  auto stage = [&](int B, int buf) {
#pragma unroll
    for (int u = 0; u < (G + 255) / 256; ++u) {
      const int c = u * 256 + tid;
      if (G % 256 != 0 && c >= G) break;
      const int64_t j = (int64_t)B * G + c;
      float rec[4 * CW], ph[4 * NP];
      S::load_col(a, sc, j < M ? j : 0, j < M, rec);
#pragma unroll
      for (int k = 0; k < 4 * NP; ++k) ph[k] = 0.f;
#pragma unroll
      for (int i = 0; i < S::kUsed; ++i) ph[LY::slot(i)] = rec[i];
      if constexpr (LY::kDupW) {
#pragma unroll
        for (int m = 0; m < NP; ++m) ph[4 * m + 3] = ph[4 * m + 2];
      }
#pragma unroll
      for (int m = 0; m < NP; ++m)
        planes[buf][m][c] = make_float4(ph[4 * m], ph[4 * m + 1], ph[4 * m + 2], ph[4 * m + 3]);
    }
  };
  int buf = 0;
  auto ldrec = [&](int col, float* rec) {
    float ph[4 * NP];
#pragma unroll
    for (int m = 0; m < NP; ++m) {
      const float4 v = planes[buf][m][col];
      ph[4 * m] = v.x, ph[4 * m + 1] = v.y, ph[4 * m + 2] = v.z, ph[4 * m + 3] = v.w;
    }
#pragma unroll
    for (int i = 0; i < 4 * CW; ++i) rec[i] = i < S::kUsed ? ph[LY::slot(i)] : 0.f;
#pragma unroll
    for (int m = 0; m < NP; ++m) rec[4 * CW + m] = LY::kDupW ? ph[4 * m + 3] : 0.f;
  };
  stage(B0, 0);
  __syncthreads();
  for (int B = B0; B < B1; ++B) {
    if (B + 1 < B1) stage(B + 1, buf ^ 1);
    const bool sym = A < B;          // wave-uniform
    const bool diag = A == B;
#pragma unroll 1
    for (int h = 0; h < G / 64; ++h) {   // 64-column slices of the group
      {
        float cacc[W];
#pragma unroll
        for (int k = 0; k < W; ++k) cacc[k] = 0.f;
        if (sym) {
#pragma unroll 1
          for (int k2 = 0; k2 < 64; ++k2) {
            const int col = h * 64 + ((l + k2) & 63);
            float rec[4 * CW + NP];
            ldrec(col, rec);
            float ct[W];
            P::pair_sym(row, rec, racc, ct);
#pragma unroll
            for (int k = 0; k < W; ++k) cacc[k] = rol1(cacc[k]) + ct[k];
          }
#pragma unroll
          for (int k = 0; k < W; ++k) cacc[k] = rol1(cacc[k]);
        } else if (diag) {
#pragma unroll 1
          for (int k2 = 0; k2 < 64; ++k2) {
            const int col = h * 64 + ((l + k2) & 63);
            float rec[4 * CW + NP];
            ldrec(col, rec);
#pragma unroll
            for (int r = 0; r < NRP; ++r) P::pair_row(row[r], rec, racc[r]);
          }
        }
#pragma unroll
        for (int k = 0; k < W; ++k) colacc[wv][l][k] = cacc[k];
      }
      __syncthreads();
      {
        // the slice's 64 column sums of the 4 waves, added in wave order (contiguous stores)
        const int64_t j0 = (int64_t)B * G + h * 64;
        float* dst = slab + (int64_t)Q * slot_stride + j0 * W;
        for (int e = tid; e < 64 * W; e += 256) {
          const int c = e / W, k = e - c * W;
          if (j0 + c < M) dst[e] = ((colacc[0][c][k] + colacc[1][c][k]) + colacc[2][c][k]) + colacc[3][c][k];
        }
      }
      __syncthreads();
    }
    buf ^= 1;
  }
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    const int64_t ri = rbase + r * 64;
    if (!(A < nG && ri < M)) continue;
    float* dst = slab + (int64_t)(Q + 1 + kc) * slot_stride + ri * W;
    const f2* ra = racc[r >> 1];
#pragma unroll
    for (int k = 0; k < W; ++k) dst[k] = (r & 1) == 0 ? ra[k].x : ra[k].y;
  }
}

template <int D, bool DIV, int NRP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NRP == 4 ? DICP_SYMFWD8_WPE : 3, 4))) void sym_fwd_pkn_kernel(
    Args a, Scal sc, int64_t M, int nG, int L, float* __restrict__ slab, int64_t slot_stride) {
  sym_fwd_pkn_body<D, DIV, NRP>(a, sc, M, nG, L, slab, slot_stride, blockIdx.x, blockIdx.y);
}
// one grid over the frames of a lockstep launch batch (batch.hpp), as sym_fwd_pk4_batch_kernel
template <int D, bool DIV, int NRP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NRP == 4 ? DICP_SYMFWD8_WPE : 3, 4))) void sym_fwd_pkn_batch_kernel(
    BatchTab<SymEntry> t) {
  const SymEntry& e = t.e[blockIdx.z];
  if (blockIdx.x >= e.gx || blockIdx.y >= e.gy) return;
  sym_fwd_pkn_body<D, DIV, NRP>(e.a, e.sc, e.M, e.nG, e.L, e.slab, e.slot_stride, blockIdx.x, blockIdx.y);
}
template <int D, bool DIV, int NRP>
int sym_fwd_pkn_batch_flush(const std::vector<const void*>& es, hipStream_t st) {
  return batch_launch<SymEntry>(sym_fwd_pkn_batch_kernel<D, DIV, NRP>, es, st, "sym_fwd_pkn");
}

// zs: the divergence rows out through the h slot (o.ptr[3], M x D), DIV required; the
// launcher of the 4-row form's contract (launch_sym_fwd4); NRP row pairs per lane
template <int D, bool DIV, int NRP = 4>
int launch_sym_fwdn(const Args& a, const Scal& sc, int64_t M, const Outs& o, void* ws, size_t wsb,
                    hipStream_t st, bool zs) {
  using S = SymFwd<D, DIV>;
  constexpr int G = sym_fwd_group<NRP>();
  if (M <= 0) return DICP_OK;
  const SymGeom g = sym_geom(M, 1, G, 4, NRP == 4 ? kSymFwd8WgMin : kSymFwd6WgMin);
  const size_t need = sym_ws_bytes(M, S::W);
  if (ws == nullptr || wsb < need) {
    set_error("ode_self_fwd(sym6/8): workspace too small (%zu < %zu bytes)", wsb, need);
    return DICP_ERR_WORKSPACE;
  }
  if (o.ptr[0] == nullptr || (zs && (!DIV || o.ptr[3] == nullptr))) {
    set_error("ode_self_fwd(sym6/8): v is required, zs needs the divergence sums");
    return DICP_ERR_INVALID;
  }
  float* slab = reinterpret_cast<float*>(ws);
  const int64_t stride = M * S::W;
  const dim3 grid((unsigned)g.Kmax, (unsigned)g.nQ), mg((unsigned)((M + 255) / 256));
  const float ia = 1.f / a.scale;
  if (batching()) {
    int rc = batch_record(sym_fwd_pkn_batch_flush<D, DIV, NRP>,
                          SymEntry{a, sc, M, g.nG, g.L, slab, stride, 0, 1, grid.x, grid.y});
    if (!rc) rc = check_launch("ode_self_fwd(sym6/8)");
    if (rc) return rc;
    const SymFwdMergeEntry e{slab, stride, M, g.nG, g.L, a.r1, sc.aux1, ia, o, mg.x, 1u};
    rc = zs ? batch_record(sym_fwd4_merge_batch_flush<D, DIV, true, G>, e)
            : batch_record(sym_fwd4_merge_batch_flush<D, DIV, false, G>, e);
    return rc ? rc : check_launch("ode_self_fwd(sym6/8 merge)");
  }
  sym_fwd_pkn_kernel<D, DIV, NRP><<<grid, dim3(256), 0, st>>>(a, sc, M, g.nG, g.L, slab, stride);
  int rc = check_launch("ode_self_fwd(sym6/8)");
  if (rc) return rc;
  if (zs)
    sym_fwd4_merge_kernel<D, DIV, true, G><<<mg, dim3(256), 0, st>>>(slab, stride, M, g.nG, g.L, a.r1, sc.aux1, ia, o);
  else
    sym_fwd4_merge_kernel<D, DIV, false, G><<<mg, dim3(256), 0, st>>>(slab, stride, M, g.nG, g.L, a.r1, sc.aux1, ia, o);
  return check_launch("ode_self_fwd(sym6/8 merge)");
}
template <int D, bool DIV>
int launch_sym_fwd8(const Args& a, const Scal& sc, int64_t M, const Outs& o, void* ws, size_t wsb,
                    hipStream_t st, bool zs) {
  return launch_sym_fwdn<D, DIV, 4>(a, sc, M, o, ws, wsb, st, zs);
}
template <int D, bool DIV>
int launch_sym_fwd6(const Args& a, const Scal& sc, int64_t M, const Outs& o, void* ws, size_t wsb,
                    hipStream_t st, bool zs) {
  return launch_sym_fwdn<D, DIV, 3>(a, sc, M, o, ws, wsb, st, zs);
}

template <int D, bool DIV>
__global__ __launch_bounds__(256) void sym_fwd_pk4_kernel(Args a, Scal sc, int64_t M, int nG, int L,
                                                          float* __restrict__ slab, int64_t slot_stride) {
  sym_pk4_body<SymFwdPk4<D, DIV>>(a, sc, M, nG, L, slab, slot_stride, 0, 1, blockIdx.x, blockIdx.y);
}
template <int D, bool DIV>
__global__ __launch_bounds__(256) void sym_fwd_pk4_batch_kernel(BatchTab<SymEntry> t) {
  const SymEntry& e = t.e[blockIdx.z];
  if (blockIdx.x >= e.gx || blockIdx.y >= e.gy) return;
  sym_pk4_body<SymFwdPk4<D, DIV>>(e.a, e.sc, e.M, e.nG, e.L, e.slab, e.slot_stride, 0, 1, blockIdx.x, blockIdx.y);
}
template <int D, bool DIV>
int sym_fwd_pk4_batch_flush(const std::vector<const void*>& es, hipStream_t st) {
  return batch_launch<SymEntry>(sym_fwd_pk4_batch_kernel<D, DIV>, es, st, "sym_fwd_pk4");
}

template <int D, bool DIV>
__global__ __launch_bounds__(256) void sym_fwd_pk_kernel(Args a, Scal sc, int64_t M, int nG, int L,
                                                         float* __restrict__ slab, int64_t slot_stride) {
  sym_pk_body<SymFwdPk<D, DIV>>(a, sc, M, nG, L, slab, slot_stride, 0, 1, blockIdx.x, blockIdx.y);
}

}  // namespace dicp
