// Symmetric (pair-once) VJP of the fused LDDMM ODE, eta = 0 (classic / hybrid models).
//
// The self-interaction VJP of OpOdeSelfBwd2 is a sum over ORDERED pairs (i, j) whose pair
// quantities are symmetric: K_ij = K_ji, pp, zb, zu, iap and w are equal for (i, j) and
// (j, i), while z, db, u and e = w z - u flip sign.  Evaluating every UNORDERED pair once
// and scattering it to both rows needs ~63 VALU per unordered pair instead of 2 x 49, and
// one exp instead of two ("Symmetric VJP").
//
// Work decomposition (all deterministic, no atomics):
//  * points are grouped in groups of kSymG = 128 (one wave: 64 lanes x 2 rows);
//  * a workgroup = kSymQ = 4 waves = 4 consecutive row groups A = 4Q + w ("quad" Q) and
//    a chunk of L consecutive column groups B in [4Q + k L, 4Q + (k+1) L);
//  * wave A vs group B: A < B -> every pair once ("sym" mode: row side into registers,
//    column side through a rotating accumulator); A == B -> the 128 x 128 ordered pairs,
//    row side only ("diag" mode, self pair included); A > B -> nothing (that pair of groups
//    is done by wave B of the same workgroup);
//  * column side: at step k lane l pairs its two rows with column (l + k) mod 64 of the
//    current 64-column half (per-lane LDS reads, conflict-free planes); the column's
//    running sum rides along in a register that a wave_rol:1 DPP rotation hands to the
//    lane that owns that column at the next step, so after 64 steps it has collected all
//    128 rows of the wave without any cross-lane reduction tree;
//  * the 4 waves' column sums are added in LDS in wave order and written to partial slot Q
//    of group B; each wave's row sums go to slot (Q_A + 1 + k) of its group A; a merge pass
//    adds the slots of every row in slot order and applies the Outs epilogue.
#pragma once
#include <cmath>

#include "launch.hpp"
#include "lddmm_ops.hpp"

namespace dicp {

constexpr int kSymG = 128;   // points per group (= rows of one wave)
constexpr int kSymQ = 4;     // row groups (waves) per workgroup
constexpr int kSymFwd4WgMin = 4096;   // sym_geom wg_min of the symmetric 4-row forward
constexpr int kSymFwd8WgMin = 2048;   // ... and of the 8-row forward (512-point groups)
// ... and of the 6-row forward (384-point groups, 3 workgroups per CU): L = 2 at 100k (4306
// workgroups; 3.185 ms against 3.25 for L = 4, tools/probes/symfwd_L.py)
constexpr int kSymFwd6WgMin = 4096;
// rows per lane of the symmetric forward: dicp_set_option "sym_fwd_rows" 4 or 8 forces, 0 =
// automatic (6 from DICP_SYM_FWD6_MIN_M, 8 from DICP_SYM_FWD8_MIN_M points, lddmm.hip)
inline int& sym_fwd_rows() {
  static int v = 0;
  return v;
}
// column groups per workgroup: dicp_set_option "sym_L" forces a value; 0 = automatic
inline int& sym_L() {
  static int L = 0;
  return L;
}
// padding coordinate: K = exp2(-|z|^2) = 0 against real points
constexpr float kFar = 1.0e12f;
// s_waitcnt lgkmcnt(0) with vmcnt / expcnt left at their maxima (gfx9 encoding)
constexpr int kLgkm0 = 0xC07F;
#ifndef DICP_SYM_PREFETCH
#define DICP_SYM_PREFETCH 1
#endif
#ifndef DICP_SYMBWD_WAVES
#define DICP_SYMBWD_WAVES 4
#endif
#ifndef DICP_SYMFWD_WAVES
#define DICP_SYMFWD_WAVES 8
#endif

struct SymGeom {
  int64_t M;
  int nG;     // groups
  int nQ;     // quads
  int L;      // column groups per workgroup
  int Kmax;   // chunks of quad 0
  int nslot;  // slots per row (max)
};

// L = 4 on one device (an MI355X sweep at 50k: L = 2..4 within 1%, 8 and 16 slower); a
// pair-subset launch (nparts > 1, row-split over ranks) has 1/nparts of the blocks, so L
// shrinks until a part still has >= 2048 workgroups (2 x 256 CUs x 4 resident) to fill the
// chip; smaller L = more (shorter) blocks and more partial slots.
// Lsmall: the L below the L = 8 range -- 4, or 2 for the 4-row VJP (256-point groups), whose
// adjoint steps measured 1.4-3.7% faster with L = 2 than 4 at 70k-100k (the zs / b0 steps;
// tools/probes/sym_L_rows4.py, profiles/r04_ab_sym_L_rows4_reps.jsonl), equal from 140k where
// L = 8 applies.
// wg_min: the halving below Lsmall stops once a launch has that many workgroups (2048; 4096
// for the symmetric 4-row forward, whose column groups measured best at L = 1 up to 60k,
// L = 2 at 80k, L = 4 at 100k -- profiles/r04_ab_fwd4_L_small.jsonl).
inline SymGeom sym_geom(int64_t M, int nparts = 1, int G = kSymG, int Lsmall = 4, int wg_min = 2048) {
  SymGeom g;
  g.M = M;
  g.nG = (int)((M + G - 1) / G);
  g.nQ = (g.nG + kSymQ - 1) / kSymQ;
  int L = sym_L();
  if (L <= 0) {
    // L = 8 where the chip stays full with >= 4096 workgroups (100k points: 9.6k): time
    // within 0.3% of L = 4 (r02_ab_vjp_symL_100k.json) and ~25% fewer partial slots written
    // and merged; otherwise L = Lsmall, halved until a launch has >= 2048 workgroups (the
    // workgroup targets are this call's share of the chip: batch_share, batch.hpp)
    const double sh = (double)batch_share();
    L = (double)g.nQ * g.nG / (2.0 * 8 * nparts) >= 4096.0 / sh ? 8 : Lsmall;
    if (L == 2 && Lsmall == 2 && nparts == 1 && batch_share() == 1) {
      // the 4-row VJP alone on the chip: L = 1 when L = 2's grid ends in a markedly emptier
      // last round of resident workgroups (4 per CU) -- 50k: 2401 workgroups = 2.34 rounds
      // against 4802 = 4.69 for L = 1, measured 1.66 vs 1.50 ms (profiles/r04_ab_rows4_L_50k.jsonl)
      const double cap = 4.0 * device_cus();
      auto fill = [&](int l) {
        const double r = (double)g.nQ * g.nG / (2.0 * l) / cap;
        return r / std::ceil(r);
      };
      if (fill(1) > fill(2) + 0.1) L = 1;
    }
    while (L > 1 && (double)g.nQ * g.nG / (2.0 * L * nparts) < (double)wg_min / sh) L /= 2;
  }
  g.L = L;
  g.Kmax = (g.nG + g.L - 1) / g.L;
  g.nslot = g.nQ + 1 + g.Kmax;
  return g;
}

// slots used by the rows of group T: column slots 0..Q_T, row slots Q_T+1 .. Q_T+K_{Q_T}
__host__ __device__ inline int sym_nslots(int T, int nG, int L) {
  const int Q = T / kSymQ;
  return Q + 1 + (nG - kSymQ * Q + L - 1) / L;
}

template <int D>
struct SymBwd {
  static constexpr int CW = cw4(5 * D);  // float4 planes per column record
  static constexpr int kUsed = 5 * D;    // live floats of a record
  static constexpr int W = 2 * D;        // accumulators per point: gp / s1 (D), gq / s (D)
  // occupancy cap: at <= 4 waves/SIMD the compiler keeps ~127 VGPRs and more pairs in
  // flight per wave; the 5-wave allocation (94 VGPRs) measured ~10% slower on MI355X
  static constexpr int kMaxWaves = DICP_SYMBWD_WAVES;

  struct Prm {
    float gt, c;  // gam s1 / alpha, s1 / alpha
  };
  __device__ static Prm params(const Args& a, const Scal& sc) {
    const float cs = sc.aux1 / a.scale;
    return Prm{sc.aux0 * cs, cs};
  }

  // Accumulator units: gp / alpha and gq / s (alpha = coordinate scale, s = 1/sigma^2):
  //   gp_i / alpha = sum_j K (ia_a_j - gt z) + (c K zb) p_j,   ia_a = a / alpha,
  //   gt = gam s1 / alpha, c = s1 / alpha (s1 = s / alpha), and iap = ia_a_i.p_j + ia_a_j.p_i,
  // which keeps the row state at 5 D floats (q', p, b, a / alpha, gam p).
  struct Row {
    float q[D], p[D], b[D], ia_a[D], gp[D];
  };

  __device__ static void load_row(const Args& a, const Scal& sc, int64_t i, bool valid, Row& r) {
    const float ia = 1.0f / a.scale, gam = sc.aux0;
    float c[D];
    load_shift<D>(a, c);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const float q = valid ? a.r0[i * D + d] : 0.f;
      const float p = valid ? a.r1[i * D + d] : 0.f;
      const float av = valid ? a.r2[i * D + d] : 0.f;
      const float b = valid ? a.r3[i * D + d] : 0.f;
      r.q[d] = valid ? a.scale * (q - c[d]) : kFar;
      r.p[d] = p;
      r.b[d] = b;
      r.ia_a[d] = ia * av;
      r.gp[d] = gam * p;
    }
  }

  // column record: q' (D), p (D), a / alpha (D), b (D), gam p (D)
  __device__ static void load_col(const Args& a, const Scal& sc, int64_t j, bool valid, float* rec) {
    const float ia = 1.0f / a.scale, gam = sc.aux0;
    float c[D];
    load_shift<D>(a, c);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const float q = valid ? a.c0[j * D + d] : 0.f;
      const float p = valid ? a.c1[j * D + d] : 0.f;
      const float av = valid ? a.c2[j * D + d] : 0.f;
      const float b = valid ? a.c3[j * D + d] : 0.f;
      rec[d] = valid ? a.scale * (q - c[d]) : kFar;
      rec[D + d] = p;
      rec[2 * D + d] = ia * av;
      rec[3 * D + d] = b;
      rec[4 * D + d] = gam * p;
    }
#pragma unroll
    for (int k = 5 * D; k < 4 * CW; ++k) rec[k] = 0.f;
  }

  struct Shared {
    float z[D], u[D];
    float K, w, cKzb;
  };

  // the pair quantities common to (i, j) and (j, i) (sign of z, u as seen from row i)
  __device__ static void shared_terms(float c, const Row& r, const float* rec, Shared& t) {
    float db[D];
    t.K = fast_exp2(-diff_sq<D>(r.q, rec, t.z));
    const float* pj = rec + D;
    const float* aj = rec + 2 * D;
    const float* bj = rec + 3 * D;
    const float* gpj = rec + 4 * D;
    const float pp = dot<D>(r.p, pj);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      db[d] = r.b[d] - bj[d];
      t.u[d] = fmaf(-pp, db[d], r.gp[d] - gpj[d]);
    }
    const float zu = dot<D>(t.z, t.u);
    const float zb = dot<D>(t.z, db);
    const float iap = dot<D>(r.ia_a, pj) + dot<D>(aj, r.p);
    t.w = fmaf(kS2, zu, -iap);
    t.cKzb = (c * zb) * t.K;
  }

  // ordered pair (i, j), row side only
  __device__ static void pair_row(const Prm& prm, const Row& r, const float* rec, float* acc) {
    const float gt = prm.gt;
    Shared t;
    shared_terms(prm.c, r, rec, t);
    const float* pj = rec + D;
    const float* aj = rec + 2 * D;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      acc[d] = fmaf(t.cKzb, pj[d], fmaf(t.K, fmaf(-gt, t.z[d], aj[d]), acc[d]));  // gp_i / alpha
      acc[D + d] = fmaf(t.K, fmaf(t.w, t.z[d], -t.u[d]), acc[D + d]);            // gq_i / s
    }
  }

  // unordered pair {i, j}: row side into acc, column side (the (j, i) terms) into ct
  // (FIRST: ct is initialised instead of accumulated).
  template <bool FIRST>
  __device__ static void pair_sym(const Prm& prm, const Row& r, const float* rec, float* acc,
                                  float* ct) {
    const float gt = prm.gt;
    Shared t;
    shared_terms(prm.c, r, rec, t);
    const float* pj = rec + D;
    const float* aj = rec + 2 * D;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const float e = fmaf(t.w, t.z[d], -t.u[d]);
      acc[d] = fmaf(t.cKzb, pj[d], fmaf(t.K, fmaf(-gt, t.z[d], aj[d]), acc[d]));  // gp_i / alpha
      acc[D + d] = fmaf(t.K, e, acc[D + d]);                                       // gq_i / s
      const float tt = fmaf(gt, t.z[d], r.ia_a[d]);                                // (j,i): z -> -z
      ct[d] = fmaf(t.cKzb, r.p[d], FIRST ? t.K * tt : fmaf(t.K, tt, ct[d]));       // gp_j / alpha
      ct[D + d] = FIRST ? -t.K * e : fmaf(-t.K, e, ct[D + d]);                     // gq_j / s
    }
  }
};

// Symmetric (pair-once) fused ODE forward, eta = 0 (classic / hybrid models): per point
//   V_i = sum_j K p_j,  Gs_i = sum_j K (p_i.p_j) z'_ij,  Z_i = sum_j K z'_ij  (z' = alpha z),
// the accumulators of OpOdeSelfFwd<D, false, DIV> (lddmm_ops.hpp).  K and p_i.p_j are
// symmetric, z' flips sign, so the column side of an unordered pair is
//   V_j += K p_i,  Gs_j -= K pp z',  Z_j -= K z'.
// The merge turns them into v = V, mG = (s/alpha) Gs, g = -(s/alpha) p.Z, h = p.V / 2.
template <int D, bool DIV>
struct SymFwd {
  static constexpr int kMaxWaves = DICP_SYMFWD_WAVES;
  static constexpr int CW = cw4(2 * D);
  static constexpr int kUsed = 2 * D;
  static constexpr int W = DIV ? 3 * D : 2 * D;
  struct Prm {};
  __device__ static Prm params(const Args&, const Scal&) { return Prm{}; }
  struct Row {
    float q[D], p[D];
  };
  __device__ static void load_row(const Args& a, const Scal&, int64_t i, bool valid, Row& r) {
    float c[D];
    load_shift<D>(a, c);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      r.q[d] = valid ? a.scale * (a.r0[i * D + d] - c[d]) : kFar;
      r.p[d] = valid ? a.r1[i * D + d] : 0.f;
    }
  }
  __device__ static void load_col(const Args& a, const Scal&, int64_t j, bool valid, float* rec) {
    float c[D];
    load_shift<D>(a, c);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      rec[d] = valid ? a.scale * (a.c0[j * D + d] - c[d]) : kFar;
      rec[D + d] = valid ? a.c1[j * D + d] : 0.f;
    }
#pragma unroll
    for (int k = 2 * D; k < 4 * CW; ++k) rec[k] = 0.f;
  }
  __device__ static void pair_row(const Prm&, const Row& r, const float* rec, float* acc) {
    float z[D];
    const float K = fast_exp2(-diff_sq<D>(r.q, rec, z));
    const float* pj = rec + D;
    const float Kpp = K * dot<D>(r.p, pj);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      acc[d] = fmaf(K, pj[d], acc[d]);
      acc[D + d] = fmaf(Kpp, z[d], acc[D + d]);
      if (DIV) acc[2 * D + d] = fmaf(K, z[d], acc[2 * D + d]);
    }
  }
  template <bool FIRST>
  __device__ static void pair_sym(const Prm&, const Row& r, const float* rec, float* acc, float* ct) {
    float z[D];
    const float K = fast_exp2(-diff_sq<D>(r.q, rec, z));
    const float* pj = rec + D;
    const float Kpp = K * dot<D>(r.p, pj);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      acc[d] = fmaf(K, pj[d], acc[d]);
      acc[D + d] = fmaf(Kpp, z[d], acc[D + d]);
      ct[d] = FIRST ? K * r.p[d] : fmaf(K, r.p[d], ct[d]);
      ct[D + d] = FIRST ? -Kpp * z[d] : fmaf(-Kpp, z[d], ct[D + d]);
      if (DIV) {
        acc[2 * D + d] = fmaf(K, z[d], acc[2 * D + d]);
        ct[2 * D + d] = FIRST ? -K * z[d] : fmaf(-K, z[d], ct[2 * D + d]);
      }
    }
  }
};

// Symmetric (pair-once) VJP with gradcomponent (eta != 0, the "logdet" model, e.g. the
// exact ICP_two_set model): the pair algebra of OpOdeSelfBwdEta (lddmm_ops.hpp).  Under
// (m, j) -> (j, m): z, da, db, dp flip sign; r2, pp, ap, zb, zp, za, bp, Phi and the
// coefficients cz_p, cz_q, cdb are symmetric.  Hence per unordered pair
//   gp_m += K a_j + K s zb p_j + T,   gp_j += K a_m + K s zb p_m - T,  T = K (cz_p z - es db)
//   gq_m += G,                         gq_j -= G,   G = K (es da + cdb db + (es2 zb - gs) dp + cz_q z)
// Accumulators: [gp (D), gq (D)] unscaled (merge with s = alpha = 1).
// Padding points sit at kFarEta = 1e4 (not 1e12): the eta algebra multiplies up to ~|z|^4 s^3
// before the factor K = 0 is applied, which must stay finite (0 * inf = NaN); K = exp2(nc r2)
// underflows to 0 at r2 ~ 3e8 for any sigma < ~1e3.
constexpr float kFarEta = 1.0e4f;
template <int D>
struct SymBwdEta {
  static constexpr int kMaxWaves = 8;
  static constexpr int CW = cw4(4 * D);
  static constexpr int kUsed = 4 * D;
  static constexpr int W = 2 * D;
  struct Prm {
    float nc, s, es, es2, e2s2, gs, gam;
  };
  __device__ static Prm params(const Args&, const Scal& sc) {
    const float es = sc.eta * sc.s, es2 = es * sc.s;
    return Prm{sc.nc, sc.s, es, es2, sc.eta * es2, sc.aux0 * sc.s, sc.aux0};
  }
  struct Row {
    float q[D], p[D], a[D], b[D];
  };
  __device__ static void load_row(const Args& a, const Scal&, int64_t i, bool valid, Row& r) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      r.q[d] = valid ? a.r0[i * D + d] : kFarEta;
      r.p[d] = valid ? a.r1[i * D + d] : 0.f;
      r.a[d] = valid ? a.r2[i * D + d] : 0.f;
      r.b[d] = valid ? a.r3[i * D + d] : 0.f;
    }
  }
  __device__ static void load_col(const Args& a, const Scal&, int64_t j, bool valid, float* rec) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      rec[d] = valid ? a.c0[j * D + d] : kFarEta;
      rec[D + d] = valid ? a.c1[j * D + d] : 0.f;
      rec[2 * D + d] = valid ? a.c2[j * D + d] : 0.f;
      rec[3 * D + d] = valid ? a.c3[j * D + d] : 0.f;
    }
#pragma unroll
    for (int k = 4 * D; k < 4 * CW; ++k) rec[k] = 0.f;
  }
  struct Shared {
    float z[D], db[D], da[D], dp[D];
    float K, szbK, czp, es_db_c;  // K, K s zb
    float cdb, cdp, czq;
  };
  __device__ static void shared_terms(const Prm& P, const Row& r, const float* rec, Shared& t) {
    const float* pj = rec + D;
    const float* aj = rec + 2 * D;
    const float* bj = rec + 3 * D;
    float r2 = 0.f;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      t.z[d] = r.q[d] - rec[d];
      r2 = fmaf(t.z[d], t.z[d], r2);
      t.da[d] = r.a[d] - aj[d];
      t.db[d] = r.b[d] - bj[d];
      t.dp[d] = r.p[d] - pj[d];
    }
    t.K = fast_exp2(P.nc * r2);
    const float pp = dot<D>(r.p, pj);
    const float ap = dot<D>(r.a, pj) + dot<D>(aj, r.p);
    const float zb = dot<D>(t.z, t.db), zp = dot<D>(t.z, t.dp), za = dot<D>(t.z, t.da);
    const float bp = dot<D>(t.db, t.dp);
    const float sr2 = P.s * r2;
    const float Phi = ap + P.es * za + P.s * pp * zb + P.es * (P.s * zp * zb - bp) -
                      P.e2s2 * zb * (sr2 - (float)(D + 2)) - P.gs * zp +
                      2.f * P.gam * P.es * (sr2 - (float)D);
    t.czp = P.s * zb * P.es - P.gs;
    t.czq = -2.f * P.e2s2 * P.s * zb + 4.f * P.gam * P.es2 - P.s * Phi;
    t.cdb = P.s * pp + P.es2 * zp - P.e2s2 * (sr2 - (float)(D + 2));
    t.cdp = P.es2 * zb - P.gs;
    t.szbK = P.s * zb * t.K;
  }
  // ordered pair (m, j), row side only (diag blocks, self pair included)
  __device__ static void pair_row(const Prm& P, const Row& r, const float* rec, float* acc) {
    Shared t;
    shared_terms(P, r, rec, t);
    const float* pj = rec + D;
    const float* aj = rec + 2 * D;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const float Tv = fmaf(t.czp, t.z[d], -P.es * t.db[d]);
      acc[d] = fmaf(t.K, aj[d] + Tv, fmaf(t.szbK, pj[d], acc[d]));
      const float G = fmaf(P.es, t.da[d], fmaf(t.cdb, t.db[d], fmaf(t.cdp, t.dp[d], t.czq * t.z[d])));
      acc[D + d] = fmaf(t.K, G, acc[D + d]);
    }
  }
  template <bool FIRST>
  __device__ static void pair_sym(const Prm& P, const Row& r, const float* rec, float* acc, float* ct) {
    Shared t;
    shared_terms(P, r, rec, t);
    const float* pj = rec + D;
    const float* aj = rec + 2 * D;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const float Tv = fmaf(t.czp, t.z[d], -P.es * t.db[d]);
      const float G = t.K * fmaf(P.es, t.da[d], fmaf(t.cdb, t.db[d], fmaf(t.cdp, t.dp[d], t.czq * t.z[d])));
      acc[d] = fmaf(t.K, aj[d] + Tv, fmaf(t.szbK, pj[d], acc[d]));
      acc[D + d] += G;
      const float cgp = fmaf(t.K, r.a[d] - Tv, t.szbK * r.p[d]);
      ct[d] = FIRST ? cgp : ct[d] + cgp;
      ct[D + d] = FIRST ? -G : ct[D + d] - G;
    }
  }
};

__device__ __forceinline__ float rol1(float x) {
  // wave_rol:1 -- lane l receives lane (l + 1) mod 64
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x134, 0xF, 0xF, false));
}

// slab layout: slab[slot][row][W]
// The VJP keeps its own kernel body (the generic sym_kernel below compiles the SAME pair
// algebra into a schedule measured ~12% slower on MI355X: the hipcc schedule of this loop is
// sensitive to the surrounding code, so this instance is kept as first tuned).
template <int D>
__global__ __launch_bounds__(256) void sym_bwd_kernel(Args a, Scal sc, int64_t M, int nG, int L,
                                                      float* __restrict__ slab, int64_t slot_stride,
                                                      int qoff, int qstride) {
  using S = SymBwd<D>;
  constexpr int CW = S::CW, W = S::W;
  __shared__ float4 planes[2][CW][kSymG];
  __shared__ float colacc[kSymQ][kSymG][W];
  if (sc.dev0 != nullptr) sc.aux0 = sc.dev0[0];
  const float cs = sc.aux1 / a.scale;    // s1 / alpha
  const float gt = sc.aux0 * cs;         // gam s1 / alpha
  const typename S::Prm prm{gt, cs};

  const int Q = qoff + qstride * (int)blockIdx.y, kc = blockIdx.x;
  const int B0 = kSymQ * Q + kc * L;
  if (B0 >= nG) return;  // uniform for the whole workgroup, before any barrier
  const int B1 = min(B0 + L, nG);
  const int tid = threadIdx.x, wv = tid >> 6, l = tid & 63;
  const int A = kSymQ * Q + wv;

  typename S::Row row[2];
  int64_t ri[2];
  bool rv[2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    ri[r] = (int64_t)A * kSymG + r * 64 + l;
    rv[r] = A < nG && ri[r] < M;
    S::load_row(a, sc, rv[r] ? ri[r] : 0, rv[r], row[r]);
  }
  float racc[2][W];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int k = 0; k < W; ++k) racc[r][k] = 0.f;

  auto stage = [&](int B, int buf) {
    if (tid < kSymG) {
      const int64_t j = (int64_t)B * kSymG + tid;
      float rec[4 * CW];
      S::load_col(a, sc, j < M ? j : 0, j < M, rec);
#pragma unroll
      for (int m = 0; m < CW; ++m)
        planes[buf][m][tid] = make_float4(rec[4 * m], rec[4 * m + 1], rec[4 * m + 2], rec[4 * m + 3]);
    }
  };

  int buf = 0;
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
#pragma unroll 2
        for (int k2 = 0; k2 < 64; ++k2) {
          const int col = h * 64 + ((l + k2) & 63);
          float rec[4 * CW];
#pragma unroll
          for (int m = 0; m < CW; ++m) {
            const float4 v = planes[buf][m][col];
            rec[4 * m] = v.x;
            rec[4 * m + 1] = v.y;
            rec[4 * m + 2] = v.z;
            rec[4 * m + 3] = v.w;
          }
          float ct[W];
          S::template pair_sym<true>(prm, row[0], rec, racc[0], ct);
          S::template pair_sym<false>(prm, row[1], rec, racc[1], ct);
          // cacc belonged to column (l + k2 - 1); bring column (l + k2)'s sum to this lane
#pragma unroll
          for (int k = 0; k < W; ++k) cacc[k] = rol1(cacc[k]) + ct[k];
        }
        // lane l holds column (l + 63) & 63; one more rotation aligns lane l with column l
#pragma unroll
        for (int k = 0; k < W; ++k) cacc[k] = rol1(cacc[k]);
      } else if (diag) {
#pragma unroll 2
        for (int k2 = 0; k2 < 64; ++k2) {
          const int col = h * 64 + ((l + k2) & 63);
          float rec[4 * CW];
#pragma unroll
          for (int m = 0; m < CW; ++m) {
            const float4 v = planes[buf][m][col];
            rec[4 * m] = v.x;
            rec[4 * m + 1] = v.y;
            rec[4 * m + 2] = v.z;
            rec[4 * m + 3] = v.w;
          }
          S::pair_row(prm, row[0], rec, racc[0]);
          S::pair_row(prm, row[1], rec, racc[1]);
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
  // row sums of this workgroup's column chunk -> slot Q + 1 + kc of group A
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    if (!rv[r]) continue;
    float* dst = slab + (int64_t)(Q + 1 + kc) * slot_stride + ri[r] * W;
#pragma unroll
    for (int k = 0; k < W; ++k) dst[k] = racc[r][k];
  }
}

template <class S>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, S::kMaxWaves))) void sym_kernel(Args a, Scal sc, int64_t M, int nG, int L,
                                                  float* __restrict__ slab, int64_t slot_stride) {
  constexpr int CW = S::CW, W = S::W;
  __shared__ float4 planes[2][CW][kSymG];
  __shared__ float colacc[kSymQ][kSymG][W];
  if (sc.dev0 != nullptr) sc.aux0 = sc.dev0[0];
  const typename S::Prm prm = S::params(a, sc);

  const int Q = blockIdx.y, kc = blockIdx.x;
  const int B0 = kSymQ * Q + kc * L;
  if (B0 >= nG) return;  // uniform for the whole workgroup, before any barrier
  const int B1 = min(B0 + L, nG);
  const int tid = threadIdx.x, wv = tid >> 6, l = tid & 63;
  const int A = kSymQ * Q + wv;

  typename S::Row row[2];
  int64_t ri[2];
  bool rv[2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    ri[r] = (int64_t)A * kSymG + r * 64 + l;
    rv[r] = A < nG && ri[r] < M;
    S::load_row(a, sc, rv[r] ? ri[r] : 0, rv[r], row[r]);
  }
  float racc[2][W];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int k = 0; k < W; ++k) racc[r][k] = 0.f;

  auto stage = [&](int B, int buf) {
    if (tid < kSymG) {
      const int64_t j = (int64_t)B * kSymG + tid;
      float rec[4 * CW];
      S::load_col(a, sc, j < M ? j : 0, j < M, rec);
#pragma unroll
      for (int m = 0; m < CW; ++m)
        planes[buf][m][tid] = make_float4(rec[4 * m], rec[4 * m + 1], rec[4 * m + 2], rec[4 * m + 3]);
    }
  };

  int buf = 0;
  // read a column record; only the S::kUsed live floats (a dead padding lane read into a
  // register would be a WAW hazard the waitcnt pass resolves by waiting on the read)
  auto ldrec = [&](int col, float* rec) {
    constexpr int kLast = S::kUsed - 4 * (CW - 1);  // live floats of the last plane (1..4)
#pragma unroll
    for (int m = 0; m < CW; ++m) {
      const float* src = reinterpret_cast<const float*>(&planes[buf][m][col]);
      if (m < CW - 1 || kLast == 4) {
        const float4 v = *reinterpret_cast<const float4*>(src);
        rec[4 * m] = v.x, rec[4 * m + 1] = v.y, rec[4 * m + 2] = v.z, rec[4 * m + 3] = v.w;
      } else if (kLast == 3) {
        const float3 v = *reinterpret_cast<const float3*>(src);
        rec[4 * m] = v.x, rec[4 * m + 1] = v.y, rec[4 * m + 2] = v.z, rec[4 * m + 3] = 0.f;
      } else if (kLast == 2) {
        const float2 v = *reinterpret_cast<const float2*>(src);
        rec[4 * m] = v.x, rec[4 * m + 1] = v.y, rec[4 * m + 2] = rec[4 * m + 3] = 0.f;
      } else {
        rec[4 * m] = src[0], rec[4 * m + 1] = rec[4 * m + 2] = rec[4 * m + 3] = 0.f;
      }
    }
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
#if DICP_SYM_PREFETCH
        // register double-buffer: the record of step k2 + 1 is read from LDS while step k2
        // computes, so the LDS latency is not exposed once per step (the compiler's own
        // schedule varies between builds: waits right after the reads cost ~13% on the VJP)
        float rec[4 * CW];
        ldrec(h * 64 + (l & 63), rec);
#pragma unroll 2
        for (int k2 = 0; k2 < 64; ++k2) {
          float nxt[4 * CW];
          // this step's record was read one step ago: wait for it here (no stall), then
          // issue the next reads and pin them at the top (the compiler otherwise sinks
          // them next to their use and waits on them right away)
          __builtin_amdgcn_s_waitcnt(kLgkm0);
          ldrec(h * 64 + ((l + k2 + 1) & 63), nxt);  // k2 = 63 wraps to column l: harmless
          __builtin_amdgcn_sched_barrier(0);
          float ct[W];
          S::template pair_sym<true>(prm, row[0], rec, racc[0], ct);
          S::template pair_sym<false>(prm, row[1], rec, racc[1], ct);
#pragma unroll
          for (int k = 0; k < W; ++k) cacc[k] = rol1(cacc[k]) + ct[k];
#pragma unroll
          for (int k = 0; k < 4 * CW; ++k) rec[k] = nxt[k];
        }
#else
#pragma unroll 2
        for (int k2 = 0; k2 < 64; ++k2) {
          const int col = h * 64 + ((l + k2) & 63);
          float rec[4 * CW];
          ldrec(col, rec);
          float ct[W];
          S::template pair_sym<true>(prm, row[0], rec, racc[0], ct);
          S::template pair_sym<false>(prm, row[1], rec, racc[1], ct);
          // cacc belonged to column (l + k2 - 1); bring column (l + k2)'s sum to this lane
#pragma unroll
          for (int k = 0; k < W; ++k) cacc[k] = rol1(cacc[k]) + ct[k];
        }
#endif
        // lane l holds column (l + 63) & 63; one more rotation aligns lane l with column l
#pragma unroll
        for (int k = 0; k < W; ++k) cacc[k] = rol1(cacc[k]);
      } else if (diag) {
#pragma unroll 2
        for (int k2 = 0; k2 < 64; ++k2) {
          const int col = h * 64 + ((l + k2) & 63);
          float rec[4 * CW];
#pragma unroll
          for (int m = 0; m < CW; ++m) {
            const float4 v = planes[buf][m][col];
            rec[4 * m] = v.x;
            rec[4 * m + 1] = v.y;
            rec[4 * m + 2] = v.z;
            rec[4 * m + 3] = v.w;
          }
          S::pair_row(prm, row[0], rec, racc[0]);
          S::pair_row(prm, row[1], rec, racc[1]);
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
  // row sums of this workgroup's column chunk -> slot Q + 1 + kc of group A
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    if (!rv[r]) continue;
    float* dst = slab + (int64_t)(Q + 1 + kc) * slot_stride + ri[r] * W;
#pragma unroll
    for (int k = 0; k < W; ++k) dst[k] = racc[r][k];
  }
}

// out0 = gq = s * sum(gq/s), out1 = gp = alpha * sum(gp/alpha), with the Outs epilogue.
// Pair-subset mode (row-split over ranks): only the quads Q = qoff (mod qstride) ran, so a
// row of quad Q_T sums its column slots Q <= Q_T of those quads and, if Q_T is one of them,
// its row slots; (qoff, qstride) = (0, 1) is every slot in slot order.
// W = 2D: [gp, gq] channels; W = D: gp only (the gp-only VJP, sym_bwd_pk_kernel<D, false>).
// Null output pointers are skipped (a caller that needs only gp).
// zs (rows [zr0, zr0 + zn), original units): the forward's divergence rows; the VJP kernel then
// ran without the divergence cotangent's pair terms (SymBwdPk<., ., ., false>) and their row
// total, -gam s zs_i (gam = *gdiv), is added here, once per row (row split: by the rank that
// owns the row's forward slice).
template <int D, bool kPart, int W = 2 * D, int G = kSymG>
__device__ __forceinline__ void sym_merge_body(const float* __restrict__ slab, int64_t slot_stride, int64_t M,
                                               int nG, int L, float s, float alpha, const Outs& o, int qoff,
                                               int qstride, const float* __restrict__ zs, int64_t zr0, int64_t zn,
                                               const float* __restrict__ gdiv, unsigned bx) {
  const int64_t e = (int64_t)bx * 256 + threadIdx.x;
  if (e >= M * W) return;
  const int64_t row = e / W;
  const int c = (int)(e - row * W);
  const int T = (int)(row / G);
  const int ns = sym_nslots(T, nG, L);
  float acc;
  if constexpr (!kPart) {
    acc = slab[e];
    // slots in order; the loads of 8 slots are issued together (one dependent load per add
    // left the merge latency-bound at ~2.4 TB/s), the additions stay sequential
    int t = 1;
    for (; t + 8 <= ns; t += 8) {
      float v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = slab[(int64_t)(t + k) * slot_stride + e];
#pragma unroll
      for (int k = 0; k < 8; ++k) acc += v[k];
    }
    for (; t < ns; ++t) acc += slab[(int64_t)t * slot_stride + e];
  } else {
    const int QT = T / kSymQ;
    acc = 0.f;
    for (int q = qoff; q <= QT; q += qstride) acc += slab[(int64_t)q * slot_stride + e];
    if (QT >= qoff && (QT - qoff) % qstride == 0) {
      int t = QT + 1;
      for (; t + 8 <= ns; t += 8) {
        float v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = slab[(int64_t)(t + k) * slot_stride + e];
#pragma unroll
        for (int k = 0; k < 8; ++k) acc += v[k];
      }
      for (; t < ns; ++t) acc += slab[(int64_t)t * slot_stride + e];
    }
  }
  if (c < D) {
    const int64_t idx = row * D + c;
    float gp = alpha * acc;
    if (zs != nullptr && row >= zr0 && row < zr0 + zn && gdiv != nullptr)
      gp = fmaf(-s * gdiv[0], zs[(row - zr0) * D + c], gp);
    if (o.ptr[1]) o.ptr[1][idx] = epilogue(o, 1, idx, gp);
  } else {
    const int64_t idx = row * D + (c - D);
    if (o.ptr[0]) o.ptr[0][idx] = epilogue(o, 0, idx, s * acc);
  }
}

template <int D, bool kPart, int W = 2 * D, int G = kSymG>
__global__ __launch_bounds__(256) void sym_merge_kernel(const float* __restrict__ slab,
                                                        int64_t slot_stride, int64_t M, int nG,
                                                        int L, float s, float alpha, Outs o,
                                                        int qoff, int qstride,
                                                        const float* __restrict__ zs = nullptr,
                                                        int64_t zr0 = 0, int64_t zn = 0,
                                                        const float* __restrict__ gdiv = nullptr) {
  sym_merge_body<D, kPart, W, G>(slab, slot_stride, M, nG, L, s, alpha, o, qoff, qstride, zs, zr0, zn, gdiv,
                                 blockIdx.x);
}

// batched forms (batch.hpp): blockIdx.z = the recorded call
struct SymMergeEntry {
  const float* slab;
  int64_t slot_stride, M;
  int nG, L;
  float s, alpha;
  Outs o;
  int qoff, qstride;
  const float* zs;
  int64_t zr0, zn;
  const float* gdiv;
  unsigned gx, gy;
};
template <int D, bool kPart, int W, int G>
__global__ __launch_bounds__(256) void sym_merge_batch_kernel(BatchTab<SymMergeEntry> t) {
  const SymMergeEntry& e = t.e[blockIdx.z];
  if (blockIdx.x >= e.gx) return;
  sym_merge_body<D, kPart, W, G>(e.slab, e.slot_stride, e.M, e.nG, e.L, e.s, e.alpha, e.o, e.qoff, e.qstride, e.zs,
                                 e.zr0, e.zn, e.gdiv, blockIdx.x);
}
template <int D, bool kPart, int W, int G>
int sym_merge_batch_flush(const std::vector<const void*>& es, hipStream_t st) {
  return batch_launch<SymMergeEntry>(sym_merge_batch_kernel<D, kPart, W, G>, es, st, "sym_merge");
}
// launch (or record, inside a batch) one symmetric-VJP merge
template <int D, bool kPart, int W = 2 * D, int G = kSymG>
void sym_merge_launch(dim3 grid, hipStream_t st, const float* slab, int64_t slot_stride, int64_t M, int nG, int L,
                      float s, float alpha, const Outs& o, int qoff, int qstride, const float* zs, int64_t zr0,
                      int64_t zn, const float* gdiv) {
  if (batching()) {
    batch_record(sym_merge_batch_flush<D, kPart, W, G>,
                 SymMergeEntry{slab, slot_stride, M, nG, L, s, alpha, o, qoff, qstride, zs, zr0, zn, gdiv, grid.x, 1u});
    return;
  }
  sym_merge_kernel<D, kPart, W, G><<<grid, dim3(256), 0, st>>>(slab, slot_stride, M, nG, L, s, alpha, o, qoff,
                                                              qstride, zs, zr0, zn, gdiv);
}

// argument entry of a batched symmetric pair kernel (lddmm_sym_pk.hpp sym_bwd_pk(4)_batch_kernel)
struct SymEntry {
  Args a;
  Scal sc;
  int64_t M;
  int nG, L;
  float* slab;
  int64_t slot_stride;
  int qoff, qstride;
  unsigned gx, gy;
};

// W = accumulators per point (SymBwd: 2D, SymFwd: 3D with the divergence, else 2D)
inline size_t sym_ws_bytes(int64_t M, int W, int nparts = 1) {
  if (M <= 0) return 0;
  // 128 / 256-point groups (the 4-row VJP's smaller L: more row slots), 512-point groups (the
  // 8-row forward)
  const SymGeom g = sym_geom(M, nparts), g4 = sym_geom(M, nparts, 256), g4v = sym_geom(M, nparts, 256, 2),
                g4f = sym_geom(M, nparts, 256, 4, kSymFwd4WgMin),
                g8f = sym_geom(M, nparts, 512, 4, kSymFwd8WgMin),
                g6f = sym_geom(M, nparts, 384, 4, kSymFwd6WgMin);
  int ns = g.nslot > g4.nslot ? g.nslot : g4.nslot;
  ns = g4v.nslot > ns ? g4v.nslot : ns;
  ns = g4f.nslot > ns ? g4f.nslot : ns;
  ns = g8f.nslot > ns ? g8f.nslot : ns;
  ns = g6f.nslot > ns ? g6f.nslot : ns;
  return (size_t)ns * (size_t)M * (size_t)W * sizeof(float);
}

// Forward merge: one thread per row sums its slots (slot order) and applies the epilogue to
// v = V, mG = sa Gs, g = -sa p.Z, h = p.V / 2 (null outputs skipped).
template <int D, bool DIV>
__global__ __launch_bounds__(256) void sym_fwd_merge_kernel(const float* __restrict__ slab,
                                                            int64_t slot_stride, int64_t M, int nG,
                                                            int L, const float* __restrict__ p,
                                                            float sa, Outs o) {
  constexpr int W = SymFwd<D, DIV>::W;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= M) return;
  const int ns = sym_nslots((int)(i / kSymG), nG, L);
  float t[W];
  const float* src = slab + i * W;
#pragma unroll
  for (int k = 0; k < W; ++k) t[k] = src[k];
  for (int u = 1; u < ns; ++u) {
    const float* s2 = src + (int64_t)u * slot_stride;
#pragma unroll
    for (int k = 0; k < W; ++k) t[k] += s2[k];
  }
  float pv = 0.f, pz = 0.f;
#pragma unroll
  for (int d = 0; d < D; ++d) {
    const float pd = p[i * D + d];
    pv = fmaf(pd, t[d], pv);
    if (DIV) pz = fmaf(pd, t[2 * D + d], pz);
    o.ptr[0][i * D + d] = epilogue(o, 0, i * D + d, t[d]);
    o.ptr[1][i * D + d] = epilogue(o, 1, i * D + d, sa * t[D + d]);
  }
  if (o.ptr[2]) o.ptr[2][i] = epilogue(o, 2, i, DIV ? -sa * pz : 0.f);
  if (o.ptr[3]) o.ptr[3][i] = epilogue(o, 3, i, 0.5f * pv);
}

// packed-FP32 variant of the symmetric forward (lddmm_sym_pk.hpp)
template <int D, bool DIV>
__global__ void sym_fwd_pk_kernel(Args a, Scal sc, int64_t M, int nG, int L, float* __restrict__ slab,
                                  int64_t slot_stride);

template <int D, bool DIV>
int launch_sym_fwd(const Args& a, const Scal& sc, int64_t M, const Outs& o, void* ws, size_t wsb,
                   hipStream_t st, bool pk = false) {
  if (int rc = no_batch("ode_self_fwd(sym)")) return rc;
  using S = SymFwd<D, DIV>;
  if (M <= 0) return DICP_OK;
  const SymGeom g = sym_geom(M);
  const size_t need = sym_ws_bytes(M, S::W);
  if (ws == nullptr || wsb < need) {
    set_error("ode_self_fwd(sym): workspace too small (%zu < %zu bytes)", wsb, need);
    return DICP_ERR_WORKSPACE;
  }
  if (o.ptr[0] == nullptr || o.ptr[1] == nullptr) {
    set_error("ode_self_fwd(sym): v and mG outputs are required");
    return DICP_ERR_INVALID;
  }
  float* slab = reinterpret_cast<float*>(ws);
  const int64_t stride = M * S::W;
  if (pk)
    sym_fwd_pk_kernel<D, DIV><<<dim3((unsigned)g.Kmax, (unsigned)g.nQ), dim3(256), 0, st>>>(
        a, sc, M, g.nG, g.L, slab, stride);
  else
    sym_kernel<S><<<dim3((unsigned)g.Kmax, (unsigned)g.nQ), dim3(256), 0, st>>>(a, sc, M, g.nG, g.L,
                                                                                slab, stride);
  int rc = check_launch("ode_self_fwd(sym)");
  if (rc) return rc;
  sym_fwd_merge_kernel<D, DIV><<<dim3((unsigned)((M + 255) / 256)), dim3(256), 0, st>>>(
      slab, stride, M, g.nG, g.L, a.r1, sc.aux1, o);
  return check_launch("ode_self_fwd(sym merge)");
}

// ---- the symmetric forward with 4 rows per lane (fwd_alg 5, lddmm_sym_pk.hpp SymFwdPk4) ----
// Merge: one thread per row sums its slots in slot order (8 loads in flight, the additions
// sequential) and applies the epilogue to v = V, mG = sa Gs, g = -sa p.Z and either h = p.V / 2
// or (ZS) the divergence rows zs = Z' / alpha (original units, as OpOdeSelfFwdZs) in the h slot.
template <int D, bool DIV, bool ZS, int G = 256>
__device__ __forceinline__ void sym_fwd4_merge_body(const float* __restrict__ slab, int64_t slot_stride,
                                                    int64_t M, int nG, int L, const float* __restrict__ p,
                                                    float sa, float ia, const Outs& o, unsigned bx) {
  constexpr int W = SymFwd<D, DIV>::W;
  const int64_t i = (int64_t)bx * 256 + threadIdx.x;
  if (i >= M) return;
  const int ns = sym_nslots((int)(i / G), nG, L);
  float t[W];
  const float* src = slab + i * W;
#pragma unroll
  for (int k = 0; k < W; ++k) t[k] = src[k];
  int u = 1;
  for (; u + 4 <= ns; u += 4) {
    float v[4][W];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int k = 0; k < W; ++k) v[c][k] = src[(int64_t)(u + c) * slot_stride + k];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int k = 0; k < W; ++k) t[k] += v[c][k];
  }
  for (; u < ns; ++u) {
#pragma unroll
    for (int k = 0; k < W; ++k) t[k] += src[(int64_t)u * slot_stride + k];
  }
  float pv = 0.f, pz = 0.f;
#pragma unroll
  for (int d = 0; d < D; ++d) {
    const float pd = p[i * D + d];
    pv = fmaf(pd, t[d], pv);
    if (DIV) pz = fmaf(pd, t[2 * D + d], pz);
    o.ptr[0][i * D + d] = epilogue(o, 0, i * D + d, t[d]);
    if (o.ptr[1]) o.ptr[1][i * D + d] = epilogue(o, 1, i * D + d, sa * t[D + d]);
    if (ZS) o.ptr[3][i * D + d] = ia * t[2 * D + d];
  }
  if (o.ptr[2]) o.ptr[2][i] = epilogue(o, 2, i, DIV ? -sa * pz : 0.f);
  if (!ZS && o.ptr[3]) o.ptr[3][i] = epilogue(o, 3, i, 0.5f * pv);
}
template <int D, bool DIV, bool ZS, int G = 256>
__global__ __launch_bounds__(256) void sym_fwd4_merge_kernel(const float* __restrict__ slab, int64_t slot_stride,
                                                             int64_t M, int nG, int L, const float* __restrict__ p,
                                                             float sa, float ia, Outs o) {
  sym_fwd4_merge_body<D, DIV, ZS, G>(slab, slot_stride, M, nG, L, p, sa, ia, o, blockIdx.x);
}
struct SymFwdMergeEntry {
  const float* slab;
  int64_t slot_stride, M;
  int nG, L;
  const float* p;
  float sa, ia;
  Outs o;
  unsigned gx, gy;
};
template <int D, bool DIV, bool ZS, int G = 256>
__global__ __launch_bounds__(256) void sym_fwd4_merge_batch_kernel(BatchTab<SymFwdMergeEntry> t) {
  const SymFwdMergeEntry& e = t.e[blockIdx.z];
  if (blockIdx.x >= e.gx) return;
  sym_fwd4_merge_body<D, DIV, ZS, G>(e.slab, e.slot_stride, e.M, e.nG, e.L, e.p, e.sa, e.ia, e.o, blockIdx.x);
}
template <int D, bool DIV, bool ZS, int G = 256>
int sym_fwd4_merge_batch_flush(const std::vector<const void*>& es, hipStream_t st) {
  return batch_launch<SymFwdMergeEntry>(sym_fwd4_merge_batch_kernel<D, DIV, ZS, G>, es, st, "sym_fwd4_merge");
}

template <int D, bool DIV>
__global__ void sym_fwd_pk4_kernel(Args a, Scal sc, int64_t M, int nG, int L, float* __restrict__ slab,
                                   int64_t slot_stride);
template <int D, bool DIV>
int sym_fwd_pk4_batch_flush(const std::vector<const void*>& es, hipStream_t st);

// zs: the divergence rows out through the h slot (o.ptr[3], M x D), DIV required
template <int D, bool DIV>
int launch_sym_fwd4(const Args& a, const Scal& sc, int64_t M, const Outs& o, void* ws, size_t wsb,
                    hipStream_t st, bool zs) {
  using S = SymFwd<D, DIV>;
  if (M <= 0) return DICP_OK;
  const SymGeom g = sym_geom(M, 1, 256, 4, kSymFwd4WgMin);
  const size_t need = sym_ws_bytes(M, S::W);
  if (ws == nullptr || wsb < need) {
    set_error("ode_self_fwd(sym4): workspace too small (%zu < %zu bytes)", wsb, need);
    return DICP_ERR_WORKSPACE;
  }
  if (o.ptr[0] == nullptr || (zs && (!DIV || o.ptr[3] == nullptr))) {
    set_error("ode_self_fwd(sym4): v is required, zs needs the divergence sums");
    return DICP_ERR_INVALID;
  }
  float* slab = reinterpret_cast<float*>(ws);
  const int64_t stride = M * S::W;
  const dim3 grid((unsigned)g.Kmax, (unsigned)g.nQ), mg((unsigned)((M + 255) / 256));
  const float ia = 1.f / a.scale;
  if (batching()) {
    int rc = batch_record(sym_fwd_pk4_batch_flush<D, DIV>,
                          SymEntry{a, sc, M, g.nG, g.L, slab, stride, 0, 1, grid.x, grid.y});
    if (!rc) rc = check_launch("ode_self_fwd(sym4)");
    if (rc) return rc;
    const SymFwdMergeEntry e{slab, stride, M, g.nG, g.L, a.r1, sc.aux1, ia, o, mg.x, 1u};
    rc = zs ? batch_record(sym_fwd4_merge_batch_flush<D, DIV, true>, e)
            : batch_record(sym_fwd4_merge_batch_flush<D, DIV, false>, e);
    return rc ? rc : check_launch("ode_self_fwd(sym4 merge)");
  }
  sym_fwd_pk4_kernel<D, DIV><<<grid, dim3(256), 0, st>>>(a, sc, M, g.nG, g.L, slab, stride);
  int rc = check_launch("ode_self_fwd(sym4)");
  if (rc) return rc;
  if (zs)
    sym_fwd4_merge_kernel<D, DIV, true><<<mg, dim3(256), 0, st>>>(slab, stride, M, g.nG, g.L, a.r1, sc.aux1, ia, o);
  else
    sym_fwd4_merge_kernel<D, DIV, false><<<mg, dim3(256), 0, st>>>(slab, stride, M, g.nG, g.L, a.r1, sc.aux1, ia, o);
  return check_launch("ode_self_fwd(sym4 merge)");
}

// packed-FP32 rows of the eta != 0 VJP (lddmm_sym_pk.hpp); GQ = false: gp half only, B0: zero
// cotangent on mG
template <int D, bool GQ, bool B0>
__global__ void sym_bwd_eta_pk_kernel(Args a, Scal sc, int64_t M, int nG, int L, float* __restrict__ slab,
                                      int64_t slot_stride, int qoff, int qstride);

// b0: the cotangent on mG (Args r3 / c3) is identically zero and is not read (packed kernel
// only); o.ptr[0] == NULL with the packed kernel: the gq half is never evaluated
template <int D>
int launch_sym_bwd_eta(const Args& a, const Scal& sc, int64_t M, const Outs& o, void* ws,
                       size_t wsb, hipStream_t st, bool pk = false, int part = 0, int nparts = 1,
                       bool b0 = false) {
  if (int rc = no_batch("ode_self_bwd(sym eta)")) return rc;
  using S = SymBwdEta<D>;
  if (M <= 0) return DICP_OK;
  if ((nparts > 1 || b0) && !pk) {
    set_error("ode_self_bwd(sym eta): pair-subset parts and a zero mG cotangent need the packed "
              "kernel (bwd_eta_alg 2)");
    return DICP_ERR_INVALID;
  }
  const SymGeom g = sym_geom(M, nparts);
  const size_t need = sym_ws_bytes(M, S::W, nparts);
  if (ws == nullptr || wsb < need) {
    set_error("ode_self_bwd(sym eta): workspace too small (%zu < %zu bytes)", wsb, need);
    return DICP_ERR_WORKSPACE;
  }
  if (o.ptr[1] == nullptr) {
    set_error("ode_self_bwd(sym eta): the gp output is required");
    return DICP_ERR_INVALID;
  }
  float* slab = reinterpret_cast<float*>(ws);
  const bool gq = !pk || o.ptr[0] != nullptr;
  const int W = gq ? S::W : D;
  const int64_t stride = M * W;
  const int nq_own = part < g.nQ ? (g.nQ - part + nparts - 1) / nparts : 0;
  if (nq_own > 0) {
    const dim3 grid((unsigned)g.Kmax, (unsigned)nq_own);
    if (pk && gq && b0)
      sym_bwd_eta_pk_kernel<D, true, true><<<grid, dim3(256), 0, st>>>(a, sc, M, g.nG, g.L, slab, stride, part, nparts);
    else if (pk && gq)
      sym_bwd_eta_pk_kernel<D, true, false><<<grid, dim3(256), 0, st>>>(a, sc, M, g.nG, g.L, slab, stride, part, nparts);
    else if (pk && b0)
      sym_bwd_eta_pk_kernel<D, false, true><<<grid, dim3(256), 0, st>>>(a, sc, M, g.nG, g.L, slab, stride, part, nparts);
    else if (pk)
      sym_bwd_eta_pk_kernel<D, false, false><<<grid, dim3(256), 0, st>>>(a, sc, M, g.nG, g.L, slab, stride, part, nparts);
    else
      sym_kernel<S><<<dim3((unsigned)g.Kmax, (unsigned)g.nQ), dim3(256), 0, st>>>(a, sc, M, g.nG, g.L,
                                                                                  slab, stride);
    int rc = check_launch("ode_self_bwd(sym eta)");
    if (rc) return rc;
  }
  const dim3 mg((unsigned)((M * W + 255) / 256));
  if (gq) {
    if (nparts > 1)
      sym_merge_kernel<D, true><<<mg, dim3(256), 0, st>>>(slab, stride, M, g.nG, g.L, 1.f, 1.f, o, part, nparts);
    else
      sym_merge_kernel<D, false><<<mg, dim3(256), 0, st>>>(slab, stride, M, g.nG, g.L, 1.f, 1.f, o, 0, 1);
  } else {
    if (nparts > 1)
      sym_merge_kernel<D, true, D><<<mg, dim3(256), 0, st>>>(slab, stride, M, g.nG, g.L, 1.f, 1.f, o, part, nparts);
    else
      sym_merge_kernel<D, false, D><<<mg, dim3(256), 0, st>>>(slab, stride, M, g.nG, g.L, 1.f, 1.f, o, 0, 1);
  }
  return check_launch("ode_self_bwd(sym eta merge)");
}

// packed-FP32 variant of sym_bwd_kernel (lddmm_sym_pk.hpp); GQ = false: gp half only; GT =
// false: without the divergence cotangent's pair terms; RAW: coordinates in original units
template <int D, bool GQ, bool B0, bool GT, bool RAW>
__global__ void sym_bwd_pk_kernel(Args a, Scal sc, int64_t M, int nG, int L, float* __restrict__ slab,
                                  int64_t slot_stride, int qoff, int qstride);

// 4 rows per lane (two float2 row pairs, 256-point groups: lddmm_sym_pk.hpp sym_pk4_body) for
// the packed eta = 0 VJP.  dicp_set_option "sym_rp" (row pairs per lane): 1 = 2 rows, 2 = 4
// rows, 0 = automatic -- whole passes from DICP_SYM_ROWS4_WHOLE_MIN_M points; row-split parts
// from DICP_SYM_ROWS4_MIN_M points when the part (1/nparts of the pairs) still has
// >= DICP_SYM_ROWS4_MIN_PAIRS pairs; below that the quarter as many workgroups leave a tail.  Measured on MI355X (tools/probes/sym_rp_ab.py,
// profiles/r04_ab_sym_rp.jsonl): adjoint step with divergence rows 0.91x at 50k, 1.05x at
// 70k, 1.07x at 90k-200k (gp-only step 1.10-1.14x); row-split parts 0.91x at 70k / 8 parts,
// 1.03-1.15x from ~2e9 pairs per part.
constexpr int kSymG4 = 256;
inline int& sym_rp() {
  static int v = 0;
  return v;
}
#ifndef DICP_SYM_ROWS4_MIN_M
#define DICP_SYM_ROWS4_MIN_M 64000
#endif
#ifndef DICP_SYM_ROWS4_MIN_PAIRS
#define DICP_SYM_ROWS4_MIN_PAIRS 2.0e9
#endif
// whole passes (one launch over all pairs): with the column-group rule of sym_geom (L = 2, or
// 1 where L = 2 leaves an emptier last round) 4 rows win from 40k: adjoint step with divergence
// rows 1.08x at 40k, 1.04x at 46k, 1.00x at 50k (L = 1), 1.08x at 52k, 1.07x at 56k, 1.08x at
// 64k, 1.10x at 80k (profiles/r04_ab_sym_rp_L2.jsonl, r04_ab_rows4_L_50k.jsonl)
#ifndef DICP_SYM_ROWS4_WHOLE_MIN_M
#define DICP_SYM_ROWS4_WHOLE_MIN_M 40000
#endif
// With a geometry hint batch_share > 1 (a launch shares the chip with the other frames'
// launches, PSR concurrent frames): the 4-row forms from 1e9 pairs over the sharing calls --
// the other streams' launches fill the quarter-size grids' tails.  Measured on the 32-frame
// 20k atlas with 4 concurrent frames (profiles/r04_c4fixed_r4_*.json): 0.379 atlas it/s with
// the 2-row forms, 0.388 with the 4-row VJP, 0.398 with the 4-row symmetric forward, 0.414
// with both.
#ifndef DICP_SYM_SHARE4_MIN_PAIRS
#define DICP_SYM_SHARE4_MIN_PAIRS 1.0e9
#endif
inline bool sym_use_rows4(int64_t M, int nparts) {
  if (sym_rp() == 1) return false;
  if (sym_rp() == 2) return true;
  if (batch_share() > 1)   // concurrent / batched calls: their total pairs decide
    return M >= 8192 && (double)M * (double)M * batch_share() / (double)nparts >= DICP_SYM_SHARE4_MIN_PAIRS;
  if (nparts == 1) return M >= DICP_SYM_ROWS4_WHOLE_MIN_M;
  return M >= DICP_SYM_ROWS4_MIN_M && (double)M * (double)M / (double)nparts >= DICP_SYM_ROWS4_MIN_PAIRS;
}
template <int D, bool GQ, bool B0, bool GT, bool RAW>
__global__ void sym_bwd_pk4_kernel(Args a, Scal sc, int64_t M, int nG, int L, float* __restrict__ slab,
                                   int64_t slot_stride, int qoff, int qstride);

template <int D, bool GQ, bool B0, bool GT, bool RAW>
int sym_bwd_pk_batch_flush(const std::vector<const void*>& es, hipStream_t st);
template <int D, bool GQ, bool B0, bool GT, bool RAW>
int sym_bwd_pk4_batch_flush(const std::vector<const void*>& es, hipStream_t st);

template <int D, bool GQ, bool B0>
inline void sym_bwd_pk4_launch(bool gt, bool raw, dim3 grid, hipStream_t st, const Args& a, const Scal& sc,
                               int64_t M, const SymGeom& g, float* slab, int64_t stride, int part, int nparts) {
  if (batching()) {
    const SymEntry e{a, sc, M, g.nG, g.L, slab, stride, part, nparts, grid.x, grid.y};
    if (gt && raw) batch_record(sym_bwd_pk4_batch_flush<D, GQ, B0, true, true>, e);
    else if (gt) batch_record(sym_bwd_pk4_batch_flush<D, GQ, B0, true, false>, e);
    else if (raw) batch_record(sym_bwd_pk4_batch_flush<D, GQ, B0, false, true>, e);
    else batch_record(sym_bwd_pk4_batch_flush<D, GQ, B0, false, false>, e);
    return;
  }
  if (gt && raw)
    sym_bwd_pk4_kernel<D, GQ, B0, true, true><<<grid, dim3(256), 0, st>>>(a, sc, M, g.nG, g.L, slab, stride, part, nparts);
  else if (gt)
    sym_bwd_pk4_kernel<D, GQ, B0, true, false><<<grid, dim3(256), 0, st>>>(a, sc, M, g.nG, g.L, slab, stride, part, nparts);
  else if (raw)
    sym_bwd_pk4_kernel<D, GQ, B0, false, true><<<grid, dim3(256), 0, st>>>(a, sc, M, g.nG, g.L, slab, stride, part, nparts);
  else
    sym_bwd_pk4_kernel<D, GQ, B0, false, false><<<grid, dim3(256), 0, st>>>(a, sc, M, g.nG, g.L, slab, stride, part, nparts);
}

template <int D, bool GQ, bool B0>
inline void sym_bwd_pk_launch(bool g4, bool gt, bool raw, dim3 grid, hipStream_t st, const Args& a, const Scal& sc,
                              int64_t M, const SymGeom& g, float* slab, int64_t stride, int part, int nparts) {
  if (g4) {
    sym_bwd_pk4_launch<D, GQ, B0>(gt, raw, grid, st, a, sc, M, g, slab, stride, part, nparts);
    return;
  }
  if (batching()) {
    const SymEntry e{a, sc, M, g.nG, g.L, slab, stride, part, nparts, grid.x, grid.y};
    if (gt && raw) batch_record(sym_bwd_pk_batch_flush<D, GQ, B0, true, true>, e);
    else if (gt) batch_record(sym_bwd_pk_batch_flush<D, GQ, B0, true, false>, e);
    else if (raw) batch_record(sym_bwd_pk_batch_flush<D, GQ, B0, false, true>, e);
    else batch_record(sym_bwd_pk_batch_flush<D, GQ, B0, false, false>, e);
    return;
  }
  if (gt && raw)
    sym_bwd_pk_kernel<D, GQ, B0, true, true><<<grid, dim3(256), 0, st>>>(a, sc, M, g.nG, g.L, slab, stride, part, nparts);
  else if (gt)
    sym_bwd_pk_kernel<D, GQ, B0, true, false><<<grid, dim3(256), 0, st>>>(a, sc, M, g.nG, g.L, slab, stride, part, nparts);
  else if (raw)
    sym_bwd_pk_kernel<D, GQ, B0, false, true><<<grid, dim3(256), 0, st>>>(a, sc, M, g.nG, g.L, slab, stride, part, nparts);
  else
    sym_bwd_pk_kernel<D, GQ, B0, false, false><<<grid, dim3(256), 0, st>>>(a, sc, M, g.nG, g.L, slab, stride, part, nparts);
}

// b0: the cotangent on mG (Args r3 / c3) is identically zero -- those pointers are then not
// read (SymBwdPk<., ., true>, packed kernel only).
// zs (rows [zr0, zr0 + zn)): the forward's divergence rows (OpOdeSelfFwdZs); with them, or
// without a divergence cotangent (sc.dev0 == NULL: gam = 0), the packed kernels run without
// the divergence cotangent's pair terms and the merge adds their row totals.
// raw: the packed kernels in original coordinates (the caller passes Args::scale = 1, no shift,
// Scal::aux1 = s); ignored by the scalar kernel (pk = false), which is scaled only
template <int D>
int launch_sym_bwd(const Args& a, const Scal& sc, int64_t M, const Outs& o, void* ws, size_t wsb,
                   hipStream_t st, int part = 0, int nparts = 1, bool pk = false, bool b0 = false,
                   const float* zs = nullptr, int64_t zr0 = 0, int64_t zn = 0, bool raw = false) {
  if (M <= 0) return DICP_OK;
  if (zs != nullptr && !pk) {
    set_error("ode_self_bwd(sym): divergence rows need the packed kernel (bwd_alg 3)");
    return DICP_ERR_INVALID;
  }
  const bool gt = !(zs != nullptr || sc.dev0 == nullptr);  // pair loop with the gam terms
  const float* gd = zs != nullptr ? sc.dev0 : nullptr;
  const bool g4 = pk && sym_use_rows4(M, nparts);   // 256-point groups (fewer slots: the 128 workspace fits)
  const SymGeom g = g4 ? sym_geom(M, nparts, kSymG4, 2) : sym_geom(M, nparts, kSymG);
  const size_t need = sym_ws_bytes(M, 2 * D, nparts);
  if (ws == nullptr || wsb < need) {
    set_error("ode_self_bwd(sym): workspace too small (%zu < %zu bytes)", wsb, need);
    return DICP_ERR_WORKSPACE;
  }
  if (o.ptr[1] == nullptr) {
    set_error("ode_self_bwd(sym): the gp output is required");
    return DICP_ERR_INVALID;
  }
  float* slab = reinterpret_cast<float*>(ws);
  if (pk && o.ptr[0] == nullptr) {
    // gp only: the gq half of the pair algebra is never evaluated (also per pair-subset part)
    const int64_t stride1 = M * D;
    const int nq1 = part < g.nQ ? (g.nQ - part + nparts - 1) / nparts : 0;
    if (nq1 > 0) {
      const dim3 grid((unsigned)g.Kmax, (unsigned)nq1);
      if (b0)
        sym_bwd_pk_launch<D, false, true>(g4, gt, raw, grid, st, a, sc, M, g, slab, stride1, part, nparts);
      else
        sym_bwd_pk_launch<D, false, false>(g4, gt, raw, grid, st, a, sc, M, g, slab, stride1, part, nparts);
      int rc = check_launch("ode_self_bwd(sym gp)");
      if (rc) return rc;
    }
    const dim3 mg((unsigned)((M * D + 255) / 256));
    if (g4 && nparts > 1)
      sym_merge_launch<D, true, D, kSymG4>(mg, st, slab, stride1, M, g.nG, g.L, sc.s, a.scale, o, part, nparts, zs,
                                           zr0, zn, gd);
    else if (g4)
      sym_merge_launch<D, false, D, kSymG4>(mg, st, slab, stride1, M, g.nG, g.L, sc.s, a.scale, o, 0, 1, zs, zr0,
                                            zn, gd);
    else if (nparts > 1)
      sym_merge_launch<D, true, D>(mg, st, slab, stride1, M, g.nG, g.L, sc.s, a.scale, o, part, nparts, zs, zr0, zn,
                                   gd);
    else
      sym_merge_launch<D, false, D>(mg, st, slab, stride1, M, g.nG, g.L, sc.s, a.scale, o, 0, 1, zs, zr0, zn, gd);
    return check_launch("ode_self_bwd(sym gp merge)");
  }
  const int64_t stride = M * 2 * D;
  const int nq_own = part < g.nQ ? (g.nQ - part + nparts - 1) / nparts : 0;
  if (nq_own > 0) {
    const dim3 grid((unsigned)g.Kmax, (unsigned)nq_own);
    if (pk && b0)
      sym_bwd_pk_launch<D, true, true>(g4, gt, raw, grid, st, a, sc, M, g, slab, stride, part, nparts);
    else if (pk)
      sym_bwd_pk_launch<D, true, false>(g4, gt, raw, grid, st, a, sc, M, g, slab, stride, part, nparts);
    else if (batching()) {
      set_error("ode_self_bwd(sym): the scalar symmetric VJP (bwd_alg 2) has no batched form");
      return DICP_ERR_UNSUPPORTED;
    } else
      sym_bwd_kernel<D><<<dim3((unsigned)g.Kmax, (unsigned)nq_own), dim3(256), 0, st>>>(
          a, sc, M, g.nG, g.L, slab, stride, part, nparts);
    int rc = check_launch("ode_self_bwd(sym)");
    if (rc) return rc;
  }
  const int64_t n = M * 2 * D;
  const dim3 mgn((unsigned)((n + 255) / 256));
  if (g4 && nparts > 1)
    sym_merge_launch<D, true, 2 * D, kSymG4>(mgn, st, slab, stride, M, g.nG, g.L, sc.s, a.scale, o, part, nparts, zs,
                                             zr0, zn, gd);
  else if (g4)
    sym_merge_launch<D, false, 2 * D, kSymG4>(mgn, st, slab, stride, M, g.nG, g.L, sc.s, a.scale, o, 0, 1, zs, zr0,
                                              zn, gd);
  else if (nparts > 1)
    sym_merge_launch<D, true>(mgn, st, slab, stride, M, g.nG, g.L, sc.s, a.scale, o, part, nparts, zs, zr0, zn, gd);
  else
    sym_merge_launch<D, false>(mgn, st, slab, stride, M, g.nG, g.L, sc.s, a.scale, o, 0, 1, zs, zr0, zn, gd);
  return check_launch("ode_self_bwd(sym merge)");
}

}  // namespace dicp
