// Packed-FP32 variant of the row-reduction skeleton (common.hpp rowred_kernel) for the
// fused LDDMM forward: each thread's two rows (i, i + 256) are held as float2 vectors, so
// every per-pair FMA / mul / sub of the two rows is ONE v_pk_*_f32 instruction (two lanes of
// work per VALU issue slot; the MI355X vector peak, 157 TF/s, is only reachable packed).
// The column record is a scalar broadcast into both halves (VOP3P op_sel).  Split columns,
// slabs, merge and the Outs epilogue are those of the generic kernel (same row mapping as
// rowred_kernel<Op, 2>), so results differ only by fp32 contraction order.
#pragma once
#include "launch.hpp"
#include "lddmm_ops.hpp"

namespace dicp {

typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2 pk_fma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 splat(float x) { return f2{x, x}; }

// Launch constants of the eta != 0 (logdet / gradcomponent) forward, formed in double on the
// host for the coordinate scale the kernel actually applies (Args::scale = alpha rounded to
// float; 1 for raw coordinates).  In that model the velocity V + eta s sum K z, the divergence
// rows and the Hamiltonian rows are small differences of large sums (the ridge zero-speed a0 of
// ICP_two_set: K a0 ~ eta GradKRed), so a relative error of ~1e-7 in a launch constant is a
// SYSTEMATIC error of every row, which the shooting integrates into its cost
// (tools/probes/logdet_cost_diag.py, DESIGN.md section 3: the float32 alpha in the exponent
// and eta * (s / alpha) rounded in float gave 2.5x the float32 restatement's cost error).  So
// the exponent carries the float32 scale's correction and every cancelling coefficient is a
// (hi, lo) float pair.
struct EtaConsts {
  float e0, e1;   // exponent e = e0 r2 + e1 r2 (scaled: e0 = -1, e1 = -(alpha^2 / scale^2 - 1);
                  // raw: (e0, e1) = nc = -log2(e) s / 2 as hi + lo)
  float s2;       // s / scale^2: s |z|^2 in the kernel's units (the L, GL' and Hs terms)
  float sa;       // s / scale
  float cv[2];    // eta s / scale  (v = V + cv Z', h)
  float cg[2];    // eta scale      (g = -sa (p.Z' - cg L), mG = sa (Gs' + cg Hs - ch GL'))
  float ch[2];    // eta^2 s
};

inline void split_hi_lo(double x, float* hl) {
  hl[0] = (float)x;
  hl[1] = (float)(x - (double)hl[0]);
}

inline EtaConsts eta_consts(float scale, bool raw) {
  const double sg = tl_launch_sigma, eta = tl_launch_eta;
  const double s = 1.0 / (sg * sg);
  const double a = raw ? 1.0 : (double)scale;
  const double nc = -1.4426950408889634 * 0.5 * s;   // K = exp2(nc |z|^2)
  EtaConsts c;
  if (raw) {
    c.e0 = (float)nc;
    c.e1 = (float)(nc - (double)c.e0);
  } else {
    c.e0 = -1.f;
    c.e1 = (float)(nc / (a * a) + 1.0);   // -(alpha^2 / scale^2 - 1), alpha^2 = -nc
  }
  c.s2 = (float)(s / (a * a));
  c.sa = (float)(s / a);
  split_hi_lo(eta * s / a, c.cv);
  split_hi_lo(eta * a, c.cg);
  split_hi_lo(eta * eta * s, c.ch);
  return c;
}

struct NoConsts {};
// ops with launch constants (Op::kConsts, Op::Consts) get them as a kernel argument of their own
template <class T, class = void>
struct op_consts { using type = NoConsts; static constexpr bool value = false; };
template <class T>
struct op_consts<T, std::enable_if_t<T::kConsts>> { using type = typename T::Consts; static constexpr bool value = true; };

template <class Op>
inline typename op_consts<Op>::type make_op_consts(const Args& a) {
  if constexpr (op_consts<Op>::value) return Op::make_consts(a);
  else return NoConsts{};
}

// OpOdeSelfFwd<D, ETA, DIV> (lddmm_ops.hpp) on two rows at once: V, Gs' (, Z'), and for
// eta != 0 (ETA, which implies Z') the Hs, GL' and L sums of the logdet / gradcomponent model.
// G = false: the sums feeding mG only (Gs', and for eta != 0 Hs and GL') are not formed (mG not
// wanted: the last step of a shooting whose final momenta are not used) -- eta = 0: 7 of the
// 19 per-pair packed instructions drop; eta != 0: 25 of 39.
// ZS = true (eta = 0, DIV): the row's Z' sum also goes out, in original units, through the
// h slot (which an Euler step does not use): zs_i = sum_j K (q_i - q_j) = Z'_i / alpha -- the
// divergence rows the matching VJP reuses (OpOdeSelfFwdZs, sym_merge_kernel).
// RAW = true: coordinates in original units (the launcher sets Args::scale = 1, no shift,
// Scal::aux1 = s): z = q_i - q_j is exact for nearby points whatever the cloud's extent, and
// the exponent costs one packed multiply more per two pairs (K = exp2(nc r2)); every sum and
// epilogue is otherwise the same (coord_raw).
template <int D, bool DIV, bool ETA = false, bool G = true, bool ZS = false, bool RAW = false>
struct OpOdeSelfFwdPk {
  static_assert(!ZS || (DIV && !ETA), "zs rows: eta = 0 with the divergence sums only");
  using Base = std::conditional_t<ZS, OpOdeSelfFwdZs<D>, OpOdeSelfFwd<D, ETA, DIV || ETA>>;
  // column splits as the full pass: the same chunk boundaries, hence bitwise the same v / g
  using SplitAs = OpOdeSelfFwdPk<D, DIV, ETA, true, false, RAW>;
  static constexpr int kRP = ETA ? 1 : 2;   // 4 rows per thread at eta = 0 (rowred_pk_kernel)
  static constexpr int CW4 = Base::CW4;
  static constexpr int NACC = Base::NACC;
  static constexpr int kNOut = Base::kNOut;
  static constexpr bool kMin = false;
  struct Row2 {
    f2 q[D], p[D];
    f2 nc, s2;   // exponent multiplier (RAW) and s / alpha^2 (kS2 scaled, s raw); eta != 0: the
                 // exponent's e1 and EtaConsts::s2
    f2 e0;       // eta != 0, RAW: the exponent's e0
  };
  // eta != 0: the launch constants of the model's cancelling sums (EtaConsts)
  static constexpr bool kConsts = ETA;
  using Consts = EtaConsts;
  static EtaConsts make_consts(const Args& a) { return eta_consts(a.scale, RAW); }
  // LDS column record of the packed pair: D = 3 as [q (3) | q_z | p (3) | p_z], so that the
  // z components are the aligned register pairs (.z, .w) of one ds_read_b128 each instead of
  // broadcasts, which the register allocator materialises with a v_mov per column (the x / y
  // broadcasts go through op_sel); D = 2 keeps the base record [q | p]
#ifndef DICP_FWD_PK_REC4
#define DICP_FWD_PK_REC4 1
#endif
  static constexpr int kP = (DICP_FWD_PK_REC4 && D == 3) ? 4 : D;
  static_assert(kP + D <= 4 * CW4, "record fits the base op's float4s");
  __device__ static void load_col_pk(const Args& a, const Scal& sc, int64_t j, float* rec) {
    float t[4 * CW4];
    op_load_col<Base>(a, sc, j, t);
#pragma unroll
    for (int k = 0; k < 4 * CW4; ++k) rec[k] = 0.f;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      rec[d] = t[d];
      rec[kP + d] = t[D + d];
    }
    if (kP > D) {
      rec[D] = t[D - 1];
      rec[kP + D] = t[2 * D - 1];
    }
  }
  // column field d of the record as a broadcast pair (the duplicated z components: the pair)
  __device__ static f2 colq(const float* rec, int d) {
    return (kP > D && d == D - 1) ? f2{rec[d], rec[D]} : splat(rec[d]);
  }
  __device__ static f2 colp(const float* rec, int d) {
    return (kP > D && d == D - 1) ? f2{rec[kP + d], rec[kP + D]} : splat(rec[kP + d]);
  }
  __device__ static void load_rows_s(const Args& a, const Scal& sc, int64_t i0, int64_t i1, Row2& r,
                                     typename Base::Row& b0, typename Base::Row& b1) {
    Base::load_row(a, i0, b0);
    Base::load_row(a, i1, b1);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      r.q[d] = f2{b0.q[d], b1.q[d]};
      r.p[d] = f2{b0.p[d], b1.p[d]};
    }
    r.nc = splat(sc.nc);
    r.s2 = splat(RAW ? sc.s : kS2);
  }
  __device__ static void load_rows_c(const Args& a, const Scal& sc, const EtaConsts& cx, int64_t i0, int64_t i1,
                                     Row2& r, typename Base::Row& b0, typename Base::Row& b1) {
    load_rows_s(a, sc, i0, i1, r, b0, b1);
    r.nc = splat(cx.e1);
    r.e0 = splat(cx.e0);
    r.s2 = splat(cx.s2);
  }
  // eta != 0: the sums whose cancellation forms v, g and h -- V, Z' and L -- are totalled in
  // double over sub-tiles of DICP_PK_F64_SUB columns (rowred_pk_body_f64), the outputs formed
  // from them in double (store_d) and the column-split partials merged in double
  static constexpr bool kF64 = ETA;
  __host__ __device__ static constexpr bool f64_acc(int k) {
    return ETA && (k < D || (k >= 2 * D && k < 3 * D) || k == 5 * D);
  }
  __device__ static void store_d(const Scal&, const EtaConsts& cx, const typename Base::Row& r, const float* t,
                                 const double* td, double* v) {
    const double cv = (double)cx.cv[0] + (double)cx.cv[1];
    const double cg = (double)cx.cg[0] + (double)cx.cg[1];
    const double ch = (double)cx.ch[0] + (double)cx.ch[1];
    const double sa = cx.sa;
    double pV = 0.0, pZ = 0.0;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      v[d] = td[d] + cv * td[2 * D + d];
      v[D + d] = sa * ((double)t[D + d] + cg * (double)t[3 * D + d] - ch * (double)t[4 * D + d]);
      pV += (double)r.p[d] * td[d];
      pZ += (double)r.p[d] * td[2 * D + d];
    }
    const double L = td[5 * D];
    v[2 * D] = -sa * (pZ - cg * L);
    v[2 * D + 1] = 0.5 * pV + cv * pZ - 0.5 * ch * L;
  }
  // OpOdeSelfFwd::store (eta != 0) with the EtaConsts coefficients: the same outputs, each
  // cancelling coefficient applied as hi + lo
  __device__ static void store_c(const Scal&, const EtaConsts& cx, const typename Base::Row& r, const float* t,
                                 float* v) {
    const float* V = t;
    const float* Gs = t + D;
    const float* Z = t + 2 * D;
    const float* Hs = t + 3 * D;
    const float* GL = t + 4 * D;
    const float L = t[5 * D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
      v[d] = fmaf(cx.cv[0], Z[d], fmaf(cx.cv[1], Z[d], V[d]));
      float m = fmaf(cx.cg[0], Hs[d], fmaf(cx.cg[1], Hs[d], Gs[d]));
      m = fmaf(-cx.ch[0], GL[d], fmaf(-cx.ch[1], GL[d], m));
      v[D + d] = cx.sa * m;
    }
    const float pV = dot<D>(r.p, V);
    const float pZ = dot<D>(r.p, Z);
    v[2 * D] = -cx.sa * fmaf(-cx.cg[0], L, fmaf(-cx.cg[1], L, pZ));
    const float h = fmaf(cx.cv[0], pZ, fmaf(cx.cv[1], pZ, 0.5f * pV));
    v[2 * D + 1] = fmaf(-0.5f * cx.ch[0], L, fmaf(-0.5f * cx.ch[1], L, h));
  }
  __device__ static void pair2(const Row2& r, const float* rec, f2* acc) {
    f2 z[D];
    f2 r2 = splat(0.f);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      z[d] = r.q[d] - colq(rec, d);
      r2 = pk_fma(z[d], z[d], r2);
    }
    f2 K;
    if constexpr (ETA) {   // the exponent of the exact alpha (EtaConsts): one packed FMA more
      const f2 e = RAW ? pk_fma(r2, r.nc, r.e0 * r2) : pk_fma(r2, r.nc, -r2);
      K = f2{fast_exp2(e.x), fast_exp2(e.y)};
    } else if constexpr (RAW) {
      const f2 e = r.nc * r2;
      K = f2{fast_exp2(e.x), fast_exp2(e.y)};
    } else {
      K = f2{fast_exp2(-r2.x), fast_exp2(-r2.y)};
    }
    f2 pj[D];
#pragma unroll
    for (int d = 0; d < D; ++d) pj[d] = colp(rec, d);
    if constexpr (G) {
      f2 pp = r.p[0] * pj[0];
#pragma unroll
      for (int d = 1; d < D; ++d) pp = pk_fma(r.p[d], pj[d], pp);
      const f2 Kpp = K * pp;
#pragma unroll
      for (int d = 0; d < D; ++d) acc[D + d] = pk_fma(Kpp, z[d], acc[D + d]);
    }
#pragma unroll
    for (int d = 0; d < D; ++d) {
      acc[d] = pk_fma(K, pj[d], acc[d]);
      if (DIV || ETA) acc[2 * D + d] = pk_fma(K, z[d], acc[2 * D + d]);
    }
    if (ETA) {  // OpOdeSelfFwd::pair, eta != 0 terms
      const f2 sr2 = r.s2 * r2;
      if constexpr (G) {  // Hs, GL' feed mG only
        f2 u[D];
#pragma unroll
        for (int d = 0; d < D; ++d) u[d] = r.p[d] - pj[d];
        f2 zu = z[0] * u[0];
#pragma unroll
        for (int d = 1; d < D; ++d) zu = pk_fma(z[d], u[d], zu);
        const f2 szu = r.s2 * zu;
        const f2 KGL = K * (sr2 - splat((float)(D + 2)));
#pragma unroll
        for (int d = 0; d < D; ++d) {
          acc[3 * D + d] = pk_fma(K, pk_fma(szu, z[d], -u[d]), acc[3 * D + d]);  // Hs
          acc[4 * D + d] = pk_fma(KGL, z[d], acc[4 * D + d]);                     // GL'
        }
      }
      acc[5 * D] = pk_fma(K, sr2 - splat((float)D), acc[5 * D]);  // L
    }
  }
};

// occupancy experiments (tools/ab_libs.py): -DDICP_FWD_PK_WAVES=n asks for n waves per SIMD
#ifdef DICP_FWD_PK_WAVES
#define DICP_FWD_PK_ATTR __attribute__((amdgpu_waves_per_eu(DICP_FWD_PK_WAVES, 8)))
#else
#define DICP_FWD_PK_ATTR
#endif
#ifndef DICP_PK_PAIR_UNROLL
#define DICP_PK_PAIR_UNROLL DICP_PAIR_UNROLL
#endif
// packed ops may define load_rows_s, which also sees the launch scalars (row constants such
// as a cotangent scale read from device memory at kernel start)
template <class T, class = void>
struct has_rows_s : std::false_type {};
template <class T>
struct has_rows_s<T, std::void_t<decltype(&T::load_rows_s)>> : std::true_type {};

// packed ops may lay the LDS column record out for their pair2 (load_col_pk)
template <class T, class = void>
struct has_col_pk : std::false_type {};
template <class T>
struct has_col_pk<T, std::void_t<decltype(&T::load_col_pk)>> : std::true_type {};
template <class Op>
__device__ __forceinline__ void pk_load_col(const Args& a, const Scal& sc, int64_t j, float* rec) {
  if constexpr (has_col_pk<Op>::value) Op::load_col_pk(a, sc, j, rec);
  else op_load_col<typename Op::Base>(a, sc, j, rec);
}

// Row pairs per thread RP (each pair = one f2 lane pair of rows i, i + 256): RP = 2 shares every
// column record (LDS reads, LDS address, broadcast moves) among 4 rows.  Ops opt in with
// kRP = 2 (the eta = 0 fused forward; tools/probes/pk_rp_sweep.py, profiles/
// r03_ab_pk_rp_sweep.jsonl: Euler step 1.01x at 30k, 1.02-1.05x at 40k-70k, 1.045x at 100k,
// 1.05x at 200k, 0.96x at 20k where the halved workgroup count leaves a tail; the external-
// point passes, tools/probes/pk_rp_ext.py, profiles/r03_ab_pk_rp_ext.jsonl: 1.02-1.05x from 10k
// columns on, 0.93-0.94x at 2k columns); the launcher uses it from DICP_PK_RP2_ROWS rows and
// DICP_PK_RP2_COLS columns on.
// dicp_set_option "pk_rp" (0 auto, 1, 2) forces it for every packed op (A/B).
inline int& pk_rp_force() {
  static int v = 0;
  return v;
}
#ifndef DICP_PK_RP2_ROWS
#define DICP_PK_RP2_ROWS 32768
#endif
template <class T, class = void>
struct pk_rp_pref { static constexpr int value = 1; };
template <class T>
struct pk_rp_pref<T, std::void_t<decltype(T::kRP)>> { static constexpr int value = T::kRP; };
// experiment builds (-DDICP_PK_RP_EXTRA=1) also instantiate 3 and 4 row pairs per thread
#ifndef DICP_PK_RP_EXTRA
#define DICP_PK_RP_EXTRA 0
#endif
constexpr int kPkRPMax = DICP_PK_RP_EXTRA ? 4 : 2;
#ifndef DICP_PK_RP2_COLS
#define DICP_PK_RP2_COLS 8192
#endif
template <class Op>
int pk_rp(int64_t M, int64_t N) {
  if (pk_rp_force() > 0) return pk_rp_force() > kPkRPMax ? kPkRPMax : pk_rp_force();
  // batch_share: the rows of the whole batch decide (the tail the 4-row form leaves is the
  // batch's, not the call's)
  return (pk_rp_pref<Op>::value >= 2 && M * batch_share() >= DICP_PK_RP2_ROWS && N >= DICP_PK_RP2_COLS) ? 2 : 1;
}

// The body of rowred_pk_kernel for block (bx, by) of a grid with S column splits (by < S;
// S > 1: partial slabs, S = 1: the epilogue) -- shared by the plain and the batched kernel.
// WRAP (the row split's column phases): column j is read at (coff + j) mod ntot.
template <class Op, int RP, bool WRAP = false>
__device__ __forceinline__ void rowred_pk_body(Args args, Scal sc, int64_t M, int64_t N, int64_t chunk,
                                               const Outs& outs, unsigned bx, unsigned by, unsigned S,
                                               int64_t coff = 0, int64_t ntot = 0,
                                               const typename op_consts<Op>::type& cx = {}) {
  auto col = [&](int64_t j) {
    if constexpr (WRAP) {
      j += coff;
      if (j >= ntot) j -= ntot;
    }
    return j;
  };
  using Base = typename Op::Base;
  constexpr int CW4 = Op::CW4;
  constexpr int NACC = Op::NACC;
  __shared__ float4 lds[2][kTile * CW4];
  if (sc.dev0 != nullptr) sc.aux0 = sc.dev0[0];

  const int tid = threadIdx.x;
  const int64_t ibase = (int64_t)bx * (kBlock * 2 * RP) + tid;
  typename Base::Row brow[RP][2];
  typename Op::Row2 row[RP];
#pragma unroll
  for (int h = 0; h < RP; ++h) {
    const int64_t i0 = ibase + (int64_t)(2 * h) * kBlock, i1 = i0 + kBlock;
    if constexpr (op_consts<Op>::value)
      Op::load_rows_c(args, sc, cx, i0 < M ? i0 : M - 1, i1 < M ? i1 : M - 1, row[h], brow[h][0], brow[h][1]);
    else if constexpr (has_rows_s<Op>::value)
      Op::load_rows_s(args, sc, i0 < M ? i0 : M - 1, i1 < M ? i1 : M - 1, row[h], brow[h][0], brow[h][1]);
    else
      Op::load_rows(args, i0 < M ? i0 : M - 1, i1 < M ? i1 : M - 1, row[h], brow[h][0], brow[h][1]);
  }

  f2 tot[RP][NACC];
#pragma unroll
  for (int h = 0; h < RP; ++h)
#pragma unroll
    for (int k = 0; k < NACC; ++k) tot[h][k] = splat(0.f);

  const int64_t j0 = (int64_t)by * chunk;
  int64_t j1 = j0 + chunk;
  if (j1 > N) j1 = N;

  float pre[CW4 * 4];
  int cnt = (int)((j1 - j0) < kTile ? (j1 - j0) : kTile);
  if (cnt > 0 && tid < cnt) {
    pk_load_col<Op>(args, sc, col(j0 + tid), pre);
#pragma unroll
    for (int k = 0; k < CW4; ++k)
      lds[0][tid * CW4 + k] = make_float4(pre[4 * k], pre[4 * k + 1], pre[4 * k + 2], pre[4 * k + 3]);
  }
  __syncthreads();
  int buf = 0;
  for (int64_t jt = j0; jt < j1; jt += kTile) {
    const int64_t jn = jt + kTile;
    const int cntn = jn < j1 ? (int)((j1 - jn) < kTile ? (j1 - jn) : kTile) : 0;
    if (tid < cntn) {
      pk_load_col<Op>(args, sc, col(jn + tid), pre);
#pragma unroll
      for (int k = 0; k < CW4; ++k)
        lds[buf ^ 1][tid * CW4 + k] =
            make_float4(pre[4 * k], pre[4 * k + 1], pre[4 * k + 2], pre[4 * k + 3]);
    }
    f2 acc[RP][NACC];
#pragma unroll
    for (int h = 0; h < RP; ++h)
#pragma unroll
      for (int k = 0; k < NACC; ++k) acc[h][k] = splat(0.f);
    const float4* tile = lds[buf];
#pragma unroll DICP_PK_PAIR_UNROLL
    for (int t = 0; t < cnt; ++t) {
      float rec[CW4 * 4];
#pragma unroll
      for (int k = 0; k < CW4; ++k) {
        const float4 q = tile[t * CW4 + k];
        rec[4 * k + 0] = q.x;
        rec[4 * k + 1] = q.y;
        rec[4 * k + 2] = q.z;
        rec[4 * k + 3] = q.w;
      }
#pragma unroll
      for (int h = 0; h < RP; ++h) Op::pair2(row[h], rec, acc[h]);
    }
#pragma unroll
    for (int h = 0; h < RP; ++h)
#pragma unroll
      for (int k = 0; k < NACC; ++k) tot[h][k] = tot[h][k] + acc[h][k];
    __syncthreads();
    buf ^= 1;
    cnt = cntn;
  }

  const bool split = S > 1;
#pragma unroll
  for (int h = 0; h < RP; ++h) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int64_t i = ibase + (int64_t)(2 * h + r) * kBlock;
      if (i >= M) continue;
      float t[NACC];
#pragma unroll
      for (int k = 0; k < NACC; ++k) t[k] = r == 0 ? tot[h][k].x : tot[h][k].y;
      float vals[Base::kOutW[0] + Base::kOutW[1] + Base::kOutW[2] + Base::kOutW[3]];
      if constexpr (op_consts<Op>::value)
        Op::store_c(sc, cx, brow[h][r], t, vals);
      else
        Base::store(sc, brow[h][r], t, vals);
      int off = 0;
#pragma unroll
      for (int k = 0; k < Base::kNOut; ++k) {
        const int w = Base::kOutW[k];
        float* base = outs.ptr[k];
        if (base != nullptr) {
          if (split) {
            float* dst = base + (int64_t)by * M * w + i * w;
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
}

// ops whose column sums are partly totalled in double (Op::kF64: the eta != 0 forward)
template <class T, class = void>
struct op_f64 : std::false_type {};
template <class T>
struct op_f64<T, std::enable_if_t<T::kF64>> : std::true_type {};

#ifndef DICP_PK_F64_SUB
#define DICP_PK_F64_SUB 32
#endif
// rowred_pk_body for Op::kF64 ops (with launch constants): the pair loop as rowred_pk_body, but
// every DICP_PK_F64_SUB columns the float sums of the channels Op::f64_acc are added into double
// totals (one conversion + one double add per channel and row per sub-tile: ~1% of the pair
// work at 32), Op::store_d forms the outputs in double, and split partials are stored as double
// (slab width doubled; merge_slabs_f64_kernel).  tools/probes/logdet_cost_diag.py accum_main:
// float sums over 256-column tiles leave a systematic velocity error that the logdet model's
// cost integrates; 32-column float sub-tiles with double totals remove most of it.
template <class Op, int RP, bool WRAP = false>
__device__ __forceinline__ void rowred_pk_body_f64(Args args, Scal sc, int64_t M, int64_t N, int64_t chunk,
                                                   const Outs& outs, unsigned bx, unsigned by, unsigned S,
                                                   int64_t coff, int64_t ntot, const typename Op::Consts& cx) {
  auto col = [&](int64_t j) {
    if constexpr (WRAP) {
      j += coff;
      if (j >= ntot) j -= ntot;
    }
    return j;
  };
  using Base = typename Op::Base;
  constexpr int CW4 = Op::CW4;
  constexpr int NACC = Op::NACC;
  constexpr int kSub = DICP_PK_F64_SUB;
  __shared__ float4 lds[2][kTile * CW4];
  if (sc.dev0 != nullptr) sc.aux0 = sc.dev0[0];

  const int tid = threadIdx.x;
  const int64_t ibase = (int64_t)bx * (kBlock * 2 * RP) + tid;
  typename Base::Row brow[RP][2];
  typename Op::Row2 row[RP];
#pragma unroll
  for (int h = 0; h < RP; ++h) {
    const int64_t i0 = ibase + (int64_t)(2 * h) * kBlock, i1 = i0 + kBlock;
    Op::load_rows_c(args, sc, cx, i0 < M ? i0 : M - 1, i1 < M ? i1 : M - 1, row[h], brow[h][0], brow[h][1]);
  }

  f2 tot[RP][NACC];
  double td[RP][2][NACC];
#pragma unroll
  for (int h = 0; h < RP; ++h)
#pragma unroll
    for (int k = 0; k < NACC; ++k) {
      tot[h][k] = splat(0.f);
      td[h][0][k] = td[h][1][k] = 0.0;
    }

  const int64_t j0 = (int64_t)by * chunk;
  int64_t j1 = j0 + chunk;
  if (j1 > N) j1 = N;

  float pre[CW4 * 4];
  int cnt = (int)((j1 - j0) < kTile ? (j1 - j0) : kTile);
  if (cnt > 0 && tid < cnt) {
    pk_load_col<Op>(args, sc, col(j0 + tid), pre);
#pragma unroll
    for (int k = 0; k < CW4; ++k)
      lds[0][tid * CW4 + k] = make_float4(pre[4 * k], pre[4 * k + 1], pre[4 * k + 2], pre[4 * k + 3]);
  }
  __syncthreads();
  int buf = 0;
  for (int64_t jt = j0; jt < j1; jt += kTile) {
    const int64_t jn = jt + kTile;
    const int cntn = jn < j1 ? (int)((j1 - jn) < kTile ? (j1 - jn) : kTile) : 0;
    if (tid < cntn) {
      pk_load_col<Op>(args, sc, col(jn + tid), pre);
#pragma unroll
      for (int k = 0; k < CW4; ++k)
        lds[buf ^ 1][tid * CW4 + k] =
            make_float4(pre[4 * k], pre[4 * k + 1], pre[4 * k + 2], pre[4 * k + 3]);
    }
    const float4* tile = lds[buf];
    for (int t0 = 0; t0 < cnt; t0 += kSub) {
      const int t1 = t0 + kSub < cnt ? t0 + kSub : cnt;
      f2 acc[RP][NACC];
#pragma unroll
      for (int h = 0; h < RP; ++h)
#pragma unroll
        for (int k = 0; k < NACC; ++k) acc[h][k] = splat(0.f);
#pragma unroll DICP_PK_PAIR_UNROLL
      for (int t = t0; t < t1; ++t) {
        float rec[CW4 * 4];
#pragma unroll
        for (int k = 0; k < CW4; ++k) {
          const float4 q = tile[t * CW4 + k];
          rec[4 * k + 0] = q.x;
          rec[4 * k + 1] = q.y;
          rec[4 * k + 2] = q.z;
          rec[4 * k + 3] = q.w;
        }
#pragma unroll
        for (int h = 0; h < RP; ++h) Op::pair2(row[h], rec, acc[h]);
      }
#pragma unroll
      for (int h = 0; h < RP; ++h)
#pragma unroll
        for (int k = 0; k < NACC; ++k) {
          if (Op::f64_acc(k)) {
            td[h][0][k] += (double)acc[h][k].x;
            td[h][1][k] += (double)acc[h][k].y;
          } else {
            tot[h][k] = tot[h][k] + acc[h][k];
          }
        }
    }
    __syncthreads();
    buf ^= 1;
    cnt = cntn;
  }

  const bool split = S > 1;
#pragma unroll
  for (int h = 0; h < RP; ++h) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int64_t i = ibase + (int64_t)(2 * h + r) * kBlock;
      if (i >= M) continue;
      float t[NACC];
#pragma unroll
      for (int k = 0; k < NACC; ++k) t[k] = r == 0 ? tot[h][k].x : tot[h][k].y;
      double vals[Base::kOutW[0] + Base::kOutW[1] + Base::kOutW[2] + Base::kOutW[3]];
      Op::store_d(sc, cx, brow[h][r], t, td[h][r], vals);
      int off = 0;
#pragma unroll
      for (int k = 0; k < Base::kNOut; ++k) {
        const int w = Base::kOutW[k];
        float* base = outs.ptr[k];
        if (base != nullptr) {
          if (split) {
            double* dst = reinterpret_cast<double*>(base) + (int64_t)by * M * w + i * w;
#pragma unroll
            for (int e = 0; e < w; ++e) dst[e] = vals[off + e];
          } else {
#pragma unroll
            for (int e = 0; e < w; ++e) {
              const int64_t ix = i * w + e;
              double v = (double)outs.alpha[k] * vals[off + e];
              if (outs.base[k]) v += (double)outs.base[k][ix];
              if (outs.add[k]) v += (double)outs.add[k][ix];
              if (outs.accumulate[k]) v += (double)base[ix];
              base[ix] = (float)v;
            }
          }
        }
        off += w;
      }
    }
  }
}

// bytes per slab element of an op's split partials (double for Op::kF64)
template <class Op>
constexpr size_t pk_slab_elem() { return op_f64<Op>::value ? sizeof(double) : sizeof(float); }

template <class Op, int RP>
__global__ __launch_bounds__(kBlock) DICP_FWD_PK_ATTR void rowred_pk_kernel(Args args, Scal sc, int64_t M, int64_t N,
                                                           int64_t chunk, Outs outs) {
  rowred_pk_body<Op, RP>(args, sc, M, N, chunk, outs, blockIdx.x, blockIdx.y, gridDim.y);
}
// the same for ops with launch constants (op_consts), passed by value
template <class Op, int RP>
__global__ __launch_bounds__(kBlock) DICP_FWD_PK_ATTR void rowred_pk_c_kernel(Args args, Scal sc,
                                                             typename op_consts<Op>::type cx, int64_t M,
                                                             int64_t N, int64_t chunk, Outs outs) {
  if constexpr (op_f64<Op>::value)
    rowred_pk_body_f64<Op, RP>(args, sc, M, N, chunk, outs, blockIdx.x, blockIdx.y, gridDim.y, 0, 0, cx);
  else
    rowred_pk_body<Op, RP>(args, sc, M, N, chunk, outs, blockIdx.x, blockIdx.y, gridDim.y, 0, 0, cx);
}

// batched form (batch.hpp): blockIdx.z = the recorded call
struct PkEntry {
  Args a;
  Scal sc;
  Outs outs;
  int64_t M, N, chunk;
  unsigned gx, gy;
  EtaConsts cx;   // ops with launch constants (op_consts)
};
template <class Op, int RP>
__global__ __launch_bounds__(kBlock) DICP_FWD_PK_ATTR void rowred_pk_batch_kernel(BatchTab<PkEntry> t) {
  const PkEntry& e = t.e[blockIdx.z];
  if (blockIdx.x >= e.gx || blockIdx.y >= e.gy) return;
  if constexpr (op_f64<Op>::value)
    rowred_pk_body_f64<Op, RP>(e.a, e.sc, e.M, e.N, e.chunk, e.outs, blockIdx.x, blockIdx.y, e.gy, 0, 0, e.cx);
  else if constexpr (op_consts<Op>::value)
    rowred_pk_body<Op, RP>(e.a, e.sc, e.M, e.N, e.chunk, e.outs, blockIdx.x, blockIdx.y, e.gy, 0, 0, e.cx);
  else
    rowred_pk_body<Op, RP>(e.a, e.sc, e.M, e.N, e.chunk, e.outs, blockIdx.x, blockIdx.y, e.gy);
}
template <class Op>
inline EtaConsts pk_entry_consts(const Args& a) {
  if constexpr (op_consts<Op>::value) return make_op_consts<Op>(a);
  else return EtaConsts{};
}
template <class Op, int RP>
int rowred_pk_batch_flush(const std::vector<const void*>& es, hipStream_t st) {
  return batch_launch<PkEntry>(rowred_pk_batch_kernel<Op, RP>, es, st, "rowred_pk");
}

template <class Op, int RP>
int64_t rowred_pk_capacity() {
  static int64_t cap = -1;
  if (cap < 0) {
    if constexpr (op_consts<Op>::value) cap = (int64_t)device_cus() * blocks_per_cu(rowred_pk_c_kernel<Op, RP>);
    else cap = (int64_t)device_cus() * blocks_per_cu(rowred_pk_kernel<Op, RP>);
  }
  return cap;
}

template <class T, class = void>
struct split_as { using type = T; };
template <class T>
struct split_as<T, std::void_t<typename T::SplitAs>> { using type = typename T::SplitAs; };

template <class Op>
int rowred_pk_splits(int64_t M, int64_t N) {
  using Base = typename Op::Base;
  using SOp = typename split_as<Op>::type;   // ops may borrow another variant's geometry
  const int RP = pk_rp<Op>(M, N);             // SplitAs variants share kRP, hence RP
  int64_t cap;
  switch (RP) {
#if DICP_PK_RP_EXTRA
    case 4: cap = rowred_pk_capacity<SOp, 4>(); break;
    case 3: cap = rowred_pk_capacity<SOp, 3>(); break;
#endif
    case 2: cap = rowred_pk_capacity<SOp, 2>(); break;
    default: cap = rowred_pk_capacity<SOp, 1>(); break;
  }
  cap = cap / batch_share() > 0 ? cap / batch_share() : 1;   // this call's share of the chip
  return num_splits_cap(M, N, 2 * RP, cap, round_rows_of<Base>::rows, round_rows_of<Base>::max);
}

template <class Op>
size_t rowred_pk_ws_bytes(int64_t M, int64_t N) {
  const int S = rowred_pk_splits<Op>(M, N);
  if (S <= 1) return 0;
  return (size_t)S * (size_t)M * (size_t)total_out_width<typename Op::Base>() * pk_slab_elem<Op>();
}

// Same contract as launch_rowred<Base, 2> (launch.hpp).
template <class Op, int RP>
int launch_rowred_pk_rp(const char* name, const Args& a, const Scal& sc, int64_t M, int64_t N,
                        const Outs& fin, void* ws, size_t ws_bytes, hipStream_t st) {
  using Base = typename Op::Base;
  const int S = rowred_pk_splits<Op>(M, N);
  const int64_t chunk = N > 0 ? chunk_of(N, S) : 0;
  const int64_t bx = (M + (int64_t)kBlock * 2 * RP - 1) / ((int64_t)kBlock * 2 * RP);
  dim3 grid((unsigned)bx, (unsigned)S, 1), block(kBlock, 1, 1);
  const EtaConsts bcx = pk_entry_consts<Op>(a);
  auto launch = [&](const Outs& o) {
    if constexpr (op_consts<Op>::value)
      rowred_pk_c_kernel<Op, RP><<<grid, block, 0, st>>>(a, sc, make_op_consts<Op>(a), M, N, chunk, o);
    else
      rowred_pk_kernel<Op, RP><<<grid, block, 0, st>>>(a, sc, M, N, chunk, o);
  };
  if (S == 1) {
    if (batching()) {
      const int rc = batch_record(rowred_pk_batch_flush<Op, RP>, PkEntry{a, sc, fin, M, N, chunk, grid.x, grid.y, bcx});
      return rc ? rc : check_launch(name);
    }
    launch(fin);
    return check_launch(name);
  }
  const size_t need = rowred_pk_ws_bytes<Op>(M, N);
  if (ws == nullptr || ws_bytes < need) {
    set_error("%s: workspace too small (%zu < %zu bytes)", name, ws_bytes, need);
    return DICP_ERR_WORKSPACE;
  }
  Outs part = fin;
  char* cur = reinterpret_cast<char*>(ws);
  for (int k = 0; k < Base::kNOut; ++k) {
    part.ptr[k] = fin.ptr[k] ? reinterpret_cast<float*>(cur) : nullptr;
    cur += (int64_t)S * M * Base::kOutW[k] * (int64_t)pk_slab_elem<Op>();
  }
  int rc;
  if (batching()) {
    rc = batch_record(rowred_pk_batch_flush<Op, RP>, PkEntry{a, sc, part, M, N, chunk, grid.x, grid.y, bcx});
    if (!rc) rc = check_launch(name);
  } else {
    launch(part);
    rc = check_launch(name);
  }
  if (rc) return rc;
  MergeSet ms;
  int nk = 0;
  int64_t nmax = 0;
  for (int k = 0; k < Base::kNOut; ++k) {
    if (!fin.ptr[k]) continue;
    ms.slab[nk] = part.ptr[k];
    ms.n[nk] = M * Base::kOutW[k];
    ms.k[nk] = k;
    nmax = ms.n[nk] > nmax ? ms.n[nk] : nmax;
    ++nk;
  }
  if (nk > 0) {
    const int64_t nb = (nmax + kBlock - 1) / kBlock;
    if (batching()) {
      rc = batch_record(merge_slabs_batch_flush,
                        MergeEntry{ms, fin, S, (unsigned)nb, (unsigned)nk, op_f64<Op>::value ? 1 : 0});
      return rc ? rc : check_launch(name);
    }
    if constexpr (op_f64<Op>::value)
      merge_slabs_f64_kernel<><<<dim3((unsigned)nb, (unsigned)nk), dim3(kBlock), 0, st>>>(ms, fin, S);
    else
      merge_slabs_kernel<false><<<dim3((unsigned)nb, (unsigned)nk), dim3(kBlock), 0, st>>>(ms, fin, S);
    rc = check_launch(name);
    if (rc) return rc;
  }
  return DICP_OK;
}

// ---- column phases of a row-split step (dicp_lddmm_euler_step_phase_f32) ----
// Phase 0: the nrows rows against n0 columns (the rank's own slice, Args columns), partial
// slabs into slots [0, S0) of the workspace; phase 1: against the n1 columns (coff + j) mod
// ntot, slots [S0, S0 + S1), then ONE merge of all S0 + S1 slots with the epilogue `fin`.
// Both phases compute S0 and S1 the same way (pk_phase_splits), so the slab layout agrees.
template <class Op, int RP>
__global__ __launch_bounds__(kBlock) DICP_FWD_PK_ATTR void rowred_pk_phase_kernel(Args args, Scal sc, int64_t M, int64_t N,
                                                                 int64_t chunk, Outs slabs, int64_t coff,
                                                                 int64_t ntot, typename op_consts<Op>::type cx) {
  // S = 2: always the slab store (a phase never applies the epilogue itself)
  if constexpr (op_f64<Op>::value)
    rowred_pk_body_f64<Op, RP, true>(args, sc, M, N, chunk, slabs, blockIdx.x, blockIdx.y, 2u, coff, ntot, cx);
  else
    rowred_pk_body<Op, RP, true>(args, sc, M, N, chunk, slabs, blockIdx.x, blockIdx.y, 2u, coff, ntot, cx);
}

template <class Op>
inline void pk_phase_splits(int64_t nrows, int64_t n0, int64_t n1, int& S0, int& S1) {
  S0 = n0 > 0 ? rowred_pk_splits<Op>(nrows, n0) : 0;
  S1 = n1 > 0 ? rowred_pk_splits<Op>(nrows, n1) : 0;
}

template <class Op>
size_t pk_phase_ws_bytes(int64_t nrows, int64_t n0, int64_t n1) {
  int S0, S1;
  pk_phase_splits<Op>(nrows, n0, n1, S0, S1);
  return (size_t)(S0 + S1) * (size_t)nrows * (size_t)total_out_width<typename Op::Base>() * pk_slab_elem<Op>();
}

template <class Op, int RP>
int launch_pk_phase_rp(const char* name, const Args& a, const Scal& sc, int64_t nrows, int64_t ncols,
                       int64_t coff, int64_t ntot, int slot0, int S, const Outs& slabs, hipStream_t st) {
  const int64_t chunk = chunk_of(ncols, S);
  const int64_t bx = (nrows + (int64_t)kBlock * 2 * RP - 1) / ((int64_t)kBlock * 2 * RP);
  Outs part = slabs;
  for (int k = 0; k < Op::Base::kNOut; ++k)
    if (part.ptr[k])
      part.ptr[k] = reinterpret_cast<float*>(reinterpret_cast<char*>(part.ptr[k]) +
                                             (int64_t)slot0 * nrows * Op::Base::kOutW[k] * (int64_t)pk_slab_elem<Op>());
  rowred_pk_phase_kernel<Op, RP><<<dim3((unsigned)bx, (unsigned)S, 1), dim3(kBlock), 0, st>>>(a, sc, nrows, ncols, chunk,
                                                                                           part, coff, ntot,
                                                                                           make_op_consts<Op>(a));
  return check_launch(name);
}

// phase 0: (a: rows and the n0 local columns); phase 1: (a: rows and the whole column array
// of ntot points, read from coff on, n1 of them), then the merge into `fin`.
template <class Op>
int launch_pk_phase(const char* name, int phase, const Args& a, const Scal& sc, int64_t nrows, int64_t n0,
                    int64_t n1, int64_t coff, int64_t ntot, const Outs& fin, void* ws, size_t ws_bytes,
                    hipStream_t st) {
  using Base = typename Op::Base;
  if (nrows <= 0) return DICP_OK;
  if (int rc = no_batch(name)) return rc;
  // the columns read are (coff + j) mod ntot, j < this phase's count: inside [0, ntot)
  const int64_t nc = phase == 0 ? n0 : n1;
  if (phase < 0 || phase > 1 || ntot <= 0 || coff < 0 || coff >= ntot || nc > ntot) {
    set_error("%s: bad column phase (phase %d, coff %lld, ncols %lld, ntot %lld)", name, phase,
              (long long)coff, (long long)nc, (long long)ntot);
    return DICP_ERR_INVALID;
  }
  int S0, S1;
  pk_phase_splits<Op>(nrows, n0, n1, S0, S1);
  const size_t need = pk_phase_ws_bytes<Op>(nrows, n0, n1);
  if (ws == nullptr || ws_bytes < need) {
    set_error("%s: workspace too small (%zu < %zu bytes)", name, ws_bytes, need);
    return DICP_ERR_WORKSPACE;
  }
  const int S = S0 + S1;
  Outs slabs = fin;
  char* cur = reinterpret_cast<char*>(ws);
  for (int k = 0; k < Base::kNOut; ++k) {
    slabs.ptr[k] = fin.ptr[k] ? reinterpret_cast<float*>(cur) : nullptr;
    cur += (int64_t)S * nrows * Base::kOutW[k] * (int64_t)pk_slab_elem<Op>();
  }
  const int64_t ncols = phase == 0 ? n0 : n1;
  const int slot0 = phase == 0 ? 0 : S0;
  const int Sp = phase == 0 ? S0 : S1;
  if (Sp > 0) {
    int rc;
    switch (pk_rp<Op>(nrows, ncols)) {
      case 2: rc = launch_pk_phase_rp<Op, 2>(name, a, sc, nrows, ncols, coff, ntot, slot0, Sp, slabs, st); break;
      default: rc = launch_pk_phase_rp<Op, 1>(name, a, sc, nrows, ncols, coff, ntot, slot0, Sp, slabs, st); break;
    }
    if (rc) return rc;
  }
  if (phase == 0) return DICP_OK;
  MergeSet ms;
  int nk = 0;
  int64_t nmax = 0;
  for (int k = 0; k < Base::kNOut; ++k) {
    if (!fin.ptr[k]) continue;
    ms.slab[nk] = slabs.ptr[k];
    ms.n[nk] = nrows * Base::kOutW[k];
    ms.k[nk] = k;
    nmax = ms.n[nk] > nmax ? ms.n[nk] : nmax;
    ++nk;
  }
  if (nk == 0) return DICP_OK;
  const int64_t nb = (nmax + kBlock - 1) / kBlock;
  if constexpr (op_f64<Op>::value)
    merge_slabs_f64_kernel<><<<dim3((unsigned)nb, (unsigned)nk), dim3(kBlock), 0, st>>>(ms, fin, S);
  else
    merge_slabs_kernel<false><<<dim3((unsigned)nb, (unsigned)nk), dim3(kBlock), 0, st>>>(ms, fin, S);
  return check_launch(name);
}

template <class Op>
int launch_rowred_pk(const char* name, const Args& a, const Scal& sc, int64_t M, int64_t N,
                     const Outs& fin, void* ws, size_t ws_bytes, hipStream_t st) {
  if (M <= 0) return DICP_OK;
  switch (pk_rp<Op>(M, N)) {
#if DICP_PK_RP_EXTRA
    case 4: return launch_rowred_pk_rp<Op, 4>(name, a, sc, M, N, fin, ws, ws_bytes, st);
    case 3: return launch_rowred_pk_rp<Op, 3>(name, a, sc, M, N, fin, ws, ws_bytes, st);
#endif
    case 2: return launch_rowred_pk_rp<Op, 2>(name, a, sc, M, N, fin, ws, ws_bytes, st);
    default: return launch_rowred_pk_rp<Op, 1>(name, a, sc, M, N, fin, ws, ws_bytes, st);
  }
}

}  // namespace dicp
