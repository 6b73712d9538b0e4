// GMM EM-step reductions (GaussianMixtureUnif.EM_step_torch, diffICP/core/GMM.py:236-325)
// for gfx950.  Three passes, each one launch (+ a tiny finalize/merge launch):
//   E  (rows n, cols c): T_n = LSE_c t_nc and responsibility-weighted row sums  (GMM.py:263-270,
//      :296 NDsigma2 with the OLD mu, :303 Y, :312-314 Cfe terms)
//   M  (rows c, cols n): log sum_n gamma_nc and the gamma-weighted mean of x  (GMM.py:287, :293)
//   T  (rows n, cols c): targets / free-energy sums with OLD gamma, NEW mu, w  (GMM.py:303-314)
// LSE passes make one exp2 sweep per pair, shifted by the maximum of the chunk's first 64
// columns (a tile that overflows is re-referenced), all in the log2 domain; column chunks (split
// mode) carry (shift, sum, acc) partials merged with max-rescaling in a fixed order ->
// deterministic, no atomics.
#include "launch.hpp"
#include "lddmm_ops.hpp"
#include "packed.hpp"

#include <type_traits>

using namespace dicp;

namespace {

#ifndef DICP_LSE_RG
#define DICP_LSE_RG 2
#endif
constexpr int kRG = 2;             // rows per thread (targets pass)
constexpr int kLseRG = DICP_LSE_RG;  // rows per thread (E and M passes)
// the E-step against many components (the two-set match: C = N = 10^5) with 4 rows per thread:
// two independent packed pairs per column hide the dependent v_pk chain's hazard stalls (100k x
// 100k: 2.63 against 2.73 ms with one pair); against a few hundred (the atlas GMMs, C = 512) one
// pair per thread keeps twice the workgroups (0.136 against 0.142 ms at 640k x 512, and the
// M-step, rows = components, 0.146 against 0.217 ms) -- profiles/r05_ab_lse_pk.json
constexpr int64_t kLseE4MinCols = 8192;
// more column-chunk partials per row than this: the one-wave-per-row merge
constexpr int kWaveMergeMinSplits = 64;

// ---------------------------------------------------------------------------------------
// LSE row-reduction skeleton: part[(s*M + i)*(2+NACC) + ...] = {m, l, acc...} with
// m = the chunk's shift (log2 domain), l = sum_j 2^(t_ij - m), acc = Op::accum weighted sums.
// One exp2 sweep: the shift m is the exact maximum over the chunk's first kLseShiftCols
// columns (a logit-only pass) -- or, with a hint (the previous EM step's T2), near the row's
// LSE -- and a logit far above it re-references the row's sums (adaptive, see kLseSlack).
// Op interface (Row carries k = the row's exponent constant minus the shift):
//   CW4 / NACC / kShifted (the acc slot holding sum e (t - m), re-referenced on merges; -1)
//   load_row(a, sc, i, row), base(row) (the row constant of the logit), load_col(a, sc, j, rec)
//   tm(sc, row, rec) = t - m, accum(rec, tm, e, acc), finalize(sc, a, i, m, l, acc, outs)
// ---------------------------------------------------------------------------------------
// Re-referencing, adaptive per workgroup: first at the tile's end (a partial above
// kLseOverflow -- a term above 2^56, or inf / NaN -- sends the row's tile through again,
// re-referenced to its exact maximum: free while events are rare); after lse_adapt() tiles
// that needed it anywhere in the workgroup, a per-pair test (a logit more than kLseSlack above
// the shift re-references the row's sums in the loop, ~20 instructions per event, a compare per
// pair).  Measured at 100k x 100k (tools/probes/estep_sigma.py): tile-end only 2.54 ms at sigma
// 0.05 but 5.9 at 0.01 (a random 64-column sample then sits ~450 log2 units below the nearest
// component: events in most tiles of most waves, each a tile summed again); per-pair only
// 3.40-3.70 ms at every sigma.
constexpr float kLseOverflow = 0x1p64f;
constexpr float kLseSlack = 64.f;
// With the hint: a workgroup where at least 1 / kLseClampedShare of the threads hold a row whose
// hint was clamped (lse_hint_clamped) tests per pair from the start; the others count
// kLseAdaptHinted eventful tiles before switching (a clamped row re-references in the few tiles
// holding its nearest columns; a stale hint rarely at all).
// Measured at 100k x 100k with the hint: tile-end 2.41 / 3.34 / 5.77 ms at sigma 0.05 / 0.02 /
// 0.01, per pair 3.42 / 3.41 / 3.49 (profiles/r05_estep_adapt_count_rule.jsonl); this rule 2.40-2.45
// / 3.46-3.49 / 3.46, the bench workload's E-step 3.30 ms (tile-end 3.05, per pair 3.46, counting
// alone 3.66; profiles/r05_estep_adapt.jsonl).
constexpr int kLseAdaptHinted = 4;
constexpr int kLseClampedShare = 4;
// columns of the chunk's first tile whose logits set the shift (the exact maximum over them):
// 64 of the <= 256 staged -- a 1/28 logit overhead at the 100k two-set E-step's ~1800-column
// chunks instead of 1/7; a row whose nearest components come later is re-referenced once
constexpr int kLseShiftCols = 64;
// a dead component (w = -inf) enters with this logit instead of -inf, so that e (t - m) is
// 0 * finite (the e-weighted sums stay finite) and a dead-only shift is re-referenced like any
// other.  Not larger: a re-reference moves the shift m by the tile's maximum of t - m, and m
// + mt is rounded to the float grid at m -- below |m| ~ 2^31 that rounding (<= 64) cannot leave
// a term above the overflow test; at -1e20 it was ~4e12 and the tile stayed at +inf.  So live
// components farther than ~1.2e4 sigma from a row weigh like dead ones there (both vanish
// against any component nearer than that), and rows farther than ~5e4 sigma from every
// component are outside the single sweep's range (the log-likelihood there is below -1e9).
constexpr float kLseDead = -1e8f;

// The shift of a row given a hint of its LSE (the previous EM step's T2): the row's largest
// term then sits near 2^8, every term of the chunk stays below the 2^56 re-reference test
// unless the logits rose by ~48 since the hint, and the clamp to [m64, m64 + 100] (m64 = the
// exact maximum of the chunk's first 64 logits) keeps any hint safe: the shift is never below
// a logit of the chunk, and never so far above one that it underflows (2^-100 > 2^-126);
// terms more than 126 below the shift are below 2^-126 of the row's sum, as in any shift.
// A non-finite hint leaves m64.
__device__ __forceinline__ float lse_hinted_shift(float m64, float hint) {
  if (!(hint > -1e30f && hint < 1e30f)) return m64;
  return fminf(fmaxf(hint - 8.f, m64), m64 + 100.f);
}
// The hint sits beyond the clamp: the row's nearest columns are far closer than the sampled
// ones, and re-reference events are to be expected in the chunk.
__device__ __forceinline__ bool lse_hint_clamped(float m64, float hint) {
  return hint > -1e30f && hint < 1e30f && hint - 8.f > m64 + 100.f;
}

// ---- the bound shift (the hinted many-component E-step: C >= kLseE4MinCols) ----------------
// Every logit is at most its column's distance-0 value, t_nc <= nc v_c = w2_c, so the shift
// min(hint - 8, U) with U = max_c nc v_c - kLseBoundSlack (a tiny pass over the C columns,
// lse_bound_kernel) can never overflow a sum: no logit-only sample pass and no re-reference
// events, whatever sigma (a 64-column sample sits hundreds of log2 units below a row's nearest
// component at the two-set bench's converged sigma).  The price
// is underflow where a row's LSE lies far below its shift (nearest component beyond ~11 sigma,
// or a stale-high hint): terms more than 126 below the shift flush to 0, so a row whose LSE
// ends more than kLseBoundGap below its shift is appended to a list (the finalize) and summed
// again exactly -- two sweeps, one workgroup per listed row (lse_fixup_kernel).
constexpr float kLseBoundSlack = 8.f;
constexpr float kLseBoundGap = 80.f;
__device__ __forceinline__ float lse_bound_shift(float U, const float* hint, int64_t i) {
  if (hint == nullptr) return U;
  const float h = hint[i];
  if (!(h > -1e30f && h < 1e30f)) return U;
  return fminf(h - 8.f, U);
}

// Store a chunk partial {m, l, acc}.  The merge weighs a partial by 2^(m_s - max m): with the
// shift up to 100 above a chunk's largest term (a clamped hint) and the sums up to 2^77 (terms
// below the re-reference slack), that factor could underflow while the partial's share did not
// (a stale-high hint lost up to 90% of a row's mass: test_estep_reref_modes).  So a partial
// whose sum lies outside [2^-24, 2^24] is stored normalised to l in [0.5, 1): m + e for
// l = f 2^e, the sums scaled by 2^-e (exact), the shifted slot re-referenced to m + e; the
// others as they are (their m is within 24 of their own log-sum).  An empty partial (l = 0)
// stores the shift -inf and is skipped; a NaN one (NaN rows) stores the shift NaN, which both
// merges turn into NaN sums (fmaxf skips it for the maximum, exp2(NaN - max) is NaN).
template <int NACC, int KS>
__device__ __forceinline__ void lse_store_part(float* dst, float m, const float* tot) {
  const float l = tot[0];
  if (l != l) {   // NaN inputs (x or mu): a NaN shift, so the merge carries NaN on to T and T2
    dst[0] = __builtin_nanf("");
#pragma unroll
    for (int k = 0; k <= NACC; ++k) dst[1 + k] = tot[k];
    return;
  }
  if (l == 0.f) {
    dst[0] = -__builtin_huge_valf();
#pragma unroll
    for (int k = 0; k <= NACC; ++k) dst[1 + k] = tot[k];
    return;
  }
  if (l >= 0x1p-24f && l <= 0x1p24f) {
    dst[0] = m;
#pragma unroll
    for (int k = 0; k <= NACC; ++k) dst[1 + k] = tot[k];
    return;
  }
  int e;
  (void)frexpf(l, &e);
  const float fe = (float)e;
  dst[0] = m + fe;
#pragma unroll
  for (int k = 0; k <= NACC; ++k) {
    float v = tot[k];
    if (KS >= 0 && k == KS + 1) v = fmaf(-fe, l, v);   // sum e (t - m) -> sum e (t - (m + e))
    dst[1 + k] = ldexpf(v, -e);
  }
}

template <class Op, int R, bool BOUND = false>
__global__ __launch_bounds__(kBlock) void lse_rowred_kernel(Args args, Scal sc,
                                                            int64_t M, int64_t N, int64_t chunk,
                                                            float* __restrict__ part, int adapt) {
  constexpr int CW4 = Op::CW4;
  constexpr int NACC = Op::NACC;
  constexpr int KS = Op::kShifted;
  constexpr int W = 2 + NACC;
  __shared__ float4 lds[kTile * CW4];
  const int tid = threadIdx.x;
  const int64_t ibase = (int64_t)blockIdx.x * (kBlock * R) + tid;
  typename Op::Row row[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    int64_t i = ibase + (int64_t)r * kBlock;
    if (i >= M) i = M - 1;
    Op::load_row(args, sc, i, row[r]);
    row[r].k = Op::base(row[r]);
  }
  const int64_t j0 = (int64_t)blockIdx.y * chunk;
  int64_t j1 = j0 + chunk;
  if (j1 > N) j1 = N;

  // the shift: exact maximum of the logits over the chunk's first kLseShiftCols columns
  float m[R];
#pragma unroll
  for (int r = 0; r < R; ++r) m[r] = -__builtin_huge_valf();
  if (j0 < j1) {
    const int cnt = (int)((j1 - j0) < kTile ? (j1 - j0) : kTile);
    if (tid < cnt) Op::load_col(args, sc, j0 + tid, reinterpret_cast<float*>(&lds[tid * CW4]));
    __syncthreads();
    const int ns = BOUND ? 0 : (cnt < kLseShiftCols ? cnt : kLseShiftCols);
#pragma unroll 2
    for (int t = 0; t < ns; ++t) {
      const float* rec = reinterpret_cast<const float*>(&lds[t * CW4]);
#pragma unroll
      for (int r = 0; r < R; ++r) m[r] = fmaxf(m[r], Op::tm(sc, row[r], rec));
    }
  }
  // -inf (a dead row of the M-step: w2 = -inf): shift 0, its terms are all 0
  const float* hint = Op::hint(args);
  bool clamped = false;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if (m[r] == -__builtin_huge_valf()) m[r] = 0.f;
    if (BOUND) {   // the bound shift min(hint - 8, U): no sample pass, never an overflow
      int64_t i = ibase + (int64_t)r * kBlock;
      if (i >= M) i = M - 1;
      m[r] = lse_bound_shift(args.r2[0], hint, i);
    } else if (hint != nullptr) {   // the row's expected LSE: m = clamp(hint - 8, m64, m64 + 100)
      int64_t i = ibase + (int64_t)r * kBlock;
      if (i >= M) i = M - 1;
      clamped = clamped || lse_hint_clamped(m[r], hint[i]);
      m[r] = lse_hinted_shift(m[r], hint[i]);
    }
    row[r].k -= m[r];
  }

  float tot[R][NACC + 1];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int k = 0; k <= NACC; ++k) tot[r][k] = 0.f;
  bool pair_mode = adapt <= 0;
  int reref_tiles = 0;
  if (hint != nullptr) {   // a hinted workgroup: per pair at once where many rows' hints were
    // clamped (their nearest columns lie far above the sample); else count more eventful tiles
    if (__syncthreads_count(clamped) * kLseClampedShare >= kBlock) pair_mode = true;
    else if (adapt > 0 && adapt < kLseAdaptHinted) adapt = kLseAdaptHinted;
  }
  bool first = true;   // the first tile is already in LDS
  for (int64_t jt = j0; jt < j1; jt += kTile) {
    const int cnt = (int)((j1 - jt) < kTile ? (j1 - jt) : kTile);
    if (!first) {
      if (tid < cnt) Op::load_col(args, sc, jt + tid, reinterpret_cast<float*>(&lds[tid * CW4]));
      __syncthreads();
    }
    first = false;
    // a tile of equal weights (every column's v = v0): its sum e v is v0 sum e (lse_uniform)
    float v0 = 0.f;
    bool uni = false;
    if (Op::kUni >= 0 && R >= 4) {   // the many-component E-step (kLseE4MinCols) only
      v0 = Op::uni_value(args, sc, jt);
      uni = !__syncthreads_or(tid < cnt && Op::uni_value(args, sc, jt + tid) != v0);
    }
    float acc[R][NACC + 1];
    auto pass = [&](auto U, auto P, int r0, int r1) {
      constexpr bool kU = decltype(U)::value, kP = decltype(P)::value;
#pragma unroll 2
      for (int t = 0; t < cnt; ++t) {
        const float* rec = reinterpret_cast<const float*>(&lds[t * CW4]);
#pragma unroll
        for (int r = 0; r < R; ++r) {
          if (r < r0 || r >= r1) continue;
          float tm = Op::tm(sc, row[r], rec);
          if (kP && tm > kLseSlack) {   // re-reference the row to tm (as lse_reref_lane_t)
            const float f = fast_exp2(-tm), t0 = tot[r][0], a0 = acc[r][0];
#pragma unroll
            for (int q = 0; q <= NACC; ++q) {
              float b = tot[r][q], a = acc[r][q];
              if (KS >= 0 && q == KS + 1) {
                b = fmaf(-tm, t0, b);
                a = fmaf(-tm, a0, a);
              }
              tot[r][q] = b * f;
              acc[r][q] = a * f;
            }
            m[r] += tm;
            row[r].k -= tm;
            tm = 0.f;
          }
          const float e = fast_exp2(tm);
          acc[r][0] += e;
          Op::template accum<kU>(rec, tm, e, acc[r] + 1);
        }
      }
      if (kU) {
#pragma unroll
        for (int r = 0; r < R; ++r)
          if (r >= r0 && r < r1) acc[r][1 + Op::kUni] = v0 * acc[r][0];
      }
    };
    auto run = [&](auto P, int r0, int r1) {
      if (uni) pass(std::true_type{}, P, r0, r1);
      else pass(std::false_type{}, P, r0, r1);
    };
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int k = 0; k <= NACC; ++k) acc[r][k] = 0.f;
    bool reref = false;
    if (pair_mode) {
      run(std::true_type{}, 0, R);
    } else {
      run(std::false_type{}, 0, R);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (!(acc[r][0] <= kLseOverflow)) {   // re-reference the row to the tile's maximum
          reref = true;
          float mt = -__builtin_huge_valf();
          for (int t = 0; t < cnt; ++t)
            mt = fmaxf(mt, Op::tm(sc, row[r], reinterpret_cast<const float*>(&lds[t * CW4])));
          const float f = fast_exp2(-mt), l0 = tot[r][0];
#pragma unroll
          for (int k = 0; k <= NACC; ++k) {
            float b = tot[r][k];
            if (KS >= 0 && k == KS + 1) b = fmaf(-mt, l0, b);   // sum e (t - m): t - m' = (t - m) - mt
            tot[r][k] = f == 0.f ? 0.f : f * b;
            acc[r][k] = 0.f;
          }
          m[r] += mt;
          row[r].k -= mt;
          run(std::false_type{}, r, r + 1);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int k = 0; k <= NACC; ++k) tot[r][k] += acc[r][k];
    if (__syncthreads_or(reref) && ++reref_tiles >= adapt) pair_mode = true;
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t i = ibase + (int64_t)r * kBlock;
    if (i >= M) continue;
    lse_store_part<NACC, KS>(part + ((int64_t)blockIdx.y * M + i) * W, m[r], tot[r]);
  }
}

// The same pass with the thread's rows packed in H float2 pairs (Op::Row2, tm2, accum2): the
// logit, the row sums and their shift arithmetic as v_pk_fma_f32 (two rows per instruction),
// the exps scalar -- ~13 packed instructions + 2 exp per column for two rows against 28 scalar
// VALU + 2 exp (E-step).  Same rows, same order, same fmas: bitwise the scalar kernel's partials
// (tests/test_gpu_em.py).  A pair whose tile overflows in either row is summed again as a pair,
// only the overflowing row(s) re-referenced (the other row's partials come out unchanged).
// Re-reference one lane (c = 0: .x, 1: .y) of a packed row pair to a logit tm above the shift
// by more than kLseSlack: the row's sums so far (tile and total) are scaled by 2^-tm, the
// e (t - m) sum also moved by -tm times the row's count, and the shift rises by tm (then tm = 0).
template <int NACC, int KS, int C>
__device__ __forceinline__ void lse_reref_lane_t(f2& tm2, f2& m2, f2& k2, f2* tot, f2* acc) {
  const float tm = C ? tm2.y : tm2.x;
  if (!(tm > kLseSlack)) return;
  const float f = fast_exp2(-tm);
  const float t0 = C ? tot[0].y : tot[0].x, a0 = C ? acc[0].y : acc[0].x;
#pragma unroll
  for (int q = 0; q <= NACC; ++q) {
    float b = C ? tot[q].y : tot[q].x, a = C ? acc[q].y : acc[q].x;
    if (KS >= 0 && q == KS + 1) {
      b = fmaf(-tm, t0, b);
      a = fmaf(-tm, a0, a);
    }
    b *= f;
    a *= f;
    if (C) { tot[q].y = b; acc[q].y = a; } else { tot[q].x = b; acc[q].x = a; }
  }
  if (C) { m2.y += tm; k2.y -= tm; tm2.y = 0.f; } else { m2.x += tm; k2.x -= tm; tm2.x = 0.f; }
}

template <class Op, int H, bool BOUND = false>
__global__ __launch_bounds__(kBlock) void lse_rowred_pk_kernel(Args args, Scal sc,
                                                               int64_t M, int64_t N, int64_t chunk,
                                                               float* __restrict__ part, int adapt) {
  constexpr int R = 2 * H;
  constexpr int CW4 = Op::CW4;
  constexpr int NACC = Op::NACC;
  constexpr int KS = Op::kShifted;
  constexpr int W = 2 + NACC;
  constexpr float kNinf = -__builtin_huge_valf();
  __shared__ float4 lds[kTile * CW4];
  const int tid = threadIdx.x;
  const int64_t ibase = (int64_t)blockIdx.x * (kBlock * R) + tid;
  typename Op::Row2 row[H];
#pragma unroll
  for (int h = 0; h < H; ++h) {
    typename Op::Row rr[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      int64_t i = ibase + (int64_t)(2 * h + c) * kBlock;
      if (i >= M) i = M - 1;
      Op::load_row(args, sc, i, rr[c]);
    }
    Op::pack(rr[0], rr[1], row[h]);
    row[h].k = Op::base2(row[h]);
  }
  const int64_t j0 = (int64_t)blockIdx.y * chunk;
  int64_t j1 = j0 + chunk;
  if (j1 > N) j1 = N;

  f2 m[H];
#pragma unroll
  for (int h = 0; h < H; ++h) m[h] = splat(kNinf);
  if (j0 < j1) {
    const int cnt = (int)((j1 - j0) < kTile ? (j1 - j0) : kTile);
    if (tid < cnt) Op::load_col(args, sc, j0 + tid, reinterpret_cast<float*>(&lds[tid * CW4]));
    __syncthreads();
    const int ns = BOUND ? 0 : (cnt < kLseShiftCols ? cnt : kLseShiftCols);
#pragma unroll 2
    for (int t = 0; t < ns; ++t) {
      const float* rec = reinterpret_cast<const float*>(&lds[t * CW4]);
#pragma unroll
      for (int h = 0; h < H; ++h) {
        const f2 tm = Op::tm2(sc, row[h], rec);
        m[h] = f2{fmaxf(m[h].x, tm.x), fmaxf(m[h].y, tm.y)};
      }
    }
  }
  const float* hint = Op::hint(args);
  bool clamped = false;
#pragma unroll
  for (int h = 0; h < H; ++h) {
    if (m[h].x == kNinf) m[h].x = 0.f;
    if (m[h].y == kNinf) m[h].y = 0.f;
    if (BOUND) {   // the bound shift (as lse_rowred_kernel)
      int64_t i0 = ibase + (int64_t)(2 * h) * kBlock, i1 = ibase + (int64_t)(2 * h + 1) * kBlock;
      if (i0 >= M) i0 = M - 1;
      if (i1 >= M) i1 = M - 1;
      const float U = args.r2[0];
      m[h] = f2{lse_bound_shift(U, hint, i0), lse_bound_shift(U, hint, i1)};
    } else if (hint != nullptr) {
      int64_t i0 = ibase + (int64_t)(2 * h) * kBlock, i1 = ibase + (int64_t)(2 * h + 1) * kBlock;
      if (i0 >= M) i0 = M - 1;
      if (i1 >= M) i1 = M - 1;
      clamped = clamped || lse_hint_clamped(m[h].x, hint[i0]) || lse_hint_clamped(m[h].y, hint[i1]);
      m[h] = f2{lse_hinted_shift(m[h].x, hint[i0]), lse_hinted_shift(m[h].y, hint[i1])};
    }
    row[h].k = row[h].k - m[h];
  }

  f2 tot[H][NACC + 1];
#pragma unroll
  for (int h = 0; h < H; ++h)
#pragma unroll
    for (int k = 0; k <= NACC; ++k) tot[h][k] = splat(0.f);
  bool pair_mode = adapt <= 0;
  int reref_tiles = 0;
  if (hint != nullptr) {   // a hinted workgroup: per pair at once where many rows' hints were
    // clamped (their nearest columns lie far above the sample); else count more eventful tiles
    if (__syncthreads_count(clamped) * kLseClampedShare >= kBlock) pair_mode = true;
    else if (adapt > 0 && adapt < kLseAdaptHinted) adapt = kLseAdaptHinted;
  }
  bool first = true;
  for (int64_t jt = j0; jt < j1; jt += kTile) {
    const int cnt = (int)((j1 - jt) < kTile ? (j1 - jt) : kTile);
    if (!first) {
      if (tid < cnt) Op::load_col(args, sc, jt + tid, reinterpret_cast<float*>(&lds[tid * CW4]));
      __syncthreads();
    }
    first = false;
    float v0 = 0.f;
    bool uni = false;
    if (Op::kUni >= 0 && H >= 2) {   // the many-component E-step (kLseE4MinCols) only
      v0 = Op::uni_value(args, sc, jt);
      uni = !__syncthreads_or(tid < cnt && Op::uni_value(args, sc, jt + tid) != v0);
    }
    f2 acc[H][NACC + 1];
    // U: uniform-weight tile; P: per-pair re-reference test (else: the tile-end test);
    // [h0, h1): the row pairs summed (a tile-end re-reference sums one pair again)
    auto pass = [&](auto U, auto P, int h0, int h1) {
      constexpr bool kU = decltype(U)::value, kP = decltype(P)::value;
#pragma unroll 2
      for (int t = 0; t < cnt; ++t) {
        const float* rec = reinterpret_cast<const float*>(&lds[t * CW4]);
#pragma unroll
        for (int h = 0; h < H; ++h) {
          if (h < h0 || h >= h1) continue;
          f2 tm = Op::tm2(sc, row[h], rec);
          if (kP && (tm.x > kLseSlack || tm.y > kLseSlack)) {   // re-reference the row(s) to tm
            lse_reref_lane_t<NACC, KS, 0>(tm, m[h], row[h].k, tot[h], acc[h]);
            lse_reref_lane_t<NACC, KS, 1>(tm, m[h], row[h].k, tot[h], acc[h]);
          }
          const f2 e = f2{fast_exp2(tm.x), fast_exp2(tm.y)};
          acc[h][0] = acc[h][0] + e;
          Op::template accum2<kU>(rec, tm, e, acc[h] + 1);
        }
      }
      if (kU) {
#pragma unroll
        for (int h = 0; h < H; ++h)
          if (h >= h0 && h < h1) acc[h][1 + Op::kUni] = splat(v0) * acc[h][0];
      }
    };
    auto run = [&](auto P, int h0, int h1) {
      if (uni) pass(std::true_type{}, P, h0, h1);
      else pass(std::false_type{}, P, h0, h1);
    };
#pragma unroll
    for (int h = 0; h < H; ++h)
#pragma unroll
      for (int k = 0; k <= NACC; ++k) acc[h][k] = splat(0.f);
    bool reref = false;
    if (pair_mode) {
      run(std::true_type{}, 0, H);
    } else {
      run(std::false_type{}, 0, H);
#pragma unroll
      for (int h = 0; h < H; ++h) {   // tile-end test: a term above 2^56 (or inf / NaN)
        const bool ox = !(acc[h][0].x <= kLseOverflow), oy = !(acc[h][0].y <= kLseOverflow);
        if (ox || oy) {
          reref = true;
          f2 mt = splat(kNinf);
          for (int t = 0; t < cnt; ++t) {
            const f2 v = Op::tm2(sc, row[h], reinterpret_cast<const float*>(&lds[t * CW4]));
            mt = f2{fmaxf(mt.x, v.x), fmaxf(mt.y, v.y)};
          }
          // the row of the pair that did not overflow keeps its shift (its sums come out
          // unchanged: scaled by 1, summed again in the same order)
          mt = f2{ox ? mt.x : 0.f, oy ? mt.y : 0.f};
          const f2 f = f2{fast_exp2(-mt.x), fast_exp2(-mt.y)}, l0 = tot[h][0];
#pragma unroll
          for (int k = 0; k <= NACC; ++k) {
            f2 b = tot[h][k];
            if (KS >= 0 && k == KS + 1) b = pk_fma(-mt, l0, b);
            tot[h][k] = f2{f.x == 0.f ? 0.f : f.x * b.x, f.y == 0.f ? 0.f : f.y * b.y};
            acc[h][k] = splat(0.f);
          }
          m[h] = m[h] + mt;
          row[h].k = row[h].k - mt;
          run(std::false_type{}, h, h + 1);
        }
      }
    }
#pragma unroll
    for (int h = 0; h < H; ++h)
#pragma unroll
      for (int k = 0; k <= NACC; ++k) tot[h][k] = tot[h][k] + acc[h][k];
    // lse_adapt() tiles that needed a tile-end re-reference somewhere in the workgroup: the
    // rest of the chunk tests per pair (events are then common: small sigma against the shift)
    if (__syncthreads_or(reref) && ++reref_tiles >= adapt) pair_mode = true;
  }
#pragma unroll
  for (int h = 0; h < H; ++h)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int64_t i = ibase + (int64_t)(2 * h + c) * kBlock;
      if (i >= M) continue;
      float t[NACC + 1];
#pragma unroll
      for (int k = 0; k <= NACC; ++k) t[k] = c ? tot[h][k].y : tot[h][k].x;
      lse_store_part<NACC, KS>(part + ((int64_t)blockIdx.y * M + i) * W, c ? m[h].y : m[h].x, t);
    }
}

// Tiles with a tile-end re-reference (anywhere in the workgroup) before the rest of the chunk
// tests per pair (0: per pair from the start); env DICP_LSE_ADAPT, option "lse_adapt"
int& lse_adapt_ref() {
  static int v = [] {
    const char* e = getenv("DICP_LSE_ADAPT");
    return e ? atoi(e) : 1;
  }();
  return v;
}

int& lse_bound_ref() {
  static int v = [] {
    const char* e = getenv("DICP_LSE_BOUND");
    return e ? atoi(e) : 1;
  }();
  return v;
}

int& lse_pk_ref() {
#ifndef DICP_LSE_PK
#define DICP_LSE_PK 1
#endif
  static int v = DICP_LSE_PK;
  return v;
}

// The bound shift's check at the merge (fix != NULL: {U, count, -, -, rows...} in the
// workspace, lse_bound_kernel): a row whose LSE ended more than kLseBoundGap below its shift may
// have lost terms to underflow -- appended to the list that lse_fixup_kernel sums again.  NaN
// rows are not listed (their NaN goes on to T / T2).
__device__ __forceinline__ void lse_bound_check(int* fix, const Args& args, int64_t i, float mx, float l) {
  if (fix == nullptr || !(l == l)) return;
  const float m0 = lse_bound_shift(reinterpret_cast<const float*>(fix)[0], args.r1, i);
  if (!(mx + log2f(l) >= m0 - kLseBoundGap)) fix[4 + atomicAdd(&fix[1], 1)] = (int)i;
}

// Merge S chunk partials of each row (fixed order) and finalize through Op::finalize.
template <class Op>
__global__ __launch_bounds__(kBlock) void lse_finalize_kernel(const float* __restrict__ part,
                                                              int64_t M, int S, Args args,
                                                              Scal sc, Outs outs, int* fix) {
  constexpr int NACC = Op::NACC;
  constexpr int W = 2 + NACC;
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= M) return;
  float mx = -__builtin_huge_valf();
  for (int s = 0; s < S; ++s) mx = fmaxf(mx, part[((int64_t)s * M + i) * W]);
  float l = 0.f, acc[NACC > 0 ? NACC : 1];
#pragma unroll
  for (int k = 0; k < NACC; ++k) acc[k] = 0.f;
  for (int s = 0; s < S; ++s) {
    const float* p = part + ((int64_t)s * M + i) * W;
    if (p[0] == -__builtin_huge_valf()) continue;
    const float f = fast_exp2(p[0] - mx);
    l = fmaf(f, p[1], l);
#pragma unroll
    for (int k = 0; k < NACC; ++k) {
      float a = p[2 + k];
      if (k == Op::kShifted) a = fmaf(p[0] - mx, p[1], a);  // re-reference t - m_s -> t - mx
      acc[k] = fmaf(f, a, acc[k]);
    }
  }
  lse_bound_check(fix, args, i, mx, l);
  Op::finalize(sc, args, i, mx, l, acc, outs);
}

// Many chunk partials per row (the M-step: C = 256-512 component rows against 10^5-10^6
// points, so ~10^3 column chunks fill the chip): one wave per row, each lane merging a strided
// share of the chunks, then a fixed xor tree across the lanes.  (The one-thread-per-row merge
// above reads the S partials of a row one after the other: at S ~ 1250 that latency chain,
// not the pair pass, was the M-step's time.)  Deterministic: fixed shares, fixed tree.
template <int NACC, int kShifted>
struct LsePart {
  float m, l, a[NACC > 0 ? NACC : 1];
  __device__ void clear() {
    m = -__builtin_huge_valf();
    l = 0.f;
#pragma unroll
    for (int k = 0; k < NACC; ++k) a[k] = 0.f;
  }
  // this <- this (+) (m2, l2, a2), both referenced to their own maxima
  __device__ void merge(float m2, float l2, const float* a2) {
    if (m2 == -__builtin_huge_valf()) return;
    if (m == -__builtin_huge_valf()) {
      m = m2;
      l = l2;
#pragma unroll
      for (int k = 0; k < NACC; ++k) a[k] = a2[k];
      return;
    }
    const float mn = fmaxf(m, m2);
    const float f1 = fast_exp2(m - mn), f2 = fast_exp2(m2 - mn);
#pragma unroll
    for (int k = 0; k < NACC; ++k) {
      float x1 = a[k], x2 = a2[k];
      if (k == kShifted) {  // re-reference sum e (t - m_s) to the merged maximum
        x1 = fmaf(m - mn, l, x1);
        x2 = fmaf(m2 - mn, l2, x2);
      }
      a[k] = fmaf(f1, x1, f2 * x2);
    }
    l = fmaf(f1, l, f2 * l2);
    m = mn;
  }
};

template <class Op>
__global__ __launch_bounds__(kBlock) void lse_finalize_wave_kernel(const float* __restrict__ part,
                                                                   int64_t M, int S, Args args,
                                                                   Scal sc, Outs outs, int* fix) {
  constexpr int NACC = Op::NACC;
  constexpr int W = 2 + NACC;
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6);
  if (i >= M) return;  // whole wave leaves together
  LsePart<NACC, Op::kShifted> acc;
  acc.clear();
  for (int s = lane; s < S; s += 64) {
    const float* p = part + ((int64_t)s * M + i) * W;
    acc.merge(p[0], p[1], p + 2);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    float a2[NACC > 0 ? NACC : 1];
#pragma unroll
    for (int k = 0; k < NACC; ++k) a2[k] = __shfl_xor(acc.a[k], off, 64);
    const float m2 = __shfl_xor(acc.m, off, 64), l2 = __shfl_xor(acc.l, off, 64);
    acc.merge(m2, l2, a2);
  }
  if (lane == 0) {
    lse_bound_check(fix, args, i, acc.m, acc.l);
    Op::finalize(sc, args, i, acc.m, acc.l, acc.a, outs);
  }
}

// U = max_c Op::col_bound(c) - kLseBoundSlack over the N columns (one 1024-thread workgroup
// reading one float per column; the maximum is order-free) and the list's count reset:
// fix = {U, count, -, -, rows...}
constexpr int kBoundThreads = 1024;
template <class Op>
__global__ __launch_bounds__(kBoundThreads) void lse_bound_kernel(Args args, Scal sc, int64_t N, int* fix) {
  __shared__ float red[kBoundThreads];
  const int tid = threadIdx.x;
  float mx = -__builtin_huge_valf();
  for (int64_t j = tid; j < N; j += kBoundThreads) mx = fmaxf(mx, Op::col_bound(args, sc, j));
  red[tid] = mx;
  __syncthreads();
  for (int o = kBoundThreads / 2; o > 0; o >>= 1) {
    if (tid < o) red[tid] = fmaxf(red[tid], red[tid + o]);
    __syncthreads();
  }
  if (tid == 0) {
    reinterpret_cast<float*>(fix)[0] = red[0] == -__builtin_huge_valf() ? 0.f : red[0] - kLseBoundSlack;
    fix[1] = 0;
  }
}

// The listed rows summed again exactly: one workgroup per row (grid-stride over the list), the
// exact maximum over all N columns, then one exp sweep against it; thread-strided partials
// and fixed trees (deterministic whatever the list's order), finalized as the merge does.
template <class Op>
__global__ __launch_bounds__(kBlock) void lse_fixup_kernel(Args args, Scal sc, int64_t N, const int* fix,
                                                           Outs outs) {
  constexpr int NACC = Op::NACC;
  __shared__ float red[NACC + 1][kBlock];
  const int tid = threadIdx.x;
  const int n = fix[1];
  for (int k = blockIdx.x; k < n; k += gridDim.x) {
    const int64_t i = fix[4 + k];
    typename Op::Row row;
    Op::load_row(args, sc, i, row);
    row.k = Op::base(row);
    float mx = -__builtin_huge_valf();
    for (int64_t j = tid; j < N; j += kBlock) {
      float rec[4 * Op::CW4];
      Op::load_col(args, sc, j, rec);
      mx = fmaxf(mx, Op::tm(sc, row, rec));
    }
    red[0][tid] = mx;
    __syncthreads();
    for (int o = kBlock / 2; o > 0; o >>= 1) {
      if (tid < o) red[0][tid] = fmaxf(red[0][tid], red[0][tid + o]);
      __syncthreads();
    }
    mx = red[0][0];
    if (mx == -__builtin_huge_valf()) mx = 0.f;
    __syncthreads();
    row.k -= mx;
    float acc[NACC + 1];
#pragma unroll
    for (int q = 0; q <= NACC; ++q) acc[q] = 0.f;
    for (int64_t j = tid; j < N; j += kBlock) {
      float rec[4 * Op::CW4];
      Op::load_col(args, sc, j, rec);
      const float tm = Op::tm(sc, row, rec);
      const float e = fast_exp2(tm);
      acc[0] += e;
      Op::template accum<false>(rec, tm, e, acc + 1);
    }
#pragma unroll
    for (int q = 0; q <= NACC; ++q) red[q][tid] = acc[q];
    __syncthreads();
    for (int o = kBlock / 2; o > 0; o >>= 1) {
      if (tid < o) {
#pragma unroll
        for (int q = 0; q <= NACC; ++q) red[q][tid] += red[q][tid + o];
      }
      __syncthreads();
    }
    if (tid == 0) {
      float a[NACC > 0 ? NACC : 1];
#pragma unroll
      for (int q = 0; q < NACC; ++q) a[q] = red[1 + q][0];
      Op::finalize(sc, args, i, mx, red[0][0], a, outs);
    }
    __syncthreads();
  }
}

// ---- E-step op ------------------------------------------------------------------------
// rows x_n ; columns (mu_c, v_c = w2_c / nc)   [w2_c = (w_c - LSE w) log2 e, nc = -log2 e/(2 s^2)]
// logit t2 = w2_c + nc |x_n - mu_c|^2 = nc (|x_n - mu_c|^2 + v_c)   (log2 domain, without -lgn):
// 3 sub + 3 fma from v_c, one fma with the row's -m -- 7 VALU (round 4: 8 + a compare).
// acc (STATS): sum e mu_c (D), sum e (t2 - m), sum e v_c -- the entropy, the log-weight and
// the squared-distance sums all follow from these at the finalize (round 4 summed e D2 and
// e |mu|^2 per pair as well): 14 VALU + 1 exp per pair.
template <int D, bool STATS>
struct OpGmmE {
  static constexpr int CW4 = cw4(D + 1);
  static constexpr int NACC = STATS ? D + 2 : 0;
  static constexpr int kShifted = STATS ? D : -1;
  struct Row { float x[D]; float k; };
  __device__ static void load_row(const Args& a, const Scal&, int64_t i, Row& r) { ld<D>(a.r0, i, r.x); }
  __device__ static float base(const Row&) { return 0.f; }
  // sc.aux1 = 1 / nc (< 0); a dead component (w2 = -inf) gets the logit kLseDead
  __device__ static void load_col(const Args& a, const Scal& sc, int64_t j, float* rec) {
    ld<D>(a.c0, j, rec);
    rec[D] = uni_value(a, sc, j);
  }
  __device__ static float tm(const Scal& sc, const Row& r, const float* rec) {
    float c = rec[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const float z = r.x[d] - rec[d];
      c = fmaf(z, z, c);
    }
    return fmaf(sc.nc, c, r.k);
  }
  // kUni: the acc slot of sum e v, which a tile of equal weights (v = v0 for every column:
  // the two-set match's frozen uniform GMM) forms as v0 sum e after the tile instead of one
  // fma per pair (uni_value(j) = column j's v, as load_col computes it).  Taken by the
  // many-component E-step (4 rows per thread, C >= kLseE4MinCols: 2.61 -> 2.47 ms at 100k x
  // 100k); a few hundred components gain nothing measurable from it, and keep their rounding
  // (the Chui two-set trace's EM stop test at tol 1e-3 flips one EM step on rounding-level
  // changes -- profiles/r05_chui_uniform_flip.txt)
  static constexpr int kUni = STATS ? D + 1 : -1;
  // the bound shift (lse_bound_kernel): the column's distance-0 logit nc v_c = w2_c
  static constexpr bool kBound = true;
  __device__ static float col_bound(const Args& a, const Scal& sc, int64_t j) { return sc.nc * uni_value(a, sc, j); }
  // per-row shift hint (dicp_gmm_estep_hint_f32): Args::r1, or NULL
  __device__ static const float* hint(const Args& a) { return a.r1; }
  static const float* hint_host(const Args& a) { return a.r1; }
  __device__ static float uni_value(const Args& a, const Scal& sc, int64_t j) {
    return fminf(a.c1[j] * sc.aux1, fminf(kLseDead * sc.aux1, 1e37f));
  }
  template <bool U = false>
  __device__ static void accum(const float* rec, float tm, float e, float* acc) {
    if (!STATS) return;
#pragma unroll
    for (int d = 0; d < D; ++d) acc[d] = fmaf(e, rec[d], acc[d]);
    acc[D] = fmaf(e, tm, acc[D]);
    if (!U) acc[D + 1] = fmaf(e, rec[D], acc[D + 1]);
  }
  // two rows packed in one VGPR pair (lse_rowred_pk_kernel): the same fmas as v_pk_fma_f32,
  // the column fields broadcast into both halves -- bitwise the scalar form
  struct Row2 { f2 x[D]; f2 k; };
  __device__ static void pack(const Row& a, const Row& b, Row2& r) {
#pragma unroll
    for (int d = 0; d < D; ++d) r.x[d] = f2{a.x[d], b.x[d]};
  }
  __device__ static f2 base2(const Row2&) { return splat(0.f); }
  __device__ static f2 tm2(const Scal& sc, const Row2& r, const float* rec) {
    f2 c = splat(rec[D]);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const f2 z = r.x[d] - splat(rec[d]);
      c = pk_fma(z, z, c);
    }
    return pk_fma(splat(sc.nc), c, r.k);
  }
  template <bool U = false>
  __device__ static void accum2(const float* rec, f2 tm, f2 e, f2* acc) {
    if (!STATS) return;
#pragma unroll
    for (int d = 0; d < D; ++d) acc[d] = pk_fma(e, splat(rec[d]), acc[d]);
    acc[D] = pk_fma(e, tm, acc[D]);
    if (!U) acc[D + 1] = pk_fma(e, splat(rec[D]), acc[D + 1]);
  }
  // outs: ptr[0] = T (natural, with -lgn), ptr[1] = T2 (log2, no lgn), ptr[2] = stats (D+4):
  //   sum gamma mu (D), sum gamma |mu|^2, sum gamma lgamma, sum gamma lpi, sum gamma D2
  // with (gamma-means, sum gamma = 1)  <t2 - m> = A, <v> = V:
  //   lgamma = ln2 (t2 - T2) -> ln2 (A - log2 l);  lpi = ln2 w2 = ln2 nc v -> ln2 nc V;
  //   D2 = (t2 - w2) / nc -> (A + m) / nc - V;  |mu|^2 = D2 + 2 x.mu - |x|^2 -> D2 + x.(2Y - x)
  // sc.aux0 = lgn
  __device__ static void finalize(const Scal& sc, const Args& a, int64_t i, float m, float l,
                                  const float* acc, const Outs& o) {
    const float lg = fast_log2(l);
    const float T2 = m + lg;
    o.ptr[0][i] = kLn2 * T2 - sc.aux0;
    if (o.ptr[1]) o.ptr[1][i] = T2;
    if (STATS && o.ptr[2]) {
      const float il = 1.f / l;
      float* st = o.ptr[2] + i * (D + 4);
      float x[D], mu2 = 0.f;
      ld<D>(a.r0, i, x);
      const float A = acc[D] * il, V = acc[D + 1] * il;
      const float D2 = fmaf(A + m, sc.aux1, -V);
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const float y = acc[d] * il;
        st[d] = y;
        mu2 = fmaf(x[d], fmaf(2.f, y, -x[d]), mu2);
      }
      st[D] = D2 + mu2;
      st[D + 1] = kLn2 * (A - lg);      // sum gamma lgamma
      st[D + 2] = kLn2 * sc.nc * V;     // sum gamma lpi
      st[D + 3] = D2;                   // sum gamma D2 (old mu)
    }
  }
};

// ---- M-step op (column pass as a row pass over components) ------------------------------
// rows c: (mu_c, w2_c) ; columns n: (x_n, u_n = -T2_n / nc)
// logit lg2 = w2_c + nc |x_n - mu_c|^2 - T2_n = nc (|x_n - mu_c|^2 + u_n) + w2_c = log2 gamma_nc
// (7 VALU, the row constant w2_c - m in the last fma) ; acc: sum e x_n (D)
template <int D>
struct OpGmmM {
  static constexpr int CW4 = cw4(D + 1);
  static constexpr int NACC = D;
  static constexpr int kShifted = -1;
  struct Row { float mu[D]; float w2; float k; };
  __device__ static void load_row(const Args& a, const Scal&, int64_t i, Row& r) {
    ld<D>(a.r0, i, r.mu);
    r.w2 = a.r1[i];
  }
  __device__ static float base(const Row& r) { return r.w2; }
  __device__ static void load_col(const Args& a, const Scal& sc, int64_t j, float* rec) {
    ld<D>(a.c0, j, rec);
    rec[D] = -a.c1[j] * sc.aux1;
  }
  __device__ static float tm(const Scal& sc, const Row& r, const float* rec) {
    float c = rec[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const float z = r.mu[d] - rec[d];
      c = fmaf(z, z, c);
    }
    return fmaf(sc.nc, c, r.k);
  }
  static constexpr int kUni = -1;
  __device__ static float uni_value(const Args&, const Scal&, int64_t) { return 0.f; }
  __device__ static const float* hint(const Args&) { return nullptr; }
  template <bool U = false>
  __device__ static void accum(const float* rec, float, float e, float* acc) {
#pragma unroll
    for (int d = 0; d < D; ++d) acc[d] = fmaf(e, rec[d], acc[d]);
  }
  struct Row2 { f2 mu[D]; f2 w2; f2 k; };
  __device__ static void pack(const Row& a, const Row& b, Row2& r) {
#pragma unroll
    for (int d = 0; d < D; ++d) r.mu[d] = f2{a.mu[d], b.mu[d]};
    r.w2 = f2{a.w2, b.w2};
  }
  __device__ static f2 base2(const Row2& r) { return r.w2; }
  __device__ static f2 tm2(const Scal& sc, const Row2& r, const float* rec) {
    f2 c = splat(rec[D]);
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const f2 z = r.mu[d] - splat(rec[d]);
      c = pk_fma(z, z, c);
    }
    return pk_fma(splat(sc.nc), c, r.k);
  }
  template <bool U = false>
  __device__ static void accum2(const float* rec, f2, f2 e, f2* acc) {
#pragma unroll
    for (int d = 0; d < D; ++d) acc[d] = pk_fma(e, splat(rec[d]), acc[d]);
  }
  // outs.ptr[0] = colstats (D+1): {log sum gamma, mean x (D)}
  __device__ static void finalize(const Scal&, const Args&, int64_t i, float m, float l,
                                  const float* acc, const Outs& o) {
    float* st = o.ptr[0] + i * (D + 1);
    st[0] = kLn2 * (m + fast_log2(l));
    const float il = 1.f / l;
#pragma unroll
    for (int d = 0; d < D; ++d) st[1 + d] = acc[d] * il;
  }
};

// ---- targets op (plain row sum; gamma <= 1 needs no max) --------------------------------
// rows n: (x_n, T2_n) ; columns c: (mu_old, w2_old, mu_new, |mu_new|^2, lpi_new)
// gamma = 2^(w2_old + nc_old |x - mu_old|^2 - T2_n)
// out (D+4): sum g mu_new (D), sum g |mu_new|^2, sum g lpi_new, sum g, sum g |x - mu_new|^2
template <int D>
struct OpGmmTargets {
  static constexpr int CW4 = cw4(2 * D + 3);
  static constexpr int NACC = D + 4;
  static constexpr int kNOut = 1;
  static constexpr int kOutW[4] = {D + 4, 0, 0, 0};
  static constexpr bool kMin = false;
  struct Row { float x[D]; float T2; };
  __device__ static void load_row(const Args& a, int64_t i, Row& r) {
    ld<D>(a.r0, i, r.x);
    r.T2 = a.r1[i];
  }
  __device__ static void load_col(const Args& a, int64_t j, float* rec) {
    ld<D>(a.c0, j, rec);
    rec[D] = a.c1[j];
    ld<D>(a.c2, j, rec + D + 1);
    float n2 = 0.f;
#pragma unroll
    for (int d = 0; d < D; ++d) n2 = fmaf(rec[D + 1 + d], rec[D + 1 + d], n2);
    rec[2 * D + 1] = n2;
    rec[2 * D + 2] = a.c3[j];
  }
  __device__ static void pair(const Scal& sc, const Row& r, const float* rec, float* acc) {
    float z[D];
    const float d2o = diff_sq<D>(r.x, rec, z);
    const float g = fast_exp2(fmaf(sc.nc, d2o, rec[D] - r.T2));
    const float* mn = rec + D + 1;
    const float d2n = diff_sq<D>(r.x, mn, z);
#pragma unroll
    for (int d = 0; d < D; ++d) acc[d] = fmaf(g, mn[d], acc[d]);
    acc[D] = fmaf(g, rec[2 * D + 1], acc[D]);
    acc[D + 1] = fmaf(g, rec[2 * D + 2], acc[D + 1]);
    acc[D + 2] += g;
    acc[D + 3] = fmaf(g, d2n, acc[D + 3]);
  }
  __device__ static void store(const Scal&, const Row&, const float* t, float* v) {
#pragma unroll
    for (int k = 0; k < D + 4; ++k) v[k] = t[k];
  }
};

template <class Op, int R>
int lse_splits(int64_t M, int64_t N, bool pk) {
  static int64_t cap[2] = {-1, -1};
  if (cap[pk] < 0)
    cap[pk] = (int64_t)device_cus() * (pk ? blocks_per_cu(lse_rowred_pk_kernel<Op, R / 2>)
                                          : blocks_per_cu(lse_rowred_kernel<Op, R>));
  return num_splits_cap(M, N, R, cap[pk]);
}

template <class T, class = void>
struct op_bound : std::false_type {};
template <class T>
struct op_bound<T, std::enable_if_t<T::kBound>> : std::true_type {};
// the bound shift: ops with Op::kBound at R = 4 rows per thread (the many-component E-step),
// option "lse_bound" (env DICP_LSE_BOUND; 0: the sampled shift as every other pass)
template <class Op, int R>
constexpr bool lse_bound_op() { return op_bound<Op>::value && R == 4; }

template <class Op, int R>
size_t lse_ws_bytes(int64_t M, int64_t N) {   // either kernel (their occupancies may differ)
  const int S0 = lse_splits<Op, R>(M, N, false), S1 = lse_splits<Op, R>(M, N, true);
  const int S = S0 > S1 ? S0 : S1;
  const size_t fix = lse_bound_op<Op, R>() ? (size_t)(4 + M) * sizeof(int) : 0;
  return (size_t)S * (size_t)M * (size_t)(2 + Op::NACC) * sizeof(float) + fix;
}

template <class Op, int R>
int launch_lse(const char* name, const Args& a, const Scal& sc, int64_t M, int64_t N,
               const Outs& fin, void* ws, size_t ws_bytes, hipStream_t st) {
  if (M <= 0) return DICP_OK;
  const bool pk = lse_pk_ref() != 0 && R % 2 == 0;
  const int S = lse_splits<Op, R>(M, N, pk);
  const int64_t chunk = N > 0 ? chunk_of(N, S) : 0;
  const size_t need = lse_ws_bytes<Op, R>(M, N);
  if (ws == nullptr || ws_bytes < need) {
    set_error("%s: workspace too small (%zu < %zu bytes)", name, ws_bytes, need);
    return DICP_ERR_WORKSPACE;
  }
  const int64_t bx = (M + (int64_t)kBlock * R - 1) / ((int64_t)kBlock * R);
  float* part = reinterpret_cast<float*>(ws);
  int* fix = nullptr;
  Args ab = a;
  if constexpr (lse_bound_op<Op, R>()) {
    // hinted calls only: unhinted, the bound sits up to ~nc d^2 above a row's largest logit and
    // the shifted logits t - m then carry that much absolute rounding into the sums e (t - m)
    // (the sigma update's sum gamma D^2 measured 3e-6 off the sampled shift's on the exact
    // two-set workload); with a hint the shift is within ~8 + log2 C of the row's maximum
    if (lse_bound_ref() != 0 && N > 0 && Op::hint_host(a) != nullptr) {   // {U, count, -, -, rows}
      fix = reinterpret_cast<int*>(part + (size_t)S * (size_t)M * (size_t)(2 + Op::NACC));
      lse_bound_kernel<Op><<<dim3(1), dim3(kBoundThreads), 0, st>>>(a, sc, N, fix);
      ab.r2 = reinterpret_cast<const float*>(fix);
    }
  }
  if (fix != nullptr) {
    if constexpr (lse_bound_op<Op, R>()) {
      if (pk)
        lse_rowred_pk_kernel<Op, R / 2, true><<<dim3((unsigned)bx, (unsigned)S), dim3(kBlock), 0, st>>>(
            ab, sc, M, N, chunk, part, lse_adapt_ref());
      else
        lse_rowred_kernel<Op, R, true><<<dim3((unsigned)bx, (unsigned)S), dim3(kBlock), 0, st>>>(
            ab, sc, M, N, chunk, part, lse_adapt_ref());
    }
  } else if (pk) {
    lse_rowred_pk_kernel<Op, R / 2><<<dim3((unsigned)bx, (unsigned)S), dim3(kBlock), 0, st>>>(
        a, sc, M, N, chunk, part, lse_adapt_ref());
  } else {
    lse_rowred_kernel<Op, R><<<dim3((unsigned)bx, (unsigned)S), dim3(kBlock), 0, st>>>(
        a, sc, M, N, chunk, part, lse_adapt_ref());
  }
  int rc = check_launch(name);
  if (rc) return rc;
  if (S > kWaveMergeMinSplits) {
    const int64_t nw = (M + kBlock / 64 - 1) / (kBlock / 64);
    lse_finalize_wave_kernel<Op><<<dim3((unsigned)nw), dim3(kBlock), 0, st>>>(part, M, S, a, sc, fin, fix);
  } else {
    const int64_t nb = (M + kBlock - 1) / kBlock;
    lse_finalize_kernel<Op><<<dim3((unsigned)nb), dim3(kBlock), 0, st>>>(part, M, S, a, sc, fin, fix);
  }
  rc = check_launch(name);
  if (rc) return rc;
  if constexpr (lse_bound_op<Op, R>()) {
    if (fix != nullptr) {   // the listed rows again, exactly (a grid-stride over the list)
      const int64_t nf = M < 1024 ? M : 1024;
      lse_fixup_kernel<Op><<<dim3((unsigned)nf), dim3(kBlock), 0, st>>>(a, sc, N, fix, fin);
      rc = check_launch(name);
    }
  }
  return rc;
}

template <int D>
int estep_d(const float* X, int64_t N, const float* mu, const float* w2, const float* mu2,
            int64_t C, double sigma, double lgn, const float* hint, float* T, float* T2,
            float* stats, void* ws, size_t wsb, hipStream_t st) {
  const Args a = {X, hint, nullptr, nullptr, mu, w2, mu2, nullptr};
  Scal sc = make_scal(sigma, 0.0);
  sc.aux0 = (float)lgn;
  sc.aux1 = 1.0f / sc.nc;
  const Outs o = make_outs(T, T2, stats);
  if (C >= kLseE4MinCols) {   // many components: 4 rows (two packed pairs) per thread
    if (stats) return launch_lse<OpGmmE<D, true>, 4>("gmm_estep", a, sc, N, C, o, ws, wsb, st);
    return launch_lse<OpGmmE<D, false>, 4>("gmm_estep", a, sc, N, C, o, ws, wsb, st);
  }
  if (stats) return launch_lse<OpGmmE<D, true>, kLseRG>("gmm_estep", a, sc, N, C, o, ws, wsb, st);
  return launch_lse<OpGmmE<D, false>, kLseRG>("gmm_estep", a, sc, N, C, o, ws, wsb, st);
}

}  // namespace

namespace dicp {
int& lse_pk() { return lse_pk_ref(); }
int& lse_adapt() { return lse_adapt_ref(); }
int& lse_bound() { return lse_bound_ref(); }
}  // namespace dicp

// The Python wrapper precomputes the C-sized column vectors (w2, |mu|^2, lpi) with torch on
// the device; the kernels here see only device pointers.
extern "C" int dicp_gmm_estep_hint_f32(const float* X, int64_t N, const float* mu, const float* w2,
                                       const float* mu2, int64_t C, int D, double sigma, double lgn,
                                       const float* hint, float* T, float* T2, float* stats, void* ws,
                                       size_t ws_bytes, dicp_stream_t stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (N < 0 || C <= 0 || (N > 0 && (!X || !T)) || !mu || !w2 || !mu2 || !(sigma > 0)) {
    set_error("dicp_gmm_estep_f32: invalid arguments");
    return DICP_ERR_INVALID;
  }
  switch (D) {
    case 2: return estep_d<2>(X, N, mu, w2, mu2, C, sigma, lgn, hint, T, T2, stats, ws, ws_bytes, st);
    case 3: return estep_d<3>(X, N, mu, w2, mu2, C, sigma, lgn, hint, T, T2, stats, ws, ws_bytes, st);
    default: set_error("gmm_estep: D=%d unsupported", D); return DICP_ERR_UNSUPPORTED;
  }
}

extern "C" int dicp_gmm_estep_f32(const float* X, int64_t N, const float* mu, const float* w2,
                                  const float* mu2, int64_t C, int D, double sigma, double lgn,
                                  float* T, float* T2, float* stats, void* ws, size_t ws_bytes,
                                  dicp_stream_t stream) {
  return dicp_gmm_estep_hint_f32(X, N, mu, w2, mu2, C, D, sigma, lgn, nullptr, T, T2, stats, ws,
                                 ws_bytes, stream);
}

extern "C" int dicp_gmm_mstep_f32(const float* X, const float* T2, int64_t N, const float* mu,
                                  const float* w2, int64_t C, int D, double sigma,
                                  float* colstats, void* ws, size_t ws_bytes,
                                  dicp_stream_t stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (N <= 0 || C <= 0 || !X || !T2 || !mu || !w2 || !colstats || !(sigma > 0)) {
    set_error("dicp_gmm_mstep_f32: invalid arguments");
    return DICP_ERR_INVALID;
  }
  const Args a = {mu, w2, nullptr, nullptr, X, T2, nullptr, nullptr};
  Scal sc = make_scal(sigma, 0.0);
  sc.aux1 = 1.0f / sc.nc;
  const Outs o = make_outs(colstats);
  switch (D) {
    case 2: return launch_lse<OpGmmM<2>, kLseRG>("gmm_mstep", a, sc, C, N, o, ws, ws_bytes, st);
    case 3: return launch_lse<OpGmmM<3>, kLseRG>("gmm_mstep", a, sc, C, N, o, ws, ws_bytes, st);
    default: set_error("gmm_mstep: D=%d unsupported", D); return DICP_ERR_UNSUPPORTED;
  }
}

extern "C" int dicp_gmm_targets_f32(const float* X, const float* T2, int64_t N,
                                    const float* mu_old, const float* w2_old, double sigma_old,
                                    const float* mu_new, const float* lpi_new, int64_t C, int D,
                                    float* rows, void* ws, size_t ws_bytes,
                                    dicp_stream_t stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (N < 0 || C <= 0 || (N > 0 && (!X || !T2 || !rows)) || !mu_old || !w2_old || !mu_new ||
      !lpi_new || !(sigma_old > 0)) {
    set_error("dicp_gmm_targets_f32: invalid arguments");
    return DICP_ERR_INVALID;
  }
  const Args a = {X, T2, nullptr, nullptr, mu_old, w2_old, mu_new, lpi_new};
  const Scal sc = make_scal(sigma_old, 0.0);
  const Outs o = make_outs(rows);
  switch (D) {
    case 2: return launch_rowred<OpGmmTargets<2>, kRG>("gmm_targets", a, sc, N, C, o, ws, ws_bytes, st);
    case 3: return launch_rowred<OpGmmTargets<3>, kRG>("gmm_targets", a, sc, N, C, o, ws, ws_bytes, st);
    default: set_error("gmm_targets: D=%d unsupported", D); return DICP_ERR_UNSUPPORTED;
  }
}

size_t dicp_gmm_ws(int kind, int64_t M, int64_t N, int D) {
  // M = rows of the data (N points), N = components (C) for the GMM kinds
  if (D != 2 && D != 3) return 0;
  switch (kind) {
    case DICP_WS_GMM_ESTEP: {  // every variant (their occupancies, hence splits, differ)
      size_t m = 0;
      for (size_t v : {D == 2 ? lse_ws_bytes<OpGmmE<2, true>, kLseRG>(M, N) : lse_ws_bytes<OpGmmE<3, true>, kLseRG>(M, N),
                       D == 2 ? lse_ws_bytes<OpGmmE<2, false>, kLseRG>(M, N) : lse_ws_bytes<OpGmmE<3, false>, kLseRG>(M, N),
                       D == 2 ? lse_ws_bytes<OpGmmE<2, true>, 4>(M, N) : lse_ws_bytes<OpGmmE<3, true>, 4>(M, N),
                       D == 2 ? lse_ws_bytes<OpGmmE<2, false>, 4>(M, N) : lse_ws_bytes<OpGmmE<3, false>, 4>(M, N)})
        m = v > m ? v : m;
      return m;
    }
    case DICP_WS_GMM_MSTEP:
      return D == 2 ? lse_ws_bytes<OpGmmM<2>, kLseRG>(N, M) : lse_ws_bytes<OpGmmM<3>, kLseRG>(N, M);
    case DICP_WS_GMM_TARGETS:
      return D == 2 ? rowred_ws_bytes<OpGmmTargets<2>, kRG>(M, N)
                    : rowred_ws_bytes<OpGmmTargets<3>, kRG>(M, N);
    default: return 0;
  }
}
