// Pair-once (symmetric) centred Gaussian-kernel sums for x = y: KBase, KRedScal, KRed
// (kernel.py:131/:135/:138, torch :178-187) when the rows and columns are the SAME point set
// -- the north_star's "100k x 100k 3D Gaussian kernel sum" as LDDMMModel.v(q, q, p) and the
// Hamiltonian evaluate it (LDDMM.py:114, :151).
//
// K_ij = K_ji, so every unordered pair is evaluated once and its two contributions go to row
// i (K f_j) and to row j (K f_i): one exp per unordered pair instead of two.  The points are
// Morton-sorted (the prep of centred.hip: bounding box, 30-bit codes, stable radix sort) and
// grouped in groups of 256 consecutive sorted points; group g has a centre c_g (mid-range) and
// a radius.  For a pair of groups (A rows, B columns) both sides are expressed relative to
// c_B in scaled units (X = alpha (x - c_B), Y = alpha (y - c_B), alpha = sqrt(log2 e / 2 sigma^2)):
//     K = exp2(-|X - Y|^2) = F_i * exp2(2 X.Y - |Y|^2 - m),   F_i = exp2(m - |X|^2)
// as centred.hpp's expansion (m = 16, the same range argument and |X| clamp), so a pair costs
// 3 FMA for its exponent; the row factor F_i multiplies the row's partial sum over group B
// once (row side) and is folded into the row's fields, F_i f_i, once per group pair (column
// side).  Per step a lane pairs its 4 rows (two float2 row pairs) with one column:
//     6 v_pk (exponents) + 4 v_exp + 6 v_pk (row sums) + 6 v_pk + 3 add + 3 DPP (column sums)
// for 8 ordered pairs, against 12 v_pk + 8 v_exp for the ordered centred kernel (cx_kernel, 4
// rows); the column sums ride the wave_rol:1 rotation of the symmetric forward / VJP
// (lddmm_sym.hpp), so no reduction tree is needed.  Groups whose radius exceeds rho_max
// (cx_rho_x100) are paired in the difference form on the raw coordinates (as cx_kernel's wide
// sub-tiles).
//
// Work decomposition, slots and merge as the symmetric 4-row kernels (lddmm_sym_pk.hpp
// sym_pk4_body): a workgroup = 4 waves = row groups A = 4Q + w of quad Q against the column
// groups B of chunk kc; A < B both sides, A == B the ordered pairs (row side, self pair
// included), A > B nothing (done by wave B).  Column sums of the 4 waves are added in LDS in
// wave order into slot Q of group B, row sums go to slot Q + 1 + kc; the merge adds a row's
// slots in slot order and scatters it back to the caller's order.  Deterministic, no atomics.
#pragma once
#include "centred.hpp"
#include "lddmm_sym.hpp"
#include "packed.hpp"

namespace dicp {

constexpr int kScG = 256;   // points per group: one wave of 64 lanes x 4 rows
// record (3 float4): [2Y0, 2Y1, c, c] [fields (W <= 3) | 2Y2 (D = 3) at .w] [raw y | 0]
// (2Y2 after the fields: with it in front the hipcc schedule copied the last field out of its
// register pair with a v_mov per step)
template <int D> constexpr int scx_f = 4;                  // first field
constexpr int kScY2 = 7;                                   // 2Y2 (D = 3)
constexpr int kScRaw = 8;                                  // raw coordinates
// fields per op: 0 KBase (1: the constant 1), 1 KRedScal (1: d_j), 2 KRed (D: b_j)
template <int D, int OPK> constexpr int scx_w = OPK == 2 ? D : 1;

// one workgroup per group of G sorted points (G / 256 per thread): centre, compactness and
// the records
template <int D, int OPK, int G = kScG>
__global__ __launch_bounds__(256) void scx_group_kernel(const float* __restrict__ x, const float* __restrict__ f,
                                                        int64_t N, float alpha, float rho2max,
                                                        const int32_t* __restrict__ order,
                                                        float4* __restrict__ recs, float4* __restrict__ gmeta) {
  constexpr int W = scx_w<D, OPK>;
  constexpr int U = G / 256;
  __shared__ float red[2 * D + 1][4];
  __shared__ float cen[D + 1];
  const int tid = threadIdx.x, wv = tid >> 6, l = tid & 63;
  float y[U][D], lo[D], hi[D];
  int64_t o[U];
  bool valid[U];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    lo[d] = __builtin_huge_valf();
    hi[d] = -__builtin_huge_valf();
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t s = (int64_t)blockIdx.x * G + u * 256 + tid;
    valid[u] = s < N;
    o[u] = valid[u] ? order[s] : 0;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      y[u][d] = x[o[u] * D + d];
      if (valid[u]) {
        lo[d] = fminf(lo[d], y[u][d]);
        hi[d] = fmaxf(hi[d], y[u][d]);
      }
    }
  }
#pragma unroll
  for (int d = 0; d < D; ++d)
    for (int off = 32; off > 0; off >>= 1) {
      lo[d] = fminf(lo[d], __shfl_xor(lo[d], off, 64));
      hi[d] = fmaxf(hi[d], __shfl_xor(hi[d], off, 64));
    }
  if (l == 0) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      red[d][wv] = lo[d];
      red[D + d][wv] = hi[d];
    }
  }
  __syncthreads();
  if (tid == 0) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      float a = red[d][0], b = red[D + d][0];
      for (int w = 1; w < 4; ++w) {
        a = fminf(a, red[d][w]);
        b = fmaxf(b, red[D + d][w]);
      }
      cen[d] = 0.5f * (a + b);   // raw centre of the group (mid-range)
    }
  }
  __syncthreads();
  float Yc[U][D], r2[U], rmax = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    r2[u] = 0.f;
#pragma unroll
    for (int d = 0; d < D; ++d) {
      Yc[u][d] = alpha * (y[u][d] - cen[d]);
      r2[u] = fmaf(Yc[u][d], Yc[u][d], r2[u]);
    }
    if (valid[u]) rmax = fmaxf(rmax, r2[u]);
  }
  for (int off = 32; off > 0; off >>= 1) rmax = fmaxf(rmax, __shfl_xor(rmax, off, 64));
  if (l == 0) red[0][wv] = rmax;
  __syncthreads();
  if (tid == 0) {
    float m = red[0][0];
    for (int w = 1; w < 4; ++w) m = fmaxf(m, red[0][w]);
    float mt[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int d = 0; d < D; ++d) mt[d] = cen[d];
    mt[3] = m <= rho2max ? 1.f : 0.f;
    gmeta[blockIdx.x] = make_float4(mt[0], mt[1], mt[2], mt[3]);
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (!valid[u]) continue;
    const int64_t s = (int64_t)blockIdx.x * G + u * 256 + tid;
    float rec[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) rec[k] = 0.f;
    rec[0] = 2.f * Yc[u][0];
    rec[1] = 2.f * Yc[u][1];
    if (D == 3) rec[kScY2] = 2.f * Yc[u][2];
    rec[2] = rec[3] = -r2[u] - kCxShift;
#pragma unroll
    for (int k = 0; k < W; ++k) rec[scx_f<D> + k] = OPK == 0 ? 1.f : f[o[u] * W + k];
#pragma unroll
    for (int d = 0; d < D; ++d) rec[kScRaw + d] = y[u][d];
#pragma unroll
    for (int k = 0; k < 3; ++k) recs[s * 3 + k] = make_float4(rec[4 * k], rec[4 * k + 1], rec[4 * k + 2], rec[4 * k + 3]);
  }
}

// the pair-once kernel.  grid (Kmax, nQ): blockIdx.y = quad Q, blockIdx.x = column chunk kc.
// RP row pairs per lane: 2 (4 rows, groups of 256) or 4 (8 rows, groups of 512 -- the column
// side's adds, DPP rotations and LDS addressing then serve 8 rows).
// LDS ring (DICP_SCX_RING, default): each 64-column quarter of a group is staged twice in a
// row (128 records), so the record of column (l + k2) mod 64 sits at l + k2 without the wrap:
// the step's LDS addresses are one lane base plus an immediate offset instead of 3 VALU (an
// add, an and-or, a shift-add) per step -- 6 of the loop's 70 VALU per 2 steps.
#ifndef DICP_SCX_RING
#define DICP_SCX_RING 1
#endif
template <int D, int OPK, int RP = 2>
__global__ __launch_bounds__(256) void scx_kernel(const float4* __restrict__ recs, const float4* __restrict__ gmeta,
                                                  int64_t M, int nG, int L, float alpha,
                                                  float* __restrict__ slab, int64_t slot_stride) {
  constexpr int W = scx_w<D, OPK>;
  constexpr int F0 = scx_f<D>;
  constexpr int NR = 2 * RP;         // rows per lane
  constexpr int G = 64 * NR;         // points per group
  constexpr bool kRing = DICP_SCX_RING != 0;
  constexpr int GS = kRing ? 2 * G : G;   // staged records per buffer
  __shared__ float4 planes[2][3][GS];
  __shared__ float colacc[kSymQ][64][W];   // one 64-column quarter at a time
  const int Q = (int)blockIdx.y, kc = (int)blockIdx.x;
  const int B0 = kSymQ * Q + kc * L;
  if (B0 >= nG) return;   // uniform for the whole workgroup, before any barrier
  const int B1 = min(B0 + L, nG);
  const int tid = threadIdx.x, wv = tid >> 6, l = tid & 63;
  const int A = kSymQ * Q + wv;

  // the lane's rows (r * 64 + l of group A) as float2 pairs: raw coordinates, fields.  Rows
  // past the end (or of a group past nG) take a real point's coordinates with zero fields:
  // they add nothing to any column and their own sums are not written.
  f2 xr[RP][D], fr[RP][W];
  int64_t ri[NR];
  bool rv[NR];
  {
    float xs[NR][D], fs[NR][W];
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      ri[r] = (int64_t)A * G + r * 64 + l;
      rv[r] = A < nG && ri[r] < M;
      const int64_t src = rv[r] ? ri[r] : M - 1;
      const float* rc = reinterpret_cast<const float*>(recs + src * 3);
#pragma unroll
      for (int d = 0; d < D; ++d) xs[r][d] = rc[kScRaw + d];
#pragma unroll
      for (int k = 0; k < W; ++k) fs[r][k] = rv[r] ? rc[F0 + k] : 0.f;
    }
#pragma unroll
    for (int h = 0; h < RP; ++h) {
#pragma unroll
      for (int d = 0; d < D; ++d) xr[h][d] = f2{xs[2 * h][d], xs[2 * h + 1][d]};
#pragma unroll
      for (int k = 0; k < W; ++k) fr[h][k] = f2{fs[2 * h][k], fs[2 * h + 1][k]};
    }
  }
  f2 racc[RP][W];
#pragma unroll
  for (int h = 0; h < RP; ++h)
#pragma unroll
    for (int k = 0; k < W; ++k) racc[h][k] = splat(0.f);

  // record slot of column c (0..G-1) of the staged group, first copy; the ring's second copy
  // of a quarter sits 64 slots after the first
  auto slot = [](int c) { return kRing ? (c >> 6) * 128 + (c & 63) : c; };
  auto stage = [&](int B, int buf) {
#pragma unroll
    for (int u = 0; u < G / 256; ++u) {
      const int c = u * 256 + tid;
      const int64_t j = (int64_t)B * G + c;
      float4 v[3];
      if (j < M) {
#pragma unroll
        for (int k = 0; k < 3; ++k) v[k] = recs[j * 3 + k];
      } else {   // padding column: K = 0 against every row, zero fields
        v[0] = make_float4(0.f, 0.f, -1.0e30f, -1.0e30f);
        v[1] = make_float4(0.f, 0.f, 0.f, 0.f);
        v[2] = make_float4(kFar, kFar, kFar, 0.f);
      }
      const int sl = slot(c);
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        planes[buf][k][sl] = v[k];
        if (kRing) planes[buf][k][sl + 64] = v[k];
      }
    }
  };
  int buf = 0;
  stage(B0, 0);
  __syncthreads();
  for (int B = B0; B < B1; ++B) {
    if (B + 1 < B1) stage(B + 1, buf ^ 1);
    const bool sym = A < B;    // wave-uniform
    const bool diag = A == B;
    const float4 mB = gmeta[B];
    const bool compact = mB.w != 0.f;
    const float cB[3] = {mB.x, mB.y, mB.z};
    // row side relative to c_B: X, the row factor F = exp2(m - |X|^2) (clamped as cx_kernel)
    f2 X[RP][D], F[RP], bF[RP][W], rp[RP][W];
#pragma unroll
    for (int h = 0; h < RP; ++h) {
      f2 a2 = splat(0.f);
#pragma unroll
      for (int d = 0; d < D; ++d) {
        X[h][d] = (xr[h][d] - splat(cB[d])) * splat(alpha);
        a2 = pk_fma(X[h][d], X[h][d], a2);
      }
      F[h] = f2{fast_exp2(kCxShift - a2.x), fast_exp2(kCxShift - a2.y)};
      const f2 cl = f2{a2.x > kCxClamp * kCxClamp ? kCxClamp * __builtin_amdgcn_rsqf(a2.x) : 1.f,
                       a2.y > kCxClamp * kCxClamp ? kCxClamp * __builtin_amdgcn_rsqf(a2.y) : 1.f};
#pragma unroll
      for (int d = 0; d < D; ++d) X[h][d] = X[h][d] * cl;
#pragma unroll
      for (int k = 0; k < W; ++k) {
        bF[h][k] = compact ? F[h] * fr[h][k] : fr[h][k];
        rp[h][k] = splat(0.f);
      }
    }
#pragma unroll 1
    for (int qq = 0; qq < G / 64; ++qq) {
      float cacc[W];
#pragma unroll
      for (int k = 0; k < W; ++k) cacc[k] = 0.f;
      // the lane's step-k2 column: slot lb + k2 (ring) / the wrapped slot (no ring)
      const int lb = kRing ? qq * 128 + l : 0;
      auto csl = [&](int k2) { return kRing ? lb + k2 : qq * 64 + ((l + k2) & 63); };
      if (sym && compact) {
#pragma unroll 2
        for (int k2 = 0; k2 < 64; ++k2) {
          const int col = csl(k2);
          const float4 p0 = planes[buf][0][col], p1 = planes[buf][1][col];
          const float rec[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
          const float y2[3] = {rec[0], rec[1], rec[kScY2]};
          f2 K[RP];
#pragma unroll
          for (int h = 0; h < RP; ++h) {
            f2 e = f2{rec[2], rec[3]};
#pragma unroll
            for (int d = 0; d < D; ++d) e = pk_fma(X[h][d], splat(y2[d]), e);
            K[h] = f2{fast_exp2(e.x), fast_exp2(e.y)};
#pragma unroll
            for (int k = 0; k < W; ++k) rp[h][k] = pk_fma(K[h], splat(rec[F0 + k]), rp[h][k]);
          }
#pragma unroll
          for (int k = 0; k < W; ++k) {
            f2 c = K[0] * bF[0][k];
#pragma unroll
            for (int h = 1; h < RP; ++h) c = pk_fma(K[h], bF[h][k], c);
            cacc[k] = rol1(cacc[k]) + (c.x + c.y);
          }
        }
#pragma unroll
        for (int k = 0; k < W; ++k) cacc[k] = rol1(cacc[k]);
      } else if (sym) {   // wide column group: difference form on the raw coordinates
#pragma unroll 2
        for (int k2 = 0; k2 < 64; ++k2) {
          const int col = csl(k2);
          const float4 p1 = planes[buf][1][col], p2 = planes[buf][2][col];
          const float rec[8] = {p1.x, p1.y, p1.z, p1.w, p2.x, p2.y, p2.z, p2.w};
          f2 K[RP];
#pragma unroll
          for (int h = 0; h < RP; ++h) {
            f2 e = splat(0.f);
#pragma unroll
            for (int d = 0; d < D; ++d) {
              const f2 z = (xr[h][d] - splat(rec[4 + d])) * splat(alpha);
              e = pk_fma(z, z, e);
            }
            K[h] = f2{fast_exp2(-e.x), fast_exp2(-e.y)};
#pragma unroll
            for (int k = 0; k < W; ++k) rp[h][k] = pk_fma(K[h], splat(rec[F0 - 4 + k]), rp[h][k]);
          }
#pragma unroll
          for (int k = 0; k < W; ++k) {
            f2 c = K[0] * bF[0][k];
#pragma unroll
            for (int h = 1; h < RP; ++h) c = pk_fma(K[h], bF[h][k], c);
            cacc[k] = rol1(cacc[k]) + (c.x + c.y);
          }
        }
#pragma unroll
        for (int k = 0; k < W; ++k) cacc[k] = rol1(cacc[k]);
      } else if (diag) {  // ordered pairs of the group with itself, row side only
#pragma unroll 2
        for (int k2 = 0; k2 < 64; ++k2) {
          const int col = (kRing ? qq * 128 : qq * 64) + k2;
          const float4 p0 = planes[buf][0][col], p1 = planes[buf][1][col], p2 = planes[buf][2][col];
          const float rec[12] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w, p2.x, p2.y, p2.z, p2.w};
          const float y2[3] = {rec[0], rec[1], rec[kScY2]};
#pragma unroll
          for (int h = 0; h < RP; ++h) {
            f2 K;
            if (compact) {
              f2 e = f2{rec[2], rec[3]};
#pragma unroll
              for (int d = 0; d < D; ++d) e = pk_fma(X[h][d], splat(y2[d]), e);
              K = f2{fast_exp2(e.x), fast_exp2(e.y)};
            } else {
              f2 e = splat(0.f);
#pragma unroll
              for (int d = 0; d < D; ++d) {
                const f2 z = (xr[h][d] - splat(rec[kScRaw + d])) * splat(alpha);
                e = pk_fma(z, z, e);
              }
              K = f2{fast_exp2(-e.x), fast_exp2(-e.y)};
            }
#pragma unroll
            for (int k = 0; k < W; ++k) rp[h][k] = pk_fma(K, splat(rec[F0 + k]), rp[h][k]);
          }
        }
      }
#pragma unroll
      for (int k = 0; k < W; ++k) colacc[wv][l][k] = cacc[k];
      __syncthreads();
      {
        // the quarter's 64 column sums of the 4 waves, added in wave order (contiguous stores)
        const int64_t j0 = (int64_t)B * G + qq * 64;
        float* dst = slab + (int64_t)Q * slot_stride + j0 * W;
        for (int e = tid; e < 64 * W; e += 256) {
          const int c = e / W, k = e - c * W;
          if (j0 + c < M) dst[e] = ((colacc[0][c][k] + colacc[1][c][k]) + colacc[2][c][k]) + colacc[3][c][k];
        }
      }
      __syncthreads();
    }
    // fold the row partials of group B into the row totals (compact: times F)
#pragma unroll
    for (int h = 0; h < RP; ++h)
#pragma unroll
      for (int k = 0; k < W; ++k) racc[h][k] = compact ? pk_fma(F[h], rp[h][k], racc[h][k]) : racc[h][k] + rp[h][k];
    buf ^= 1;
  }
#pragma unroll
  for (int r = 0; r < NR; ++r) {
    if (!rv[r]) continue;
    float* dst = slab + (int64_t)(Q + 1 + kc) * slot_stride + ri[r] * W;
    const f2* ra = racc[r >> 1];
#pragma unroll
    for (int k = 0; k < W; ++k) dst[k] = (r & 1) == 0 ? ra[k].x : ra[k].y;
  }
}

// merge: one thread per sorted point sums its slots in slot order and writes the result to
// the point's original row (order[s]) through the Outs epilogue of output 0
template <int W, int G = kScG>
__global__ __launch_bounds__(256) void scx_merge_kernel(const float* __restrict__ slab, int64_t slot_stride,
                                                        int64_t M, int nG, int L, const int32_t* __restrict__ order,
                                                        Outs o) {
  const int64_t s = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (s >= M) return;
  const int ns = sym_nslots((int)(s / G), nG, L);
  float t[W];
  const float* src = slab + s * W;
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
  const int64_t i = order[s];
#pragma unroll
  for (int k = 0; k < W; ++k) o.ptr[0][i * W + k] = epilogue(o, 0, i * W + k, t[k]);
}

}  // namespace dicp
