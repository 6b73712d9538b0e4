// Fused LDDMM ODE forward (eta = 0: classic / hybrid models) with the column contraction on
// the matrix cores: the VALU computes the Gaussian kernel K_ij = exp2(-|q'_i - q'_j|^2) of
// every pair (3 sub + 3 FMA + 1 exp), and one v_mfma_f32_16x16x4_f32 per 64 pairs
// contracts the 16 x 4 K block with a 4 x 16 block of per-column channels
//   W_j = [ p_j (D) | p_j^d qt_j^e (D*D) | 1 | qt_j (D) ],   qt = q' - c,
// so per row i the kernel sums S_i^n = sum_j K_ij W_j^n and the epilogue recovers the
// OpOdeSelfFwd sums (lddmm_ops.hpp; LDDMM.py:194-227, kernel.py KRed/GenDKRed/GradKRed) exactly
// in exact arithmetic:
//   V_i   = sum_j K p_j                                      = S[0:D]
//   Gs'_i = sum_j K (p_i.p_j)(q'_i - q'_j) = qt_i (p_i.V_i) - sum_d p_i^d S[D + D d + 0:D]
//   Z'_i  = sum_j K (q'_i - q'_j)          = qt_i S[D + D^2] - S[D + D^2 + 1:]
// The matrix pipe and the vector pipe of a SIMD run concurrently (MI355X_MICROARCH.md
// "Execution model"): the 16 per-pair FMAs of the channel sums move off the VALU, which keeps
// only the kernel evaluation.  One MFMA issue per 64 pairs (32 cycles) then bounds the loop,
// against ~53 cycles per 64 pairs for the packed-FP32 VALU forward (packed.hpp).
//
// Precision: the split z = q'_i - q'_j -> (qt_i, qt_j) trades cancellation for the GEMM form;
// the centre c is the mean of the workgroup's rows, so the cancellation factor is
// |qt| / |z| over the pairs that carry weight -- bounded by the rows' spread, which an optional
// row order (e.g. a spatial sort) keeps small.  The MFMA result is a k-ordered f32 fmaf chain
// (cdna_hip_programming.md §3); per-tile partial sums are folded into running totals once per
// 256-column tile (two-level accumulation, as common.hpp).
#pragma once
#include "launch.hpp"
#include "lddmm_ops.hpp"

namespace dicp {

typedef float mf4 __attribute__((ext_vector_type(4)));

constexpr int kMfRowTiles = 4;                 // 16-row MFMA tiles per wave
constexpr int kMfRowsWG = 4 * 16 * kMfRowTiles;  // 256 rows per workgroup (4 waves)
constexpr int kMfTile = 256;                   // columns per LDS tile (one per staging thread)
constexpr int kMfCh = 16;                      // channels per column record (B-operand width)
// largest row spread |q' - c| (scaled units) a workgroup may have and take the MFMA branch
// (dicp_set_option "mfma_rmax_x100"; 0 = never MFMA); the default is set in lddmm.hip
inline int& mfma_rmax_x100() {
  static int v = -1;
  return v;
}

template <int D, bool DIV>
struct MfFwd {
  static constexpr int kNCh = 2 * D + D * D + 1;  // channels in use (16 for D = 3)
  static_assert(kNCh <= kMfCh, "channel record too wide");
  static constexpr int kNOut = 4;
  static constexpr int kOutW[4] = {D, D, 1, 1};  // v, mG, g, h (as OpOdeSelfFwd)
};

// Wave-wide sum (fixed butterfly order: deterministic).
__device__ __forceinline__ float mf_wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int D, bool DIV>
__global__ __launch_bounds__(256) void mfma_fwd_kernel(Args a, Scal sc, int64_t M, int64_t N,
                                                       int64_t chunk, Outs outs,
                                                       const int* __restrict__ order, float rmax2) {
  using Op = MfFwd<D, DIV>;
  __shared__ float4 colW[2][kMfTile * kMfCh / 4];  // B-operand records, 64 B per column
  __shared__ float4 colQ[2][kMfTile];              // q'_j (xyz, w unused)
  __shared__ float red[4][D];

  const int tid = threadIdx.x, wv = tid >> 6, l = tid & 63;
  const int64_t i0 = (int64_t)blockIdx.x * kMfRowsWG;
  const float al = a.scale;
  float sh[D];
  load_shift<D>(a, sh);
  auto rowidx = [&](int64_t i) -> int64_t { return order ? (int64_t)order[i] : i; };

  // ---- centre c: mean of q' over this workgroup's rows (thread t: row i0 + t) ----
  const int64_t nvalid = (M - i0) < kMfRowsWG ? (M - i0) : kMfRowsWG;
  float c[D];
  {
    const int64_t ie = i0 + tid;
    float qe[D];
    if (ie < M) {
      const int64_t g = rowidx(ie);
#pragma unroll
      for (int d = 0; d < D; ++d) qe[d] = al * (a.r0[g * D + d] - sh[d]);
    } else {
#pragma unroll
      for (int d = 0; d < D; ++d) qe[d] = 0.f;
    }
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const float s = mf_wave_sum(qe[d]);
      if (l == 0) red[wv][d] = s;
    }
    __syncthreads();
    const float inv = 1.f / (float)nvalid;
#pragma unroll
    for (int d = 0; d < D; ++d) c[d] = (((red[0][d] + red[1][d]) + red[2][d]) + red[3][d]) * inv;
  }

  // ---- the lane's MFMA rows: tile rb, row 64 wv + 16 rb + (l & 15) (A operand row l & 15) ----
  float qr[kMfRowTiles][D];
#pragma unroll
  for (int rb = 0; rb < kMfRowTiles; ++rb) {
    int64_t ii = i0 + 64 * wv + 16 * rb + (l & 15);
    if (ii >= M) ii = M - 1;  // rows past the end: computed, never stored
    const int64_t g = rowidx(ii);
#pragma unroll
    for (int d = 0; d < D; ++d) qr[rb][d] = al * (a.r0[g * D + d] - sh[d]);
  }

  const int64_t j0 = (int64_t)blockIdx.y * chunk;
  int64_t j1 = j0 + chunk;
  if (j1 > N) j1 = N;

  // stage column tile [jt, jt + cnt) into buffer `buf`, zero records up to a multiple of 4
  auto stage = [&](int64_t jt, int cnt, int buf) {
    const int cnt4 = (cnt + 3) & ~3;
    if (tid < cnt4) {
      float w[kMfCh];
      float qj[D];
      if (tid < cnt) {
        const int64_t j = jt + tid;
        float pj[D], qt[D];
#pragma unroll
        for (int d = 0; d < D; ++d) {
          qj[d] = al * (a.c0[j * D + d] - sh[d]);
          pj[d] = a.c1[j * D + d];
          qt[d] = qj[d] - c[d];
        }
#pragma unroll
        for (int d = 0; d < D; ++d) w[d] = pj[d];
#pragma unroll
        for (int d = 0; d < D; ++d)
#pragma unroll
          for (int e = 0; e < D; ++e) w[D + D * d + e] = pj[d] * qt[e];
        w[D + D * D] = 1.f;
#pragma unroll
        for (int e = 0; e < D; ++e) w[D + D * D + 1 + e] = qt[e];
#pragma unroll
        for (int n = Op::kNCh; n < kMfCh; ++n) w[n] = 0.f;
      } else {  // padding column: K is finite, W = 0 -> contributes exactly 0
#pragma unroll
        for (int n = 0; n < kMfCh; ++n) w[n] = 0.f;
#pragma unroll
        for (int d = 0; d < D; ++d) qj[d] = 0.f;
      }
#pragma unroll
      for (int m = 0; m < kMfCh / 4; ++m)
        colW[buf][tid * (kMfCh / 4) + m] = make_float4(w[4 * m], w[4 * m + 1], w[4 * m + 2], w[4 * m + 3]);
      colQ[buf][tid] = make_float4(qj[0], qj[1], D > 2 ? qj[D - 1] : 0.f, 0.f);
    }
  };

  // ---- per-workgroup precision guard: the channel split's fp32 error is ~eps x (spread of
  // the rows about c) / |z| over the pairs that carry weight; a workgroup whose rows spread
  // wider than sqrt(rmax2) (scaled units, q' = q sqrt(log2 e / 2) / sigma) -- a sparse cloud, or rows not grouped in
  // space -- sums the pairs directly on the VALU instead (exactly the ordered-pair algebra of
  // OpOdeSelfFwd).  Uniform per workgroup and a function of its rows only, so every column
  // split of the workgroup takes the same branch.
  bool mf;
  {
    const int64_t ie = i0 + tid;
    float r2 = 0.f;
    if (ie < M) {
      const int64_t g = rowidx(ie);
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const float t = al * (a.r0[g * D + d] - sh[d]) - c[d];
        r2 = fmaf(t, t, r2);
      }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) r2 = fmaxf(r2, __shfl_xor(r2, o, 64));
    __syncthreads();  // red[] reuse
    if (l == 0) red[wv][0] = r2;
    __syncthreads();
    mf = fmaxf(fmaxf(red[0][0], red[1][0]), fmaxf(red[2][0], red[3][0])) <= rmax2;
  }

  int cnt = (int)((j1 - j0) < kMfTile ? (j1 - j0) : kMfTile);
  if (cnt > 0) stage(j0, cnt, 0);
  __syncthreads();
  int buf = 0;
  float* ep = reinterpret_cast<float*>(colW[0]);  // epilogue image: 256 rows x 16 floats = 16 KB
  if (mf) {
    mf4 tot[kMfRowTiles];
#pragma unroll
    for (int rb = 0; rb < kMfRowTiles; ++rb) tot[rb] = mf4{0.f, 0.f, 0.f, 0.f};
    for (int64_t jt = j0; jt < j1; jt += kMfTile) {
      const int64_t jn = jt + kMfTile;
      const int cntn = jn < j1 ? (int)((j1 - jn) < kMfTile ? (j1 - jn) : kMfTile) : 0;
      if (cntn > 0) stage(jn, cntn, buf ^ 1);  // the free buffer was consumed before the last barrier

      mf4 acc[kMfRowTiles];
#pragma unroll
      for (int rb = 0; rb < kMfRowTiles; ++rb) acc[rb] = mf4{0.f, 0.f, 0.f, 0.f};
      const float* Wt = reinterpret_cast<const float*>(colW[buf]);
      const float4* Qt = colQ[buf];
      const int nk = (cnt + 3) >> 2;
      const int jl = l >> 4, nl = l & 15;
      for (int kk = 0; kk < nk; ++kk) {
        const int j = 4 * kk + jl;             // A[m][k = l >> 4] / B[k = l >> 4][n = l & 15]
        const float4 qj = Qt[j];
        const float b = Wt[j * kMfCh + nl];
#pragma unroll
        for (int rb = 0; rb < kMfRowTiles; ++rb) {
          const float z0 = qr[rb][0] - qj.x;
          const float z1 = qr[rb][1] - qj.y;
          float r2 = fmaf(z1, z1, z0 * z0);
          if (D > 2) {
            const float z2 = qr[rb][D - 1] - qj.z;
            r2 = fmaf(z2, z2, r2);
          }
          const float K = fast_exp2(-r2);
          acc[rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(K, b, acc[rb], 0, 0, 0);
        }
      }
#pragma unroll
      for (int rb = 0; rb < kMfRowTiles; ++rb) tot[rb] += acc[rb];
      __syncthreads();
      buf ^= 1;
      cnt = cntn;
    }
    // channel sums of row t to thread t through LDS (D[m = 4(l>>4) + r][n = l&15])
#pragma unroll
    for (int rb = 0; rb < kMfRowTiles; ++rb)
#pragma unroll
      for (int r = 0; r < 4; ++r) ep[(64 * wv + 16 * rb + 4 * (l >> 4) + r) * kMfCh + (l & 15)] = tot[rb][r];
  } else {
    // direct pair sums, thread t = row i0 + t: V, Gs', Z' (OpOdeSelfFwd::pair, eta = 0)
    float qi[D], pi[D];
    {
      int64_t ii = i0 + tid;
      if (ii >= M) ii = M - 1;
      const int64_t g = rowidx(ii);
#pragma unroll
      for (int d = 0; d < D; ++d) {
        qi[d] = al * (a.r0[g * D + d] - sh[d]);
        pi[d] = a.r1[g * D + d];
      }
    }
    float tot[3 * D];
#pragma unroll
    for (int k = 0; k < 3 * D; ++k) tot[k] = 0.f;
    for (int64_t jt = j0; jt < j1; jt += kMfTile) {
      const int64_t jn = jt + kMfTile;
      const int cntn = jn < j1 ? (int)((j1 - jn) < kMfTile ? (j1 - jn) : kMfTile) : 0;
      if (cntn > 0) stage(jn, cntn, buf ^ 1);
      float acc[3 * D];
#pragma unroll
      for (int k = 0; k < 3 * D; ++k) acc[k] = 0.f;
      for (int j = 0; j < cnt; ++j) {
        const float4 qj4 = colQ[buf][j];
        const float4 pj4 = colW[buf][j * (kMfCh / 4)];  // channels 0..D-1 = p_j
        const float qj[3] = {qj4.x, qj4.y, qj4.z};
        const float pj[3] = {pj4.x, pj4.y, pj4.z};
        float z[D];
        float r2 = 0.f;
#pragma unroll
        for (int d = 0; d < D; ++d) {
          z[d] = qi[d] - qj[d];
          r2 = fmaf(z[d], z[d], r2);
        }
        const float K = fast_exp2(-r2);
        float pp = 0.f;
#pragma unroll
        for (int d = 0; d < D; ++d) pp = fmaf(pi[d], pj[d], pp);
        const float Kpp = K * pp;
#pragma unroll
        for (int d = 0; d < D; ++d) {
          acc[d] = fmaf(K, pj[d], acc[d]);
          acc[D + d] = fmaf(Kpp, z[d], acc[D + d]);
          if (DIV) acc[2 * D + d] = fmaf(K, z[d], acc[2 * D + d]);
        }
      }
#pragma unroll
      for (int k = 0; k < 3 * D; ++k) tot[k] += acc[k];
      __syncthreads();
      buf ^= 1;
      cnt = cntn;
    }
#pragma unroll
    for (int k = 0; k < 3 * D; ++k) ep[tid * kMfCh + k] = tot[k];
  }

  // ---- epilogue ----
  __syncthreads();
  const int64_t i = i0 + tid;
  if (i >= M) return;
  float S[kMfCh];
#pragma unroll
  for (int m = 0; m < kMfCh / 4; ++m) {
    const float4 v = colW[0][tid * (kMfCh / 4) + m];
    S[4 * m] = v.x, S[4 * m + 1] = v.y, S[4 * m + 2] = v.z, S[4 * m + 3] = v.w;
  }
  const int64_t g = rowidx(i);
  float qt[D], p[D];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    qt[d] = al * (a.r0[g * D + d] - sh[d]) - c[d];
    p[d] = a.r1[g * D + d];
  }
  const float* V = S;
  const float pV = dot<D>(p, V);
  const float sa = sc.aux1;  // s / alpha
  float vals[2 * D + 2];
  float pZ = 0.f;
  if (mf) {  // channel sums -> V, Gs', Z'
#pragma unroll
    for (int e = 0; e < D; ++e) {
      float B = 0.f;
#pragma unroll
      for (int d = 0; d < D; ++d) B = fmaf(p[d], S[D + D * d + e], B);
      vals[e] = V[e];
      vals[D + e] = sa * fmaf(qt[e], pV, -B);
      if (DIV) pZ = fmaf(p[e], fmaf(qt[e], S[D + D * D], -S[D + D * D + 1 + e]), pZ);
    }
  } else {   // direct sums V, Gs', Z'
#pragma unroll
    for (int e = 0; e < D; ++e) {
      vals[e] = V[e];
      vals[D + e] = sa * S[D + e];
      if (DIV) pZ = fmaf(p[e], S[2 * D + e], pZ);
    }
  }
  vals[2 * D] = DIV ? -sa * pZ : 0.f;
  vals[2 * D + 1] = 0.5f * pV;
  const bool split = gridDim.y > 1;
  int off = 0;
#pragma unroll
  for (int k = 0; k < Op::kNOut; ++k) {
    const int w = Op::kOutW[k];
    float* base = outs.ptr[k];
    if (base != nullptr) {
      if (split) {
        float* dst = base + (int64_t)blockIdx.y * M * w + g * w;
#pragma unroll
        for (int e = 0; e < w; ++e) dst[e] = vals[off + e];
      } else {
#pragma unroll
        for (int e = 0; e < w; ++e) base[g * w + e] = epilogue(outs, k, g * w + e, vals[off + e]);
      }
    }
    off += w;
  }
}

template <int D, bool DIV>
int64_t mfma_fwd_capacity() {
  static int64_t cap = -1;
  if (cap < 0) cap = (int64_t)device_cus() * blocks_per_cu(mfma_fwd_kernel<D, DIV>);
  return cap;
}

template <int D, bool DIV>
int mfma_fwd_splits(int64_t M, int64_t N) {
  // 256 rows per workgroup = kBlock x R with R = 1
  return num_splits_cap(M, N, kMfRowsWG / kBlock, mfma_fwd_capacity<D, DIV>());
}

template <int D, bool DIV>
size_t mfma_fwd_ws_bytes(int64_t M, int64_t N) {
  const int S = mfma_fwd_splits<D, DIV>(M, N);
  if (S <= 1) return 0;
  return (size_t)S * (size_t)M * (size_t)(2 * D + 2) * sizeof(float);
}

// Same contract as launch_rowred (launch.hpp): rows [0, M) x columns [0, N), outputs / epilogue
// in `fin`, split partial slabs carved from ws and merged in chunk order.  `order` (optional,
// M int32 row indices, a permutation) selects which rows share a workgroup.
template <int D, bool DIV>
int launch_mfma_fwd(const char* name, const Args& a, const Scal& sc, int64_t M, int64_t N,
                    const Outs& fin, void* ws, size_t ws_bytes, hipStream_t st,
                    const int* order = nullptr) {
  if (int rc = no_batch("ode_self_fwd(mfma)")) return rc;
  using Op = MfFwd<D, DIV>;
  if (M <= 0) return DICP_OK;
  const int S = mfma_fwd_splits<D, DIV>(M, N);
  const int64_t chunk = N > 0 ? chunk_of(N, S) : 0;
  const int64_t bx = (M + kMfRowsWG - 1) / kMfRowsWG;
  const float rm = 0.01f * (float)mfma_rmax_x100();
  const float rmax2 = mfma_rmax_x100() >= 100000 ? 3.0e38f : (mfma_rmax_x100() <= 0 ? -1.f : rm * rm);
  dim3 grid((unsigned)bx, (unsigned)S, 1), block(256, 1, 1);
  if (S == 1) {
    mfma_fwd_kernel<D, DIV><<<grid, block, 0, st>>>(a, sc, M, N, chunk, fin, order, rmax2);
    return check_launch(name);
  }
  const size_t need = mfma_fwd_ws_bytes<D, DIV>(M, N);
  if (ws == nullptr || ws_bytes < need) {
    set_error("%s: workspace too small (%zu < %zu bytes)", name, ws_bytes, need);
    return DICP_ERR_WORKSPACE;
  }
  Outs part = fin;
  float* cur = reinterpret_cast<float*>(ws);
  for (int k = 0; k < Op::kNOut; ++k) {
    part.ptr[k] = fin.ptr[k] ? cur : nullptr;
    cur += (int64_t)S * M * Op::kOutW[k];
  }
  mfma_fwd_kernel<D, DIV><<<grid, block, 0, st>>>(a, sc, M, N, chunk, part, order, rmax2);
  int rc = check_launch(name);
  if (rc) return rc;
  MergeSet ms;
  int nk = 0;
  int64_t nmax = 0;
  for (int k = 0; k < Op::kNOut; ++k) {
    if (!fin.ptr[k]) continue;
    ms.slab[nk] = part.ptr[k];
    ms.n[nk] = M * Op::kOutW[k];
    ms.k[nk] = k;
    nmax = ms.n[nk] > nmax ? ms.n[nk] : nmax;
    ++nk;
  }
  if (nk > 0) {
    const int64_t nb = (nmax + kBlock - 1) / kBlock;
    merge_slabs_kernel<false><<<dim3((unsigned)nb, (unsigned)nk), dim3(kBlock), 0, st>>>(ms, fin, S);
    rc = check_launch(name);
    if (rc) return rc;
  }
  return DICP_OK;
}

}  // namespace dicp
