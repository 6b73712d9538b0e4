// GMM EM-step reductions (GaussianMixtureUnif.EM_step_torch, diffICP/core/GMM.py:236-325)
// for gfx950.  Three passes, each one launch (+ a tiny finalize/merge launch):
//   E  (rows n, cols c): T_n = LSE_c t_nc and responsibility-weighted row sums  (GMM.py:263-270,
//      :296 NDsigma2 with the OLD mu, :303 Y, :312-314 Cfe terms)
//   M  (rows c, cols n): log sum_n gamma_nc and the gamma-weighted mean of x  (GMM.py:287, :293)
//   T  (rows n, cols c): targets / free-energy sums with OLD gamma, NEW mu, w  (GMM.py:303-314)
// LSE passes use the exact row maximum (first sweep, no exp) and then one exp2 per pair
// (second sweep), all in the log2 domain; column chunks (split mode) carry (max, sum, acc)
// partials merged with max-rescaling in chunk order -> deterministic, no atomics.
#include "launch.hpp"
#include "lddmm_ops.hpp"

using namespace dicp;

namespace {

constexpr int kRG = 2;  // rows per thread

// ---------------------------------------------------------------------------------------
// LSE row-reduction skeleton: part[(s*M + i)*(2+NACC) + ...] = {m, l, acc...} with
// m = max_j t_ij (log2 domain), l = sum_j 2^(t_ij - m), acc = Op::accum weighted sums.
// ---------------------------------------------------------------------------------------
template <class Op, int R>
__global__ __launch_bounds__(kBlock) void lse_rowred_kernel(Args args, Scal sc,
                                                            int64_t M, int64_t N, int64_t chunk,
                                                            float* __restrict__ part) {
  constexpr int CW4 = Op::CW4;
  constexpr int NACC = Op::NACC;
  constexpr int W = 2 + NACC;
  __shared__ float4 lds[kTile * CW4];
  const int tid = threadIdx.x;
  const int64_t ibase = (int64_t)blockIdx.x * (kBlock * R) + tid;
  typename Op::Row row[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    int64_t i = ibase + (int64_t)r * kBlock;
    if (i >= M) i = M - 1;
    Op::load_row(args, i, row[r]);
  }
  const int64_t j0 = (int64_t)blockIdx.y * chunk;
  int64_t j1 = j0 + chunk;
  if (j1 > N) j1 = N;

  // sweep 1: exact row maximum of the logits over this chunk
  float m[R];
#pragma unroll
  for (int r = 0; r < R; ++r) m[r] = -__builtin_huge_valf();
  for (int64_t jt = j0; jt < j1; jt += kTile) {
    const int cnt = (int)((j1 - jt) < kTile ? (j1 - jt) : kTile);
    if (tid < cnt) Op::load_col(args, jt + tid, reinterpret_cast<float*>(&lds[tid * CW4]));
    __syncthreads();
#pragma unroll 2
    for (int t = 0; t < cnt; ++t) {
      const float* rec = reinterpret_cast<const float*>(&lds[t * CW4]);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        float aux;
        m[r] = fmaxf(m[r], Op::logit(sc, row[r], rec, aux));
      }
    }
    __syncthreads();
  }
  // guard: an all -inf chunk contributes nothing (stored max stays -inf, merge skips it)
  float ms[R];
#pragma unroll
  for (int r = 0; r < R; ++r) ms[r] = (m[r] == -__builtin_huge_valf()) ? 0.f : m[r];

  // sweep 2: one exp2 per pair
  float tot[R][NACC + 1];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int k = 0; k <= NACC; ++k) tot[r][k] = 0.f;
  for (int64_t jt = j0; jt < j1; jt += kTile) {
    const int cnt = (int)((j1 - jt) < kTile ? (j1 - jt) : kTile);
    if (tid < cnt) Op::load_col(args, jt + tid, reinterpret_cast<float*>(&lds[tid * CW4]));
    __syncthreads();
    float acc[R][NACC + 1];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int k = 0; k <= NACC; ++k) acc[r][k] = 0.f;
#pragma unroll 2
    for (int t = 0; t < cnt; ++t) {
      const float* rec = reinterpret_cast<const float*>(&lds[t * CW4]);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        float aux;
        const float tm = Op::logit(sc, row[r], rec, aux) - ms[r];
        const float e = fast_exp2(tm);
        acc[r][0] += e;
        Op::accum(sc, row[r], rec, tm, aux, e, acc[r] + 1);
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int k = 0; k <= NACC; ++k) tot[r][k] += acc[r][k];
    __syncthreads();
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t i = ibase + (int64_t)r * kBlock;
    if (i >= M) continue;
    float* dst = part + ((int64_t)blockIdx.y * M + i) * W;
    dst[0] = m[r];
#pragma unroll
    for (int k = 0; k <= NACC; ++k) dst[1 + k] = tot[r][k];
  }
}

// Merge S chunk partials of each row (fixed order) and finalize through Op::finalize.
template <class Op>
__global__ __launch_bounds__(kBlock) void lse_finalize_kernel(const float* __restrict__ part,
                                                              int64_t M, int S, Scal sc,
                                                              Outs outs) {
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
  Op::finalize(sc, i, mx, l, acc, outs);
}

// ---- E-step op ------------------------------------------------------------------------
// rows x_n ; columns (mu_c, w2_c = (w_c - LSE w) log2 e, |mu_c|^2)
// logit t2 = w2_c + nc |x_n - mu_c|^2   (log2 domain, without -lgn)
// acc (STATS): sum e mu_c (D), sum e |mu_c|^2, sum e (t2 - m), sum e w2_c, sum e D2_nc
template <int D, bool STATS>
struct OpGmmE {
  static constexpr int CW4 = cw4(D + 2);
  static constexpr int NACC = STATS ? D + 4 : 0;
  static constexpr int kShifted = STATS ? D + 1 : -1;
  struct Row { float x[D]; };
  __device__ static void load_row(const Args& a, int64_t i, Row& r) { ld<D>(a.r0, i, r.x); }
  __device__ static void load_col(const Args& a, int64_t j, float* rec) {
    ld<D>(a.c0, j, rec);
    rec[D] = a.c1[j];
    rec[D + 1] = a.c2[j];
  }
  __device__ static float logit(const Scal& sc, const Row& r, const float* rec, float& d2) {
    float z[D];
    d2 = diff_sq<D>(r.x, rec, z);
    return fmaf(sc.nc, d2, rec[D]);
  }
  __device__ static void accum(const Scal&, const Row&, const float* rec, float tm, float d2,
                               float e, float* acc) {
    if (!STATS) return;
#pragma unroll
    for (int d = 0; d < D; ++d) acc[d] = fmaf(e, rec[d], acc[d]);
    acc[D] = fmaf(e, rec[D + 1], acc[D]);
    acc[D + 1] = fmaf(e, tm, acc[D + 1]);
    acc[D + 2] = fmaf(e, rec[D], acc[D + 2]);
    acc[D + 3] = fmaf(e, d2, acc[D + 3]);
  }
  // outs: ptr[0] = T (natural, with -lgn), ptr[1] = T2 (log2, no lgn), ptr[2] = stats (D+4)
  // sc.aux0 = lgn
  __device__ static void finalize(const Scal& sc, int64_t i, float m, float l, const float* acc,
                                  const Outs& o) {
    const float lg = fast_log2(l);
    const float T2 = m + lg;
    o.ptr[0][i] = kLn2 * T2 - sc.aux0;
    if (o.ptr[1]) o.ptr[1][i] = T2;
    if (STATS && o.ptr[2]) {
      const float il = 1.f / l;
      float* st = o.ptr[2] + i * (D + 4);
#pragma unroll
      for (int d = 0; d < D; ++d) st[d] = acc[d] * il;
      st[D] = acc[D] * il;
      st[D + 1] = kLn2 * (acc[D + 1] * il - lg);  // sum gamma lgamma
      st[D + 2] = kLn2 * acc[D + 2] * il;         // sum gamma lpi
      st[D + 3] = acc[D + 3] * il;                // sum gamma D2 (old mu)
    }
  }
};

// ---- M-step op (column pass as a row pass over components) ------------------------------
// rows c: (mu_c, w2_c) ; columns n: (x_n, T2_n)
// logit lg2 = w2_c + nc |x_n - mu_c|^2 - T2_n = log2 gamma_nc ; acc: sum e x_n (D)
template <int D>
struct OpGmmM {
  static constexpr int CW4 = cw4(D + 1);
  static constexpr int NACC = D;
  static constexpr int kShifted = -1;
  struct Row { float mu[D]; float w2; };
  __device__ static void load_row(const Args& a, int64_t i, Row& r) {
    ld<D>(a.r0, i, r.mu);
    r.w2 = a.r1[i];
  }
  __device__ static void load_col(const Args& a, int64_t j, float* rec) {
    ld<D>(a.c0, j, rec);
    rec[D] = a.c1[j];
  }
  __device__ static float logit(const Scal& sc, const Row& r, const float* rec, float& d2) {
    float z[D];
    d2 = diff_sq<D>(r.mu, rec, z);
    return fmaf(sc.nc, d2, r.w2 - rec[D]);
  }
  __device__ static void accum(const Scal&, const Row&, const float* rec, float, float, float e,
                               float* acc) {
#pragma unroll
    for (int d = 0; d < D; ++d) acc[d] = fmaf(e, rec[d], acc[d]);
  }
  // outs.ptr[0] = colstats (D+1): {log sum gamma, mean x (D)}
  __device__ static void finalize(const Scal&, int64_t i, float m, float l, const float* acc,
                                  const Outs& o) {
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
int lse_splits(int64_t M, int64_t N) {
  static int64_t cap = -1;
  if (cap < 0) cap = (int64_t)device_cus() * blocks_per_cu(lse_rowred_kernel<Op, R>);
  return num_splits_cap(M, N, R, cap);
}

template <class Op, int R>
size_t lse_ws_bytes(int64_t M, int64_t N) {
  const int S = lse_splits<Op, R>(M, N);
  return (size_t)S * (size_t)M * (size_t)(2 + Op::NACC) * sizeof(float);
}

template <class Op, int R>
int launch_lse(const char* name, const Args& a, const Scal& sc, int64_t M, int64_t N,
               const Outs& fin, void* ws, size_t ws_bytes, hipStream_t st) {
  if (M <= 0) return DICP_OK;
  const int S = lse_splits<Op, R>(M, N);
  const int64_t chunk = N > 0 ? chunk_of(N, S) : 0;
  const size_t need = lse_ws_bytes<Op, R>(M, N);
  if (ws == nullptr || ws_bytes < need) {
    set_error("%s: workspace too small (%zu < %zu bytes)", name, ws_bytes, need);
    return DICP_ERR_WORKSPACE;
  }
  const int64_t bx = (M + (int64_t)kBlock * R - 1) / ((int64_t)kBlock * R);
  float* part = reinterpret_cast<float*>(ws);
  lse_rowred_kernel<Op, R><<<dim3((unsigned)bx, (unsigned)S), dim3(kBlock), 0, st>>>(
      a, sc, M, N, chunk, part);
  int rc = check_launch(name);
  if (rc) return rc;
  const int64_t nb = (M + kBlock - 1) / kBlock;
  lse_finalize_kernel<Op><<<dim3((unsigned)nb), dim3(kBlock), 0, st>>>(part, M, S, sc, fin);
  return check_launch(name);
}

template <int D>
int estep_d(const float* X, int64_t N, const float* mu, const float* w2, const float* mu2,
            int64_t C, double sigma, double lgn, float* T, float* T2, float* stats, void* ws,
            size_t wsb, hipStream_t st) {
  const Args a = {X, nullptr, nullptr, nullptr, mu, w2, mu2, nullptr};
  Scal sc = make_scal(sigma, 0.0);
  sc.aux0 = (float)lgn;
  const Outs o = make_outs(T, T2, stats);
  if (stats) return launch_lse<OpGmmE<D, true>, kRG>("gmm_estep", a, sc, N, C, o, ws, wsb, st);
  return launch_lse<OpGmmE<D, false>, kRG>("gmm_estep", a, sc, N, C, o, ws, wsb, st);
}

}  // namespace

// The Python wrapper precomputes the C-sized column vectors (w2, |mu|^2, lpi) with torch on
// the device; the kernels here see only device pointers.
extern "C" int dicp_gmm_estep_f32(const float* X, int64_t N, const float* mu, const float* w2,
                                  const float* mu2, int64_t C, int D, double sigma, double lgn,
                                  float* T, float* T2, float* stats, void* ws, size_t ws_bytes,
                                  dicp_stream_t stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (N < 0 || C <= 0 || (N > 0 && (!X || !T)) || !mu || !w2 || !mu2 || !(sigma > 0)) {
    set_error("dicp_gmm_estep_f32: invalid arguments");
    return DICP_ERR_INVALID;
  }
  switch (D) {
    case 2: return estep_d<2>(X, N, mu, w2, mu2, C, sigma, lgn, T, T2, stats, ws, ws_bytes, st);
    case 3: return estep_d<3>(X, N, mu, w2, mu2, C, sigma, lgn, T, T2, stats, ws, ws_bytes, st);
    default: set_error("gmm_estep: D=%d unsupported", D); return DICP_ERR_UNSUPPORTED;
  }
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
  const Scal sc = make_scal(sigma, 0.0);
  const Outs o = make_outs(colstats);
  switch (D) {
    case 2: return launch_lse<OpGmmM<2>, kRG>("gmm_mstep", a, sc, C, N, o, ws, ws_bytes, st);
    case 3: return launch_lse<OpGmmM<3>, kRG>("gmm_mstep", a, sc, C, N, o, ws, ws_bytes, st);
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
    case DICP_WS_GMM_ESTEP: {  // both variants (their occupancies, hence splits, differ)
      size_t a = D == 2 ? lse_ws_bytes<OpGmmE<2, true>, kRG>(M, N) : lse_ws_bytes<OpGmmE<3, true>, kRG>(M, N);
      size_t b = D == 2 ? lse_ws_bytes<OpGmmE<2, false>, kRG>(M, N) : lse_ws_bytes<OpGmmE<3, false>, kRG>(M, N);
      return a > b ? a : b;
    }
    case DICP_WS_GMM_MSTEP:
      return D == 2 ? lse_ws_bytes<OpGmmM<2>, kRG>(N, M) : lse_ws_bytes<OpGmmM<3>, kRG>(N, M);
    case DICP_WS_GMM_TARGETS:
      return D == 2 ? rowred_ws_bytes<OpGmmTargets<2>, kRG>(M, N)
                    : rowred_ws_bytes<OpGmmTargets<3>, kRG>(M, N);
    default: return 0;
  }
}
