// Launchers of the centred-expansion reductions (centred.hpp): the prep pass (bounding box,
// Morton codes, stable rocPRIM radix sort, one wave per 64-column sub-tile building the
// records) and the main row pass with the usual deterministic split-column merge.
#include "centred.hpp"
#include "sym_cx.hpp"

#include <rocprim/device/device_radix_sort.hpp>

#include <cmath>

namespace dicp {

namespace {

inline size_t align256(size_t b) { return (b + 255) / 256 * 256; }

// rocPRIM's scratch for sorting n (uint32 key, int32 value) pairs; the size query needs the
// device (target selection) -- without one (host-only callers asking for workspace sizes)
// a safe bound is returned
size_t sort_temp_bytes(int64_t n) {
  size_t bytes = 0;
  uint32_t* k = nullptr;
  int32_t* v = nullptr;
  if (rocprim::radix_sort_pairs(nullptr, bytes, k, k, v, v, (unsigned int)n, 0, 30) != hipSuccess) {
    (void)hipGetLastError();
    bytes = (size_t)n * 16 + (8u << 20);
  }
  return bytes;
}

struct CxLayout {
  size_t box, keys0, keys1, vals0, vals1, recs, meta, sort, slabs, total;
};

CxLayout cx_layout(int64_t N, int rw4, int64_t slab_floats) {
  CxLayout L;
  const int64_t nsub = (N + kSub - 1) / kSub;
  size_t o = 0;
  L.box = o; o += align256((size_t)kBoxBlocks * 8 * sizeof(float));
  L.keys0 = o; o += align256((size_t)N * 4);
  L.keys1 = o; o += align256((size_t)N * 4);
  L.vals0 = o; o += align256((size_t)N * 4);
  L.vals1 = o; o += align256((size_t)N * 4);
  L.recs = o; o += align256((size_t)N * rw4 * 16);
  L.meta = o; o += align256((size_t)nsub * 16);
  L.sort = o; o += align256(sort_temp_bytes(N));
  L.slabs = o; o += align256((size_t)slab_floats * 4);
  L.total = o;
  return L;
}

template <class Op, int D, int R>
int64_t cx_capacity() {
  static int64_t cap = -1;
  if (cap < 0) cap = (int64_t)device_cus() * blocks_per_cu(cx_kernel<Op, D, R>);
  return cap;
}

template <class Op, int D, int R>
int cx_splits(int64_t M, int64_t N, int64_t* chunk) {
  const int S0 = num_splits_cap(M, N, R, cx_capacity<Op, D, R>());
  int64_t c = (N + S0 - 1) / S0;
  c = (c + kTile - 1) / kTile * kTile;
  *chunk = c;
  return (int)((N + c - 1) / c);
}

template <class Op, int D, int R>
size_t cx_ws(int64_t M, int64_t N) {
  int64_t chunk = 0;
  const int S = cx_splits<Op, D, R>(M, N, &chunk);
  const int64_t w = Op::kOutW[0] + Op::kOutW[1] + Op::kOutW[2] + Op::kOutW[3];
  return cx_layout(N, Op::RW4, S > 1 ? (int64_t)S * M * w : 0).total;
}

}  // namespace

int& cx_rho_x100() {
  static int v = 150;
  return v;
}
int& red_alg() {
  static int v = 1;
  return v;
}

bool cx_eligible(int64_t M, int64_t N, bool ext) {
  if (red_alg() == 0) return false;
  if (red_alg() == 2) return M > 0 && N > 0;
  // the prep pass (bounding box, Morton codes, radix sort, records) costs ~40-60 us: measured
  // break-even against the generic reductions between 20k x 20k (0.8x) and 50k x 50k (1.09x),
  // at 100k rows x 20k columns (1.04x) (tools/cx_ab.py, profiles/r03_ab_centred_shapes.json);
  // with the packed scaled-coordinate KRed below it, the centred form wins from 50k x 50k
  // (1.04x) and loses at 100k x 20k (0.91x) and 30k x 30k (0.80x) (profiles/r03_ab_cx_r4.json).
  // The external-point forward has a packed scaled-coordinate kernel below these sizes
  // (ext_pk.hpp, 1.2x the generic one), which the centred form only beats from ~50k x 50k on
  // (tools/ext_ab.py, profiles/r03_ab_ext_packed.json).
  if (ext) return N >= 32768 && (double)M * (double)N >= 2.5e9;
  return N >= 32768 && (double)M * (double)N >= 2.5e9;
}

// Launch the centred reduction Op over rows x (M, D) and columns (y, fields in a.c1..) (N).
// `fin`: final outputs (epilogue as the generic skeleton).
template <class Op, int D, int R>
int launch_cx(const char* name, const float* x, int64_t M, Args a, int64_t N, double sigma, double eta,
              const Outs& fin, void* ws, size_t wsb, hipStream_t st) {
  if (M <= 0) return DICP_OK;
  int64_t chunk = 0;
  const int S = cx_splits<Op, D, R>(M, N, &chunk);
  const int64_t w = Op::kOutW[0] + Op::kOutW[1] + Op::kOutW[2] + Op::kOutW[3];
  const CxLayout L = cx_layout(N, Op::RW4, S > 1 ? (int64_t)S * M * w : 0);
  if (ws == nullptr || wsb < L.total) {
    set_error("%s: workspace too small (%zu < %zu bytes)", name, wsb, L.total);
    return DICP_ERR_WORKSPACE;
  }
  char* base = reinterpret_cast<char*>(ws);
  float* box = reinterpret_cast<float*>(base + L.box);
  uint32_t* k0 = reinterpret_cast<uint32_t*>(base + L.keys0);
  uint32_t* k1 = reinterpret_cast<uint32_t*>(base + L.keys1);
  int32_t* v0 = reinterpret_cast<int32_t*>(base + L.vals0);
  int32_t* v1 = reinterpret_cast<int32_t*>(base + L.vals1);
  float4* recs = reinterpret_cast<float4*>(base + L.recs);
  float4* meta = reinterpret_cast<float4*>(base + L.meta);
  const double alpha = std::sqrt(1.4426950408889634 / (2.0 * sigma * sigma));
  Scal sc = make_scal(sigma, eta);
  sc.aux1 = (float)(1.0 / (sigma * sigma) / alpha);
  float rho = cx_rho_x100() / 100.f;
  if (rho > kCxRhoCap) rho = kCxRhoCap;   // the factored exponent's range (centred.hpp)
  // prep: sort the columns along a Morton curve, build the sub-tile records
  int64_t nparts = (N + 1023) / 1024;
  if (nparts > kBoxBlocks) nparts = kBoxBlocks;
  cx_bbox_kernel<D><<<(unsigned)nparts, 256, 0, st>>>(a.c0, N, box);
  int rc = check_launch(name);
  if (rc) return rc;
  cx_codes_kernel<D><<<(unsigned)((N + 255) / 256), 256, 0, st>>>(a.c0, N, box, (int)nparts, k0, v0);
  if ((rc = check_launch(name))) return rc;
  size_t tb = sort_temp_bytes(N);
  if (rocprim::radix_sort_pairs(base + L.sort, tb, k0, k1, v0, v1, (unsigned int)N, 0, 30, st) != hipSuccess) {
    (void)hipGetLastError();
    set_error("%s: rocprim radix sort failed", name);
    return DICP_ERR_HIP;
  }
  const int64_t nsub = (N + kSub - 1) / kSub;
  cx_build_kernel<D, Op><<<(unsigned)((nsub + 3) / 4), 256, 0, st>>>(a, N, (float)alpha, rho * rho, v1, recs, meta);
  if ((rc = check_launch(name))) return rc;
  const int64_t bx = (M + (int64_t)kBlock * R - 1) / ((int64_t)kBlock * R);
  dim3 grid((unsigned)bx, (unsigned)S, 1), block(kBlock, 1, 1);
  if (S == 1) {
    cx_kernel<Op, D, R><<<grid, block, 0, st>>>(x, M, (float)alpha, recs, meta, N, chunk, sc, fin);
    return check_launch(name);
  }
  Outs part = fin;
  float* cur = reinterpret_cast<float*>(base + L.slabs);
  for (int k = 0; k < Op::kNOut; ++k) {
    part.ptr[k] = fin.ptr[k] ? cur : nullptr;
    cur += (int64_t)S * M * Op::kOutW[k];
  }
  cx_kernel<Op, D, R><<<grid, block, 0, st>>>(x, M, (float)alpha, recs, meta, N, chunk, sc, part);
  if ((rc = check_launch(name))) return rc;
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
    if ((rc = check_launch(name))) return rc;
  }
  return DICP_OK;
}

int& sym_red() {
  static int v = 1;
  return v;
}
int& sym_red_rows() {
  static int v = 0;
  return v;
}

namespace {

// rows per lane of the pair-once sums: sym_red_rows 4 / 8 forces, 0 = automatic (8 from
// DICP_SCX8_MIN_M points)
// (8 rows measured slower at 100k -- 1.87 against 1.59 ms with 4 rows, L = 2 -- and equal at
// 200k: profiles/r05_ab_sym_red.jsonl; so 8 only when forced)
#ifndef DICP_SCX8_MIN_M
#define DICP_SCX8_MIN_M (int64_t(1) << 40)
#endif
bool scx_rows8(int64_t M) {
  if (sym_red_rows() == 4) return false;
  if (sym_red_rows() == 8) return true;
  return M >= DICP_SCX8_MIN_M;
}
// sym_geom wg_min: L halves until a launch has >= 8192 workgroups -- L = 2 at 100k (9580
// workgroups: 1.590 ms against 1.620 with L = 4), L = 1 at 50k, L = 8 from ~190k
// (profiles/r05_ab_sym_red.jsonl)
constexpr int kScxWgMin = 8192;

inline SymGeom scx_geom(int64_t M, bool rows8) {
  return sym_geom(M, 1, rows8 ? 2 * kScG : kScG, 4, kScxWgMin);
}

template <int D, int OPK>
size_t scx_ws(int64_t M) {
  if (M <= 0) return 0;
  const SymGeom g4 = scx_geom(M, false), g8 = scx_geom(M, true);
  const int ns = g4.nslot > g8.nslot ? g4.nslot : g8.nslot;
  return cx_layout(M, 3, (int64_t)ns * M * scx_w<D, OPK>).total;
}

// Pair-once centred sum (sym_cx.hpp) of rows = columns = x (M, D); f: the column fields
// (KRedScal: d (M,), KRed: b (M, D), KBase: none)
template <int D, int OPK>
int launch_scx(const char* name, const float* x, int64_t M, const float* f, double sigma,
               const Outs& fin, void* ws, size_t wsb, hipStream_t st) {
  if (M <= 0) return DICP_OK;
  constexpr int W = scx_w<D, OPK>;
  const bool rows8 = scx_rows8(M);
  const SymGeom g = scx_geom(M, rows8);
  const CxLayout L = cx_layout(M, 3, (int64_t)g.nslot * M * W);
  if (ws == nullptr || wsb < L.total) {
    set_error("%s: workspace too small (%zu < %zu bytes)", name, wsb, L.total);
    return DICP_ERR_WORKSPACE;
  }
  char* base = reinterpret_cast<char*>(ws);
  float* box = reinterpret_cast<float*>(base + L.box);
  uint32_t* k0 = reinterpret_cast<uint32_t*>(base + L.keys0);
  uint32_t* k1 = reinterpret_cast<uint32_t*>(base + L.keys1);
  int32_t* v0 = reinterpret_cast<int32_t*>(base + L.vals0);
  int32_t* v1 = reinterpret_cast<int32_t*>(base + L.vals1);
  float4* recs = reinterpret_cast<float4*>(base + L.recs);
  float4* meta = reinterpret_cast<float4*>(base + L.meta);
  float* slab = reinterpret_cast<float*>(base + L.slabs);
  const double alpha = std::sqrt(1.4426950408889634 / (2.0 * sigma * sigma));
  float rho = cx_rho_x100() / 100.f;
  if (rho > kCxRhoCap) rho = kCxRhoCap;
  int64_t nparts = (M + 1023) / 1024;
  if (nparts > kBoxBlocks) nparts = kBoxBlocks;
  cx_bbox_kernel<D><<<(unsigned)nparts, 256, 0, st>>>(x, M, box);
  int rc = check_launch(name);
  if (rc) return rc;
  cx_codes_kernel<D><<<(unsigned)((M + 255) / 256), 256, 0, st>>>(x, M, box, (int)nparts, k0, v0);
  if ((rc = check_launch(name))) return rc;
  size_t tb = sort_temp_bytes(M);
  if (rocprim::radix_sort_pairs(base + L.sort, tb, k0, k1, v0, v1, (unsigned int)M, 0, 30, st) != hipSuccess) {
    (void)hipGetLastError();
    set_error("%s: rocprim radix sort failed", name);
    return DICP_ERR_HIP;
  }
  const int64_t stride = M * W;
  const dim3 grid((unsigned)g.Kmax, (unsigned)g.nQ), mg((unsigned)((M + 255) / 256));
  if (rows8) {
    scx_group_kernel<D, OPK, 2 * kScG><<<(unsigned)g.nG, 256, 0, st>>>(x, f, M, (float)alpha, rho * rho, v1, recs, meta);
    if ((rc = check_launch(name))) return rc;
    scx_kernel<D, OPK, 4><<<grid, dim3(256), 0, st>>>(recs, meta, M, g.nG, g.L, (float)alpha, slab, stride);
    if ((rc = check_launch(name))) return rc;
    scx_merge_kernel<W, 2 * kScG><<<mg, 256, 0, st>>>(slab, stride, M, g.nG, g.L, v1, fin);
    return check_launch(name);
  }
  scx_group_kernel<D, OPK><<<(unsigned)g.nG, 256, 0, st>>>(x, f, M, (float)alpha, rho * rho, v1, recs, meta);
  if ((rc = check_launch(name))) return rc;
  scx_kernel<D, OPK, 2><<<grid, dim3(256), 0, st>>>(recs, meta, M, g.nG, g.L, (float)alpha, slab, stride);
  if ((rc = check_launch(name))) return rc;
  scx_merge_kernel<W><<<mg, 256, 0, st>>>(slab, stride, M, g.nG, g.L, v1, fin);
  return check_launch(name);
}

}  // namespace

#ifndef DICP_CX_R
#define DICP_CX_R 4
#endif
constexpr int kCxR = DICP_CX_R;  // rows per thread

template <int D>
int cx_gauss_red_d(int op, const float* x, int64_t M, const float* y, int64_t N, const float* b,
                   double sigma, float* out, void* ws, size_t wsb, hipStream_t st) {
  const Args a = {nullptr, nullptr, nullptr, nullptr, y, b, nullptr, nullptr, 0.f};
  const Outs o = make_outs(out);
  if (scx_eligible(op, x, M, y, N)) {   // rows = columns: the pair-once form (sym_cx.hpp)
    switch (op) {
      case DICP_KBASE: return launch_scx<D, 0>("KBase(sym cx)", x, M, nullptr, sigma, o, ws, wsb, st);
      case DICP_KREDSCAL: return launch_scx<D, 1>("KRedScal(sym cx)", x, M, b, sigma, o, ws, wsb, st);
      default: return launch_scx<D, 2>("KRed(sym cx)", x, M, b, sigma, o, ws, wsb, st);
    }
  }
  switch (op) {
    case DICP_KBASE: return launch_cx<CxKBase<D>, D, kCxR>("KBase(cx)", x, M, a, N, sigma, 0.0, o, ws, wsb, st);
    case DICP_KREDSCAL: return launch_cx<CxKRedScal<D>, D, kCxR>("KRedScal(cx)", x, M, a, N, sigma, 0.0, o, ws, wsb, st);
    case DICP_KRED: return launch_cx<CxKRed<D>, D, kCxR>("KRed(cx)", x, M, a, N, sigma, 0.0, o, ws, wsb, st);
    case DICP_GRADK: return launch_cx<CxGradK<D>, D, kCxR>("GradKRed(cx)", x, M, a, N, sigma, 0.0, o, ws, wsb, st);
    default: set_error("cx_gauss_red: op %d has no centred form", op); return DICP_ERR_UNSUPPORTED;
  }
}

// the pair-once form: x is y (same buffer and size), an op with a symmetric pair term, sym_red
// 1 (automatic: the centred form's size rule, cx_eligible) or 2 (always)
bool scx_eligible(int op, const float* x, int64_t M, const float* y, int64_t N) {
  if (sym_red() == 0 || x != y || M != N || M <= 0) return false;
  if (op != DICP_KBASE && op != DICP_KREDSCAL && op != DICP_KRED) return false;
  return sym_red() == 2 || red_alg() == 2 || (red_alg() == 1 && cx_eligible(M, N));
}

bool cx_has_op(int op) {
  return op == DICP_KBASE || op == DICP_KREDSCAL || op == DICP_KRED || op == DICP_GRADK;
}

int cx_gauss_red(int op, const float* x, int64_t M, const float* y, int64_t N, int D, const float* b,
                 double sigma, float* out, void* ws, size_t wsb, hipStream_t st) {
  return D == 2 ? cx_gauss_red_d<2>(op, x, M, y, N, b, sigma, out, ws, wsb, st)
                : cx_gauss_red_d<3>(op, x, M, y, N, b, sigma, out, ws, wsb, st);
}

template <int D>
int cx_ext_fwd_d(const float* x, int64_t N, const float* q, const float* p, int64_t M, double sigma,
                 double eta, float* vx, float* gx, void* ws, size_t wsb, hipStream_t st) {
  // rows = the external points x (N), columns = the support (q, p) (M)
  const Args a = {nullptr, nullptr, nullptr, nullptr, q, p, nullptr, nullptr, 0.f};
  const Outs o = make_outs(vx, gx);
  if (eta != 0.0)
    return gx ? launch_cx<CxExtFwd<D, true, true>, D, kCxR>("ode_ext_fwd(cx)", x, N, a, M, sigma, eta, o, ws, wsb, st)
              : launch_cx<CxExtFwd<D, true, false>, D, kCxR>("ode_ext_fwd(cx)", x, N, a, M, sigma, eta, o, ws, wsb, st);
  return gx ? launch_cx<CxExtFwd<D, false, true>, D, kCxR>("ode_ext_fwd(cx)", x, N, a, M, sigma, eta, o, ws, wsb, st)
            : launch_cx<CxExtFwd<D, false, false>, D, kCxR>("ode_ext_fwd(cx)", x, N, a, M, sigma, eta, o, ws, wsb, st);
}

int cx_ext_fwd(const float* x, int64_t N, const float* q, const float* p, int64_t M, int D, double sigma,
               double eta, float* vx, float* gx, void* ws, size_t wsb, hipStream_t st) {
  return D == 2 ? cx_ext_fwd_d<2>(x, N, q, p, M, sigma, eta, vx, gx, ws, wsb, st)
                : cx_ext_fwd_d<3>(x, N, q, p, M, sigma, eta, vx, gx, ws, wsb, st);
}

template <int D>
size_t cx_ws_d(int64_t M, int64_t N) {
  size_t m = 0;
  for (size_t v : {cx_ws<CxKBase<D>, D, kCxR>(M, N), cx_ws<CxKRedScal<D>, D, kCxR>(M, N),
                   cx_ws<CxKRed<D>, D, kCxR>(M, N), cx_ws<CxGradK<D>, D, kCxR>(M, N)})
    m = v > m ? v : m;
  if (M == N) {   // rows may be the columns: the pair-once form
    for (size_t v : {scx_ws<D, 0>(M), scx_ws<D, 1>(M), scx_ws<D, 2>(M)}) m = v > m ? v : m;
  }
  return m;
}

// workspace of the centred reductions: rows M, columns N (gauss_red), or rows N (external
// points), columns M (support) for the external-point forward
size_t cx_red_ws(int64_t M, int64_t N, int D) {
  if (D != 2 && D != 3) return 0;
  return D == 2 ? cx_ws_d<2>(M, N) : cx_ws_d<3>(M, N);
}

template <int D>
size_t cx_ext_ws_d(int64_t N, int64_t M) {
  size_t m = 0;
  for (size_t v : {cx_ws<CxExtFwd<D, true, true>, D, kCxR>(N, M), cx_ws<CxExtFwd<D, true, false>, D, kCxR>(N, M),
                   cx_ws<CxExtFwd<D, false, true>, D, kCxR>(N, M), cx_ws<CxExtFwd<D, false, false>, D, kCxR>(N, M)})
    m = v > m ? v : m;
  return m;
}

size_t cx_ext_ws(int64_t N, int64_t M, int D) {
  if (D != 2 && D != 3) return 0;
  return D == 2 ? cx_ext_ws_d<2>(N, M) : cx_ext_ws_d<3>(N, M);
}

}  // namespace dicp
