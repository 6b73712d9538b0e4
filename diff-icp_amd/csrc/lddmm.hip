// C-ABI entry points of the Gaussian-kernel reductions (GenKernel, kernel.py:58-337) and of
// the fused LDDMM geodesic-shooting ODE (LDDMMModel.ODE, LDDMM.py:176-227) for gfx950.
#include "launch.hpp"
#include "lddmm_ops.hpp"
#include "lddmm_sym.hpp"
#include "packed.hpp"
#include "lddmm_sym_pk.hpp"
#include "mfma_fwd.hpp"
#include "ext_pk.hpp"

#include <stdlib.h>

#include <cmath>

using namespace dicp;

namespace {

#ifndef DICP_KR
#define DICP_KR 2
#endif
constexpr int kR = DICP_KR;  // rows per thread for the light reductions (KRed etc.)

// Rows per thread of the fused ODE passes (tuning knobs, env DICP_R_FWD / DICP_R_BWD in
// {1, 2, 4}; read once).  Defaults chosen from measurements on MI355X.
int env_r(const char* name, int def) {
  const char* v = getenv(name);
  if (!v) return def;
  const int r = atoi(v);
  return (r == 1 || r == 2 || r == 4) ? r : def;
}
int g_r_fwd = -1, g_r_bwd = -1;
int r_fwd() { if (g_r_fwd < 0) g_r_fwd = env_r("DICP_R_FWD", 2); return g_r_fwd; }
int r_bwd() { if (g_r_bwd < 0) g_r_bwd = env_r("DICP_R_BWD", 1); return g_r_bwd; }
// eta = 0 VJP: 0 = OpOdeSelfBwd (55 VALU/pair), 1 = OpOdeSelfBwd2 (48), 2 = symmetric
// pair-once kernel (lddmm_sym.hpp, ~32 VALU per ordered pair), 3 = the same pair-once
// decomposition with the lane's two rows packed as float2 (lddmm_sym_pk.hpp, v_pk_*_f32; default: 5-7% faster on MI355X at 50k-100k)
int g_bwd_alg = 3;
// eta != 0 VJP: 0 = ordered OpOdeSelfBwdEta, 1 = symmetric pair-once SymBwdEta (lddmm_sym.hpp),
// 2 = the same with packed-FP32 rows (lddmm_sym_pk.hpp SymBwdEtaPk)
#ifndef DICP_BWD_ETA_ALG
#define DICP_BWD_ETA_ALG 2
#endif
int g_bwd_eta_alg = DICP_BWD_ETA_ALG;
// external-point passes and KRed below the centred path's sizes: 0 = generic scalar rows in
// original units (OpOdeExtFwd / OpOdeExtBwdX / OpOdeExtBwdQ / OpKRed), 1 = packed-FP32 rows in
// scaled coordinates (ext_pk.hpp; the external-point VJP only for eta = 0)
int g_ext_alg = 1;
// coordinates of the default packed shooting kernels (OpOdeSelfFwdPk, SymBwdPk): 0 = scaled,
// q' = alpha (q - q_0), one packed multiply per two pairs fewer; 1 = original units, exact
// differences whatever the cloud's extent.  Per HOST THREAD (the shooting
// sets it around its own launches; concurrent frames run on their own threads).
thread_local int tl_coord_raw = 0;
// eta = 0 forward: 0 = OpOdeSelfFwd (ordered rows, R = 2), 1 = symmetric pair-once kernel
// (lddmm_sym.hpp SymFwd: 17 VALU + 0.5 exp per ordered pair instead of 20 + 1, but 3-5%
// slower: issue-stalled on its rotating column sums), 2 = packed-FP32 rows (packed.hpp: the
// thread's two rows as float2, 11 VALU instructions per pair; measured 4-11% faster
// than 0 at 200k-20k on MI355X), 3 = the column contraction on the matrix cores
// (mfma_fwd.hpp: VALU evaluates K, one v_mfma_f32_16x16x4_f32 per 64 pairs sums 16 channels;
// eta = 0 only, eta != 0 keeps 2), 4 = the symmetric pair-once kernel with packed-FP32 rows
// (lddmm_sym_pk.hpp SymFwdPk; all rows only, row slices take 2)
#ifndef DICP_FWD_ALG
#define DICP_FWD_ALG 2
#endif
int g_fwd_alg = DICP_FWD_ALG;
#ifndef DICP_MFMA_RMAX_X100
#define DICP_MFMA_RMAX_X100 300
#endif
struct MfmaRmaxInit {
  MfmaRmaxInit() { if (mfma_rmax_x100() < 0) mfma_rmax_x100() = DICP_MFMA_RMAX_X100; }
} g_mfma_rmax_init;

template <class Op>
int launch_r(int R, const char* name, const Args& a, const Scal& sc, int64_t M, int64_t N,
             const Outs& o, void* ws, size_t wsb, hipStream_t st) {
  switch (R) {
    case 1: return launch_rowred<Op, 1>(name, a, sc, M, N, o, ws, wsb, st);
    case 4: return launch_rowred<Op, 4>(name, a, sc, M, N, o, ws, wsb, st);
    default: return launch_rowred<Op, 2>(name, a, sc, M, N, o, ws, wsb, st);
  }
}

template <class Op>
size_t ws_r(int R, int64_t M, int64_t N) {
  switch (R) {
    case 1: return rowred_ws_bytes<Op, 1>(M, N);
    case 4: return rowred_ws_bytes<Op, 4>(M, N);
    default: return rowred_ws_bytes<Op, 2>(M, N);
  }
}

template <template <int> class OpT>
int red_dispatch(const char* name, int D, const Args& a, const Scal& sc, int64_t M, int64_t N,
                 float* out, void* ws, size_t wsb, hipStream_t st) {
  const Outs o = make_outs(out);
  switch (D) {
    case 2: return launch_rowred<OpT<2>, kR>(name, a, sc, M, N, o, ws, wsb, st);
    case 3: return launch_rowred<OpT<3>, kR>(name, a, sc, M, N, o, ws, wsb, st);
    default: set_error("%s: D=%d not compiled in (supported: 2, 3)", name, D);
      return DICP_ERR_UNSUPPORTED;
  }
}

template <int D> using OpGradLapKPlain = OpGradLapK<D, false>;
template <int D> using OpGradLapKScal = OpGradLapK<D, true>;

template <template <int> class OpT>
size_t red_ws(int D, int64_t M, int64_t N) {
  return D == 2 ? rowred_ws_bytes<OpT<2>, kR>(M, N) : rowred_ws_bytes<OpT<3>, kR>(M, N);
}

bool supported_dim(int D) { return D == 2 || D == 3; }

// Scaled-coordinate ops (OpOdeSelfFwd / OpOdeSelfBwd): alpha = sqrt(log2 e / (2 sigma^2)),
// aux1 = s / alpha.
// The coordinate origin is the first column point (a.c0: the support q of the self ops, the
// support of the external-point x pass, y of KRed), the same for rows and columns.
void scale_coords(Args& a, Scal& sc, double sigma) {
  const double alpha = std::sqrt(1.4426950408889634 / (2.0 * sigma * sigma));
  a.scale = (float)alpha;
  a.shift = a.c0;
  sc.aux1 = (float)(1.0 / (sigma * sigma) / alpha);
}

// original-unit coordinates for the RAW packed kernels: alpha = 1, no shift, aux1 = s / 1
void raw_coords(Args& a, Scal& sc) {
  a.scale = 1.f;
  a.shift = nullptr;
  sc.aux1 = sc.s;
}

template <class OpS, class OpR>
int launch_fwd_pk(bool raw, const char* name, Args a, Scal sc, int64_t nrows, int64_t M, const Outs& o,
                  void* ws, size_t wsb, hipStream_t st) {
  if (raw) {
    raw_coords(a, sc);
    return launch_rowred_pk<OpR>(name, a, sc, nrows, M, o, ws, wsb, st);
  }
  return launch_rowred_pk<OpS>(name, a, sc, nrows, M, o, ws, wsb, st);
}
template <class OpS, class OpR>
size_t fwd_pk_ws(int64_t nrows, int64_t M) {
  const size_t a = rowred_pk_ws_bytes<OpS>(nrows, M), b = rowred_pk_ws_bytes<OpR>(nrows, M);
  return a > b ? a : b;
}

}  // namespace

extern "C" int dicp_supports_dim(int D) { return supported_dim(D) ? 1 : 0; }

// Tuning knobs (A/B measurements in one process): "r_fwd", "r_bwd" in {1, 2, 4}.
extern "C" int dicp_set_option(const char* name, int value) {
  if (!strcmp(name, "split_rounds")) {
    if (value < 0 || value > 64) return DICP_ERR_INVALID;  // 0 = automatic
    split_rounds() = value;
    return DICP_OK;
  }
  if (!strcmp(name, "sym_L")) {
    if (value < 0 || value > 64) return DICP_ERR_INVALID;  // 0 = automatic
    sym_L() = value;
    return DICP_OK;
  }
  if (!strcmp(name, "min_chunk")) {
    if (value != 0 && (value < 16 || value > 65536)) return DICP_ERR_INVALID;   // 0 = automatic
    min_chunk() = value;
    return DICP_OK;
  }
  if (!strcmp(name, "force_splits")) {
    if (value < 0 || value > 65536) return DICP_ERR_INVALID;
    force_splits() = value;
    return DICP_OK;
  }
  if (!strcmp(name, "batch_share")) {   // PER HOST THREAD geometry hint (batch.hpp)
    if (value < 1 || value > 4096) return DICP_ERR_INVALID;
    tl_batch_share = value;
    return DICP_OK;
  }
  if (!strcmp(name, "sym_rp")) {   // packed eta = 0 VJP: row pairs per lane (1, 2), 0 = automatic
    if (value < 0 || value > 2) return DICP_ERR_INVALID;
    sym_rp() = value;
    return DICP_OK;
  }
  if (!strcmp(name, "pk_rp")) {   // packed row passes: row pairs per thread, 0 = automatic
    if (value < 0 || value > kPkRPMax) return DICP_ERR_INVALID;
    pk_rp_force() = value;
    return DICP_OK;
  }
  if (!strcmp(name, "fwd_alg")) {
    if (value < 0 || value > 6) return DICP_ERR_INVALID;
    g_fwd_alg = value;
    return DICP_OK;
  }
  if (!strcmp(name, "mfma_rmax_x100")) {  // >= 100000: always the MFMA branch, 0: never
    if (value < 0) return DICP_ERR_INVALID;
    mfma_rmax_x100() = value;
    return DICP_OK;
  }
  if (!strcmp(name, "bwd_eta_alg")) {
    if (value < 0 || value > 2) return DICP_ERR_INVALID;
    g_bwd_eta_alg = value;
    return DICP_OK;
  }
  if (!strcmp(name, "bwd_alg")) {
    if (value < 0 || value > 3) return DICP_ERR_INVALID;
    g_bwd_alg = value;
    return DICP_OK;
  }
  if (!strcmp(name, "red_alg")) {
    if (value < 0 || value > 2) return DICP_ERR_INVALID;
    red_alg() = value;
    return DICP_OK;
  }
  if (!strcmp(name, "coord_raw")) {
    if (value < 0 || value > 1) return DICP_ERR_INVALID;
    tl_coord_raw = value;
    return DICP_OK;
  }
  if (!strcmp(name, "ext_alg")) {
    if (value < 0 || value > 1) return DICP_ERR_INVALID;
    g_ext_alg = value;
    return DICP_OK;
  }
  if (!strcmp(name, "cx_rho_x100")) {
    if (value < 0 || value > 100000) return DICP_ERR_INVALID;
    cx_rho_x100() = value;
    return DICP_OK;
  }
  if (!strcmp(name, "sym_fwd_rows")) {
    if (value != 0 && value != 4 && value != 6 && value != 8) return DICP_ERR_INVALID;
    sym_fwd_rows() = value;
    return DICP_OK;
  }
  if (!strcmp(name, "sym_red")) {
    if (value < 0 || value > 2) return DICP_ERR_INVALID;
    sym_red() = value;
    return DICP_OK;
  }
  if (!strcmp(name, "lse_adapt")) {
    if (value < 0) return DICP_ERR_INVALID;
    lse_adapt() = value;
    return DICP_OK;
  }
  if (!strcmp(name, "lse_bound")) {
    if (value < 0 || value > 1) return DICP_ERR_INVALID;
    lse_bound() = value;
    return DICP_OK;
  }
  if (!strcmp(name, "lse_pk")) {
    if (value < 0 || value > 1) return DICP_ERR_INVALID;
    lse_pk() = value;
    return DICP_OK;
  }
  if (!strcmp(name, "sym_red_rows")) {
    if (value != 0 && value != 4 && value != 8) return DICP_ERR_INVALID;
    sym_red_rows() = value;
    return DICP_OK;
  }
  if (value != 1 && value != 2 && value != 4) return DICP_ERR_INVALID;
  if (!strcmp(name, "r_fwd")) { g_r_fwd = value; return DICP_OK; }
  if (!strcmp(name, "r_bwd")) { g_r_bwd = value; return DICP_OK; }
  set_error("dicp_set_option: unknown option %s", name);
  return DICP_ERR_INVALID;
}

extern "C" int dicp_get_option(const char* name, int* value) {
  if (name == nullptr || value == nullptr) {
    set_error("dicp_get_option: NULL argument");
    return DICP_ERR_INVALID;
  }
  if (!strcmp(name, "split_rounds")) { *value = split_rounds(); return DICP_OK; }
  if (!strcmp(name, "sym_L")) { *value = sym_L(); return DICP_OK; }
  if (!strcmp(name, "force_splits")) { *value = force_splits(); return DICP_OK; }
  if (!strcmp(name, "min_chunk")) { *value = (int)min_chunk(); return DICP_OK; }
  if (!strcmp(name, "pk_rp")) { *value = pk_rp_force(); return DICP_OK; }
  if (!strcmp(name, "sym_rp")) { *value = sym_rp(); return DICP_OK; }
  if (!strcmp(name, "batch_share")) { *value = batch_share(); return DICP_OK; }
  if (!strcmp(name, "fwd_alg")) { *value = g_fwd_alg; return DICP_OK; }
  if (!strcmp(name, "mfma_rmax_x100")) { *value = mfma_rmax_x100(); return DICP_OK; }
  if (!strcmp(name, "bwd_eta_alg")) { *value = g_bwd_eta_alg; return DICP_OK; }
  if (!strcmp(name, "bwd_alg")) { *value = g_bwd_alg; return DICP_OK; }
  if (!strcmp(name, "red_alg")) { *value = red_alg(); return DICP_OK; }
  if (!strcmp(name, "cx_rho_x100")) { *value = cx_rho_x100(); return DICP_OK; }
  if (!strcmp(name, "sym_red")) { *value = sym_red(); return DICP_OK; }
  if (!strcmp(name, "lse_pk")) { *value = lse_pk(); return DICP_OK; }
  if (!strcmp(name, "lse_adapt")) { *value = lse_adapt(); return DICP_OK; }
  if (!strcmp(name, "lse_bound")) { *value = lse_bound(); return DICP_OK; }
  if (!strcmp(name, "sym_red_rows")) { *value = sym_red_rows(); return DICP_OK; }
  if (!strcmp(name, "sym_fwd_rows")) { *value = sym_fwd_rows(); return DICP_OK; }
  if (!strcmp(name, "ext_alg")) { *value = g_ext_alg; return DICP_OK; }
  if (!strcmp(name, "coord_raw")) { *value = tl_coord_raw; return DICP_OK; }
  if (!strcmp(name, "r_fwd")) { *value = r_fwd(); return DICP_OK; }
  if (!strcmp(name, "r_bwd")) { *value = r_bwd(); return DICP_OK; }
  set_error("dicp_get_option: unknown option %s", name);
  return DICP_ERR_INVALID;
}

extern "C" int dicp_gauss_red_f32(int op, const float* x, int64_t M, const float* y, int64_t N,
                                  int D, const float* b, const float* c, double sigma, float* out,
                                  void* ws, size_t ws_bytes, dicp_stream_t stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (M < 0 || N < 0 || (M > 0 && (!x || !out)) || (N > 0 && !y) || !(sigma > 0)) {
    set_error("dicp_gauss_red_f32: invalid arguments");
    return DICP_ERR_INVALID;
  }
  Args a = {x, c, nullptr, nullptr, y, b, nullptr, nullptr};
  const Scal sc = make_scal(sigma, 0.0);
  const bool needb = op == DICP_KREDSCAL || op == DICP_KRED || op == DICP_GRADK_REV ||
                     op == DICP_DDK || op == DICP_GENDK || op == DICP_HESSK ||
                     op == DICP_GRADKSCAL || op == DICP_GRADLAPKSCAL;
  const bool needc = op == DICP_GENDK || op == DICP_HESSK;
  if ((needb && N > 0 && !b) || (needc && M > 0 && !c)) {
    set_error("dicp_gauss_red_f32: op %d needs b%s", op, needc ? " and c" : "");
    return DICP_ERR_INVALID;
  }
  if (cx_has_op(op) && (D == 2 || D == 3) && (cx_eligible(M, N) || scx_eligible(op, x, M, y, N)))
    return cx_gauss_red(op, x, M, y, N, D, b, sigma, out, ws, ws_bytes, st);
  if (op == DICP_KRED && g_ext_alg == 1 && (D == 2 || D == 3) && N > 0) {
    // KRed = the external-point forward's velocity sum: the packed scaled-coordinate kernel
    const Args ak = {x, nullptr, nullptr, nullptr, y, b, nullptr, nullptr};
    const Scal sk = make_scal(sigma, 0.0);
    const Outs o = make_outs(out);
    return D == 2 ? launch_rowred_pk<OpExtFwdPk<2, false, false>>("KRed", ak, sk, M, N, o, ws, ws_bytes, st)
                  : launch_rowred_pk<OpExtFwdPk<3, false, false>>("KRed", ak, sk, M, N, o, ws, ws_bytes, st);
  }
  switch (op) {
    case DICP_KBASE: return red_dispatch<OpKBase>("KBase", D, a, sc, M, N, out, ws, ws_bytes, st);
    case DICP_KREDSCAL: return red_dispatch<OpKRedScal>("KRedScal", D, a, sc, M, N, out, ws, ws_bytes, st);
    case DICP_KRED: return red_dispatch<OpKRed>("KRed", D, a, sc, M, N, out, ws, ws_bytes, st);
    case DICP_GRADK: return red_dispatch<OpGradK>("GradKRed", D, a, sc, M, N, out, ws, ws_bytes, st);
    case DICP_GRADK_REV: return red_dispatch<OpZDotB>("GradKRed_rev", D, a, sc, M, N, out, ws, ws_bytes, st);
    case DICP_DDK: return red_dispatch<OpDDK>("DDKRed", D, a, sc, M, N, out, ws, ws_bytes, st);
    case DICP_GENDK: return red_dispatch<OpGenDK>("GenDKRed", D, a, sc, M, N, out, ws, ws_bytes, st);
    case DICP_HESSK: return red_dispatch<OpHessK>("HessKRed", D, a, sc, M, N, out, ws, ws_bytes, st);
    case DICP_LAPK: return red_dispatch<OpLapK>("LapKRed", D, a, sc, M, N, out, ws, ws_bytes, st);
    case DICP_GRADLAPK: return red_dispatch<OpGradLapKPlain>("GradLapKRed", D, a, sc, M, N, out, ws, ws_bytes, st);
    case DICP_GRADKSCAL: return red_dispatch<OpGradKScal>("GradKScal", D, a, sc, M, N, out, ws, ws_bytes, st);
    case DICP_GRADLAPKSCAL: return red_dispatch<OpGradLapKScal>("GradLapKScal", D, a, sc, M, N, out, ws, ws_bytes, st);
    case DICP_MIN_SQDIST: return red_dispatch<OpMinSqDist>("MinSqDist", D, a, sc, M, N, out, ws, ws_bytes, st);
    case DICP_MIN_SQDIST_OTHER:
      if (N != M || x != y || M > INT32_MAX) {
        set_error("dicp_gauss_red_f32: MIN_SQDIST_OTHER needs y == x (same buffer, M == N < 2^31)");
        return DICP_ERR_INVALID;
      }
      return red_dispatch<OpMinSqDistOther>("MinSqDistOther", D, a, sc, M, N, out, ws, ws_bytes, st);
    default: set_error("dicp_gauss_red_f32: unknown op %d", op); return DICP_ERR_UNSUPPORTED;
  }
}

extern "C" int dicp_radius_count_f32(const float* x, int64_t M, const float* y, int64_t N, int D,
                                     double R, float* counts, void* ws, size_t ws_bytes,
                                     dicp_stream_t stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (M < 0 || N < 0 || (M > 0 && (!x || !counts)) || (N > 0 && !y) || !(R >= 0)) {
    set_error("dicp_radius_count_f32: invalid arguments");
    return DICP_ERR_INVALID;
  }
  const Args a = {x, nullptr, nullptr, nullptr, y, nullptr, nullptr, nullptr};
  Scal sc = make_scal(1.0, 0.0);
  sc.aux0 = (float)(R * R);  // torch compares the float32 distances with (float)(R**2)
  return red_dispatch<OpRadiusCount>("RadiusCount", D, a, sc, M, N, counts, ws, ws_bytes, st);
}

// ---------------------------------------------------------------------------------------
// Fused ODE
// ---------------------------------------------------------------------------------------
namespace {

// packed forward algorithms: 2 (default: ordered rows, the symmetric 4-row pass for whole
// passes from DICP_SYM_FWD4_MIN_M points), 5 (symmetric 4-row wherever it applies), 6 (ordered
// rows always)
bool packed_fwd_alg() { return g_fwd_alg == 2 || g_fwd_alg == 5 || g_fwd_alg == 6; }
#ifndef DICP_SYM_FWD4_MIN_M
#define DICP_SYM_FWD4_MIN_M 20000
#endif
// The symmetric 4-row forward (SymFwdPk4) for this pass?  Whole passes (all rows) in scaled
// coordinates only.  Automatic rule (fwd_alg 2), measured on MI355X: with the column groups
// of sym_geom's wg_min 4096 rule the Euler step with divergence rows is 1.03x the ordered
// pass at 20k, 1.10x at 40k, 1.01x at 50k, 1.07x at 60k, 1.10x at 80k-200k
// (tools/probes/sym_L_rows4.py KIND=fwd, profiles/r04_ab_fwd4_L_small.jsonl; with L = 4 it lost
// below 75k: r04_ab_fwd_sym4.jsonl) -- from 20k points, or, with the geometry hint
// batch_share > 1 (concurrent / batched frames), when the sharing calls have >= 1e9 pairs
// (as the 4-row VJP, lddmm_sym.hpp DICP_SYM_SHARE4_MIN_PAIRS).
bool use_sym_fwd4(int64_t M, bool all, bool raw) {
  if (!all || raw || g_fwd_alg == 6 || !(g_fwd_alg == 2 || g_fwd_alg == 5)) return false;
  if (g_fwd_alg == 5) return true;
  if (batch_share() > 1) return M >= 8192 && (double)M * (double)M * batch_share() >= DICP_SYM_SHARE4_MIN_PAIRS;
  return M >= DICP_SYM_FWD4_MIN_M;
}

// rows per lane of the symmetric forward (SymFwdPkN) when the pass runs alone on the chip
// (batch_share 1; a lockstep batch takes each frame's own rule, so a batched call equals the
// call made alone bitwise): 6 (384-point groups, 3 waves / SIMD) from
// DICP_SYM_FWD6_MIN_M points, 8 (512-point groups, 2 waves / SIMD) from DICP_SYM_FWD8_MIN_M,
// else 4; sym_fwd_rows 4 / 6 / 8 forces.  Measured r06 (tools/probes/symfwd_L.py, the Euler
// step with divergence rows, profiles/r06_symfwd_rows.jsonl): 6 rows against 4 -2% at 40k,
// -4% at 60k, -5% at 80k-100k (3.235 vs 3.394 ms at the north_star's 100k), -4% / -7% at
// 120k / 150k; 8 rows lose at 100k (3.86: 2 workgroups per CU, a ragged last round) and win
// from ~200k (12.67 vs 13.02 ms)
#ifndef DICP_SYM_FWD6_MIN_M
#define DICP_SYM_FWD6_MIN_M 40000
#endif
#ifndef DICP_SYM_FWD8_MIN_M
#define DICP_SYM_FWD8_MIN_M 180000
#endif
int sym_fwd_rows_for(int64_t M) {
  const int f = sym_fwd_rows();
  if (f == 4 || f == 6 || f == 8) return f;
  if (batch_share() > 1) return 4;
  return M >= DICP_SYM_FWD8_MIN_M ? 8 : M >= DICP_SYM_FWD6_MIN_M ? 6 : 4;
}
template <int D, bool DIV>
int launch_sym_fwd_rows(const Args& a, const Scal& sc, int64_t M, const Outs& o, void* ws, size_t wsb,
                        hipStream_t st, bool zs) {
  switch (sym_fwd_rows_for(M)) {
    case 8: return launch_sym_fwd8<D, DIV>(a, sc, M, o, ws, wsb, st, zs);
    case 6: return launch_sym_fwd6<D, DIV>(a, sc, M, o, ws, wsb, st, zs);
    default: return launch_sym_fwd4<D, DIV>(a, sc, M, o, ws, wsb, st, zs);
  }
}

// rows [row0, row0 + nrows) of the pass against all M columns (row-split over ranks);
// nrows < 0: all rows.  Output pointers in `o` address the row slice.
// order: optional nrows int32 row indices (a permutation of the slice's rows) that groups
// spatially close rows into the same workgroup -- used by the matrix-core forward, whose
// fp32 error grows with the spread of a workgroup's rows (mfma_fwd.hpp); ignored otherwise.
template <int D>
int ode_self_fwd_d(const float* q, const float* p, int64_t M, double sigma, double eta,
                   const Outs& o, void* ws, size_t wsb, hipStream_t st, int64_t row0 = 0,
                   int64_t nrows = -1, const int* order = nullptr, float* zs = nullptr) {
  if (nrows < 0) nrows = M;
  const bool all = row0 == 0 && nrows == M;
  Args a = {q + row0 * D, p + row0 * D, nullptr, nullptr, q, p, nullptr, nullptr, 0.f};
  Scal sc = make_scal(sigma, eta);
  scale_coords(a, sc, sigma);
  const bool raw = tl_coord_raw != 0;   // the packed kernels below; the others stay scaled
  if (zs != nullptr) {
    // divergence rows out through the (unused) h slot: the packed passes only
    if (eta != 0.0 || o.ptr[3] != nullptr || (o.ptr[1] != nullptr && !packed_fwd_alg())) {
      set_error("ode_self_fwd: divergence rows (zs) need eta = 0, no h output and fwd_alg 2, 5 or 6");
      return DICP_ERR_INVALID;
    }
    Outs oz = o;
    oz.ptr[3] = zs;
    oz.base[3] = oz.add[3] = nullptr;
    oz.accumulate[3] = 0;
    oz.alpha[3] = 1.f;
    // (the mG-less last step keeps the ordered pass without the Gs' sums: 2.49 against 3.27 ms
    // for the symmetric pass, which forms them anyway, at 100k)
    if (o.ptr[1] != nullptr && use_sym_fwd4(M, all, raw))
      return launch_sym_fwd_rows<D, true>(a, sc, M, oz, ws, wsb, st, true);
    if (o.ptr[1] == nullptr)
      return launch_fwd_pk<OpOdeSelfFwdPk<D, true, false, false, true>, OpOdeSelfFwdPk<D, true, false, false, true, true>>(raw, "ode_self_fwd(pk, no mG, zs)", a, sc, nrows,
                                                                           M, oz, ws, wsb, st);
    return launch_fwd_pk<OpOdeSelfFwdPk<D, true, false, true, true>, OpOdeSelfFwdPk<D, true, false, true, true, true>>(raw, "ode_self_fwd(pk, zs)", a, sc, nrows, M, oz,
                                                                        ws, wsb, st);
  }
  if (eta != 0.0) {
    if (g_fwd_alg >= 2 && o.ptr[1] == nullptr)  // mG not wanted: without the Gs', Hs, GL' sums
      return launch_fwd_pk<OpOdeSelfFwdPk<D, true, true, false>, OpOdeSelfFwdPk<D, true, true, false, false, true>>(raw, "ode_self_fwd_eta(pk, no mG)", a, sc, nrows, M, o,
                                                                     ws, wsb, st);
    return g_fwd_alg >= 2
               ? launch_fwd_pk<OpOdeSelfFwdPk<D, true, true>, OpOdeSelfFwdPk<D, true, true, true, false, true>>(raw, "ode_self_fwd_eta(pk)", a, sc, nrows, M, o, ws, wsb, st)
               : launch_r<OpOdeSelfFwd<D, true, true>>(r_fwd(), "ode_self_fwd", a, sc, nrows, M, o, ws, wsb, st);
  }
  if (o.ptr[1] == nullptr)  // mG not wanted (eta = 0): the packed forward without the Gs' sums
    return o.ptr[2] != nullptr
               ? launch_fwd_pk<OpOdeSelfFwdPk<D, true, false, false>, OpOdeSelfFwdPk<D, true, false, false, false, true>>(raw, "ode_self_fwd(pk, no mG)", a, sc, nrows, M, o, ws, wsb, st)
               : launch_fwd_pk<OpOdeSelfFwdPk<D, false, false, false>, OpOdeSelfFwdPk<D, false, false, false, false, true>>(raw, "ode_self_fwd(pk, no mG)", a, sc, nrows, M, o, ws, wsb, st);
  if ((g_fwd_alg == 1 || g_fwd_alg == 4) && all)
    return o.ptr[2] != nullptr ? launch_sym_fwd<D, true>(a, sc, M, o, ws, wsb, st, g_fwd_alg == 4)
                               : launch_sym_fwd<D, false>(a, sc, M, o, ws, wsb, st, g_fwd_alg == 4);
  if (g_fwd_alg == 3)
    return o.ptr[2] != nullptr
               ? launch_mfma_fwd<D, true>("ode_self_fwd(mfma)", a, sc, nrows, M, o, ws, wsb, st, order)
               : launch_mfma_fwd<D, false>("ode_self_fwd(mfma)", a, sc, nrows, M, o, ws, wsb, st, order);
  if (use_sym_fwd4(M, all, raw)) {  // symmetric pair-once, 4 (or 8) rows per lane
    return o.ptr[2] != nullptr ? launch_sym_fwd_rows<D, true>(a, sc, M, o, ws, wsb, st, false)
                               : launch_sym_fwd_rows<D, false>(a, sc, M, o, ws, wsb, st, false);
  }
  if (g_fwd_alg == 2 || g_fwd_alg == 4 || g_fwd_alg == 5 || g_fwd_alg == 6)
    return o.ptr[2] != nullptr
               ? launch_fwd_pk<OpOdeSelfFwdPk<D, true>, OpOdeSelfFwdPk<D, true, false, true, false, true>>(raw, "ode_self_fwd(pk)", a, sc, nrows, M, o, ws, wsb, st)
               : launch_fwd_pk<OpOdeSelfFwdPk<D, false>, OpOdeSelfFwdPk<D, false, false, true, false, true>>(raw, "ode_self_fwd(pk)", a, sc, nrows, M, o, ws, wsb, st);
  if (o.ptr[2] != nullptr)
    return launch_r<OpOdeSelfFwd<D, false, true>>(r_fwd(), "ode_self_fwd", a, sc, nrows, M, o, ws, wsb, st);
  return launch_r<OpOdeSelfFwd<D, false, false>>(r_fwd(), "ode_self_fwd", a, sc, nrows, M, o, ws, wsb, st);
}

template <int D>
size_t ode_self_fwd_rows_ws(int64_t nrows, int64_t M) {
  size_t m = 0;
  for (size_t v : {ws_r<OpOdeSelfFwd<D, true, true>>(r_fwd(), nrows, M),
                   ws_r<OpOdeSelfFwd<D, false, true>>(r_fwd(), nrows, M),
                   ws_r<OpOdeSelfFwd<D, false, false>>(r_fwd(), nrows, M),
                   fwd_pk_ws<OpOdeSelfFwdPk<D, true>, OpOdeSelfFwdPk<D, true, false, true, false, true>>(nrows, M),
                   fwd_pk_ws<OpOdeSelfFwdPk<D, false>, OpOdeSelfFwdPk<D, false, false, true, false, true>>(nrows, M),
                   fwd_pk_ws<OpOdeSelfFwdPk<D, true, true>, OpOdeSelfFwdPk<D, true, true, true, false, true>>(nrows, M),
                   fwd_pk_ws<OpOdeSelfFwdPk<D, true, false, false>, OpOdeSelfFwdPk<D, true, false, false, false, true>>(nrows, M),
                   fwd_pk_ws<OpOdeSelfFwdPk<D, true, true, false>, OpOdeSelfFwdPk<D, true, true, false, false, true>>(nrows, M),
                   fwd_pk_ws<OpOdeSelfFwdPk<D, false, false, false>, OpOdeSelfFwdPk<D, false, false, false, false, true>>(nrows, M),
                   fwd_pk_ws<OpOdeSelfFwdPk<D, true, false, true, true>, OpOdeSelfFwdPk<D, true, false, true, true, true>>(nrows, M),
                   fwd_pk_ws<OpOdeSelfFwdPk<D, true, false, false, true>, OpOdeSelfFwdPk<D, true, false, false, true, true>>(nrows, M),
                   mfma_fwd_ws_bytes<D, true>(nrows, M), mfma_fwd_ws_bytes<D, false>(nrows, M)})
    m = v > m ? v : m;
  if (nrows == M) {   // a whole pass may run the symmetric 4-row forward (fwd_alg 5)
    const size_t sy = sym_ws_bytes(M, 3 * D);
    m = sy > m ? sy : m;
  }
  return m;
}

template <int D>
size_t ode_self_fwd_ws(int64_t M) {
  // every variant that ode_self_fwd_d may launch (their occupancies, hence splits, differ)
  size_t a = ws_r<OpOdeSelfFwd<D, true, true>>(r_fwd(), M, M);
  size_t b = ws_r<OpOdeSelfFwd<D, false, true>>(r_fwd(), M, M);
  size_t c = ws_r<OpOdeSelfFwd<D, false, false>>(r_fwd(), M, M);
  a = a > b ? a : b;
  a = a > c ? a : c;
  const size_t d = sym_ws_bytes(M, 3 * D);
  a = a > d ? a : d;
  for (size_t e : {fwd_pk_ws<OpOdeSelfFwdPk<D, true>, OpOdeSelfFwdPk<D, true, false, true, false, true>>(M, M),
                   fwd_pk_ws<OpOdeSelfFwdPk<D, false>, OpOdeSelfFwdPk<D, false, false, true, false, true>>(M, M),
                   fwd_pk_ws<OpOdeSelfFwdPk<D, true, true>, OpOdeSelfFwdPk<D, true, true, true, false, true>>(M, M),
                   fwd_pk_ws<OpOdeSelfFwdPk<D, true, false, false>, OpOdeSelfFwdPk<D, true, false, false, false, true>>(M, M),
                   fwd_pk_ws<OpOdeSelfFwdPk<D, true, true, false>, OpOdeSelfFwdPk<D, true, true, false, false, true>>(M, M),
                   fwd_pk_ws<OpOdeSelfFwdPk<D, false, false, false>, OpOdeSelfFwdPk<D, false, false, false, false, true>>(M, M),
                   fwd_pk_ws<OpOdeSelfFwdPk<D, true, false, true, true>, OpOdeSelfFwdPk<D, true, false, true, true, true>>(M, M),
                   fwd_pk_ws<OpOdeSelfFwdPk<D, true, false, false, true>, OpOdeSelfFwdPk<D, true, false, false, true, true>>(M, M),
                   mfma_fwd_ws_bytes<D, true>(M, M), mfma_fwd_ws_bytes<D, false>(M, M)})
    a = a > e ? a : e;
  return a;
}

template <int D>
int ode_self_bwd_d(const float* q, const float* p, const float* gv, const float* gmG,
                   const float* gdiv, int64_t M, double sigma, double eta, const Outs& o,
                   void* ws, size_t wsb, hipStream_t st, const float* zs = nullptr, int64_t zr0 = 0,
                   int64_t zn = 0) {
  if (zs != nullptr && (eta != 0.0 || (gmG != nullptr && g_bwd_alg != 3))) {
    set_error("ode_self_bwd: divergence rows (zs) need eta = 0 and the packed VJP (bwd_alg 3)");
    return DICP_ERR_INVALID;
  }
  // gmG == NULL: zero cotangent on mG (the B0 symmetric packed kernels never read it; the
  // record slot is pointed at gv so every address stays valid)
  const bool b0 = gmG == nullptr;
  if (b0 && eta != 0.0 && g_bwd_eta_alg != 2) {
    set_error("ode_self_bwd: a NULL mG cotangent (zero) needs the packed eta kernel (bwd_eta_alg 2)");
    return DICP_ERR_INVALID;
  }
  const float* gb = b0 ? gv : gmG;
  Args a = {q, p, gv, gb, q, p, gv, gb, 0.f};
  if (eta != 0.0) {
    Scal sc = make_scal(sigma, eta);
    sc.dev0 = gdiv;
    if (g_bwd_eta_alg >= 1)
      return launch_sym_bwd_eta<D>(a, sc, M, o, ws, wsb, st, g_bwd_eta_alg == 2, 0, 1, b0);
    return launch_r<OpOdeSelfBwdEta<D>>(r_bwd(), "ode_self_bwd_eta", a, sc, M, M, o, ws, wsb, st);
  }
  Scal sc = make_scal(sigma, 0.0);
  scale_coords(a, sc, sigma);
  sc.dev0 = gdiv;  // nullptr -> aux0 = 0
  const bool raw = tl_coord_raw != 0 && (b0 || g_bwd_alg == 3);   // packed kernels only
  if (raw) raw_coords(a, sc);
  if (b0) return launch_sym_bwd<D>(a, sc, M, o, ws, wsb, st, 0, 1, true, true, zs, zr0, zn, raw);
  if (g_bwd_alg >= 2)
    return launch_sym_bwd<D>(a, sc, M, o, ws, wsb, st, 0, 1, g_bwd_alg == 3, false, zs, zr0, zn, raw);
  if (g_bwd_alg == 1)
    return launch_r<OpOdeSelfBwd2<D>>(r_bwd(), "ode_self_bwd", a, sc, M, M, o, ws, wsb, st);
  return launch_r<OpOdeSelfBwd<D>>(r_bwd(), "ode_self_bwd", a, sc, M, M, o, ws, wsb, st);
}

// Pair subset `part` of `nparts` of the VJP (row-split over ranks; the sum over parts is
// the full VJP): symmetric kernels (eta = 0, and eta != 0 packed) -> the quads Q = part (mod nparts), written to all
// rows; otherwise (ordered kernels) the row slice [part * ceil(M/nparts), ...) against all
// columns, other rows zero.  Outputs plain (no epilogue).
template <int D>
int ode_self_bwd_part_d(const float* q, const float* p, const float* gv, const float* gmG,
                        const float* gdiv, int64_t M, double sigma, double eta, int part,
                        int nparts, float* gq, float* gp, void* ws, size_t wsb, hipStream_t st,
                        const float* zs = nullptr, int64_t zr0 = 0, int64_t zn = 0) {
  if (nparts == 1)  // the whole VJP: exactly the single-device kernel
    return ode_self_bwd_d<D>(q, p, gv, gmG, gdiv, M, sigma, eta, make_outs(gq, gp), ws, wsb, st, zs, zr0, zn);
  const bool b0 = gmG == nullptr;  // zero mG cotangent: symmetric packed kernels only
  if (zs != nullptr && (eta != 0.0 || !(b0 || g_bwd_alg == 3))) {
    set_error("ode_self_bwd_part: divergence rows (zs) need eta = 0 and the packed VJP (bwd_alg 3)");
    return DICP_ERR_INVALID;
  }
  if (eta == 0.0 && (g_bwd_alg >= 2 || b0)) {
    const float* gb = b0 ? gv : gmG;
    Args a = {q, p, gv, gb, q, p, gv, gb, 0.f};
    Scal sc = make_scal(sigma, 0.0);
    scale_coords(a, sc, sigma);
    sc.dev0 = gdiv;
    const bool pk = b0 || g_bwd_alg == 3;
    const bool raw = tl_coord_raw != 0 && pk;
    if (raw) raw_coords(a, sc);
    return launch_sym_bwd<D>(a, sc, M, make_outs(gq, gp), ws, wsb, st, part, nparts, pk, b0, zs, zr0,
                             zn, raw);
  }
  if (eta != 0.0 && g_bwd_eta_alg == 2) {  // symmetric packed eta VJP: quads Q = part (mod nparts)
    const float* gb = b0 ? gv : gmG;
    Args a = {q, p, gv, gb, q, p, gv, gb, 0.f};
    Scal sc = make_scal(sigma, eta);
    sc.dev0 = gdiv;
    return launch_sym_bwd_eta<D>(a, sc, M, make_outs(gq, gp), ws, wsb, st, true, part, nparts, b0);
  }
  if (b0) {
    set_error("ode_self_bwd_part: a NULL mG cotangent (zero) needs a symmetric packed kernel");
    return DICP_ERR_INVALID;
  }
  if (int rc = no_batch("ode_self_bwd_part(ordered)")) return rc;
  const int64_t per = (M + nparts - 1) / nparts;
  const int64_t r0 = per * part < M ? per * part : M;
  const int64_t r1 = r0 + per < M ? r0 + per : M;
  if ((gq && hipMemsetAsync(gq, 0, (size_t)M * D * sizeof(float), st) != hipSuccess) ||
      hipMemsetAsync(gp, 0, (size_t)M * D * sizeof(float), st) != hipSuccess) {
    set_error("ode_self_bwd_part: hipMemsetAsync failed");
    return DICP_ERR_HIP;
  }
  if (r1 <= r0) return DICP_OK;
  const int64_t o0 = r0 * D;
  Args a = {q + o0, p + o0, gv + o0, gmG + o0, q, p, gv, gmG, 0.f};
  const Outs o = make_outs(gq ? gq + o0 : nullptr, gp + o0);
  if (eta != 0.0) {
    Scal sc = make_scal(sigma, eta);
    sc.dev0 = gdiv;
    return launch_r<OpOdeSelfBwdEta<D>>(r_bwd(), "ode_self_bwd_eta", a, sc, r1 - r0, M, o, ws, wsb, st);
  }
  Scal sc = make_scal(sigma, 0.0);
  scale_coords(a, sc, sigma);
  sc.dev0 = gdiv;
  if (g_bwd_alg == 1)
    return launch_r<OpOdeSelfBwd2<D>>(r_bwd(), "ode_self_bwd", a, sc, r1 - r0, M, o, ws, wsb, st);
  return launch_r<OpOdeSelfBwd<D>>(r_bwd(), "ode_self_bwd", a, sc, r1 - r0, M, o, ws, wsb, st);
}

template <int D>
size_t ode_self_bwd_part_ws(int64_t M, int nparts) {
  const int64_t per = (M + nparts - 1) / nparts;
  size_t m = sym_ws_bytes(M, 2 * D, nparts);
  for (size_t v : {ws_r<OpOdeSelfBwd<D>>(r_bwd(), per, M), ws_r<OpOdeSelfBwdEta<D>>(r_bwd(), per, M),
                   ws_r<OpOdeSelfBwd2<D>>(r_bwd(), per, M)})
    m = v > m ? v : m;
  return m;
}

template <int D>
int ode_ext_fwd_d(const float* x, int64_t N, const float* q, const float* p, int64_t M,
                  double sigma, double eta, float* vx, float* gx, void* ws, size_t wsb,
                  hipStream_t st) {
  if (cx_eligible(N, M, true)) return cx_ext_fwd(x, N, q, p, M, D, sigma, eta, vx, gx, ws, wsb, st);
  const Outs o = make_outs(vx, gx);
  if (g_ext_alg == 1) {
    const Args a = {x, nullptr, nullptr, nullptr, q, p, nullptr, nullptr};
    const Scal sc = make_scal(sigma, eta);
    if (eta != 0.0)
      return gx ? launch_rowred_pk<OpExtFwdPk<D, true, true>>("ode_ext_fwd", a, sc, N, M, o, ws, wsb, st)
                : launch_rowred_pk<OpExtFwdPk<D, true, false>>("ode_ext_fwd", a, sc, N, M, o, ws, wsb, st);
    return gx ? launch_rowred_pk<OpExtFwdPk<D, false, true>>("ode_ext_fwd", a, sc, N, M, o, ws, wsb, st)
              : launch_rowred_pk<OpExtFwdPk<D, false, false>>("ode_ext_fwd", a, sc, N, M, o, ws, wsb, st);
  }
  const Args a = {x, nullptr, nullptr, nullptr, q, p, nullptr, nullptr};
  const Scal sc = make_scal(sigma, eta);
  if (eta != 0.0) {
    if (gx) return launch_rowred<OpOdeExtFwd<D, true, true>, kR>("ode_ext_fwd", a, sc, N, M, o, ws, wsb, st);
    return launch_rowred<OpOdeExtFwd<D, true, false>, kR>("ode_ext_fwd", a, sc, N, M, o, ws, wsb, st);
  }
  if (gx) return launch_rowred<OpOdeExtFwd<D, false, true>, kR>("ode_ext_fwd", a, sc, N, M, o, ws, wsb, st);
  return launch_rowred<OpOdeExtFwd<D, false, false>, kR>("ode_ext_fwd", a, sc, N, M, o, ws, wsb, st);
}

template <int D>
size_t ode_ext_fwd_ws(int64_t N, int64_t M) {
  size_t m = 0;
  for (size_t v : {rowred_ws_bytes<OpOdeExtFwd<D, true, true>, kR>(N, M),
                   rowred_ws_bytes<OpOdeExtFwd<D, true, false>, kR>(N, M),
                   rowred_ws_bytes<OpOdeExtFwd<D, false, true>, kR>(N, M),
                   rowred_ws_bytes<OpOdeExtFwd<D, false, false>, kR>(N, M),
                   rowred_pk_ws_bytes<OpExtFwdPk<D, true, true>>(N, M),
                   rowred_pk_ws_bytes<OpExtFwdPk<D, true, false>>(N, M),
                   rowred_pk_ws_bytes<OpExtFwdPk<D, false, true>>(N, M),
                   rowred_pk_ws_bytes<OpExtFwdPk<D, false, false>>(N, M)})
    m = v > m ? v : m;
  if (cx_eligible(N, M, true)) {
    const size_t c = cx_ext_ws(N, M, D);
    m = c > m ? c : m;
  }
  return m;
}

template <int D>
int ode_ext_bwd_d(const float* x, int64_t N, const float* q, const float* p, int64_t M,
                  double sigma, double eta, const float* gvx, const float* gdiv, float* gxo,
                  float* gq, float* gp, void* ws, size_t wsb, hipStream_t st) {
  if (g_ext_alg == 1 && eta == 0.0) {
    const Args a = {x, gvx, nullptr, nullptr, q, p, nullptr, nullptr};
    Scal sc = make_scal(sigma, 0.0);
    sc.dev0 = gdiv;
    int rc = launch_rowred_pk<OpExtBwdXPk<D>>("ode_ext_bwd_x", a, sc, N, M, make_outs(gxo), ws, wsb, st);
    if (rc) return rc;
    const Args b = {q, p, nullptr, nullptr, x, gvx, nullptr, nullptr};
    Outs o = make_outs(gq, gp);
    o.accumulate[0] = o.accumulate[1] = 1;
    return launch_rowred_pk<OpExtBwdQPk<D>>("ode_ext_bwd_q", b, sc, M, N, o, ws, wsb, st);
  }
  Scal sc = make_scal(sigma, eta);
  sc.dev0 = gdiv;
  // rows x: gradient w.r.t. the carried points
  {
    const Args a = {x, gvx, nullptr, nullptr, q, p, nullptr, nullptr};
    const Outs o = make_outs(gxo);
    int rc = eta != 0.0
        ? launch_rowred<OpOdeExtBwdXEta<D>, kR>("ode_ext_bwd_x", a, sc, N, M, o, ws, wsb, st)
        : launch_rowred<OpOdeExtBwdX<D>, kR>("ode_ext_bwd_x", a, sc, N, M, o, ws, wsb, st);
    if (rc) return rc;
  }
  // rows q: gradient w.r.t. support points and momenta (accumulated)
  {
    const Args a = {q, p, nullptr, nullptr, x, gvx, nullptr, nullptr};
    Outs o = make_outs(gq, gp);
    o.accumulate[0] = o.accumulate[1] = 1;
    return eta != 0.0
        ? launch_rowred<OpOdeExtBwdQEta<D>, kR>("ode_ext_bwd_q", a, sc, M, N, o, ws, wsb, st)
        : launch_rowred<OpOdeExtBwdQ<D>, kR>("ode_ext_bwd_q", a, sc, M, N, o, ws, wsb, st);
  }
}

template <int D>
size_t ode_ext_bwd_ws(int64_t N, int64_t M) {
  size_t m = 0;
  for (size_t v : {rowred_ws_bytes<OpOdeExtBwdX<D>, kR>(N, M), rowred_ws_bytes<OpOdeExtBwdQ<D>, kR>(M, N),
                   rowred_ws_bytes<OpOdeExtBwdXEta<D>, kR>(N, M),
                   rowred_ws_bytes<OpOdeExtBwdQEta<D>, kR>(M, N),
                   rowred_pk_ws_bytes<OpExtBwdXPk<D>>(N, M), rowred_pk_ws_bytes<OpExtBwdQPk<D>>(M, N)})
    m = v > m ? v : m;
  return m;
}

}  // namespace

extern "C" int dicp_lddmm_ode_self_fwd_f32(const float* q, const float* p, int64_t M, int D,
                                           double sigma, double eta, float* v, float* mG,
                                           float* g, float* h, void* ws, size_t ws_bytes,
                                           dicp_stream_t stream) {
  dicp::BatchCall batch_call_;  // a call of a launch batch (batch.hpp)
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (M < 0 || (M > 0 && (!q || !p || !v || !mG)) || !(sigma > 0)) {
    set_error("dicp_lddmm_ode_self_fwd_f32: invalid arguments");
    return DICP_ERR_INVALID;
  }
  switch (D) {
    case 2: return ode_self_fwd_d<2>(q, p, M, sigma, eta, make_outs(v, mG, g, h), ws, ws_bytes, st);
    case 3: return ode_self_fwd_d<3>(q, p, M, sigma, eta, make_outs(v, mG, g, h), ws, ws_bytes, st);
    default: set_error("ode_self_fwd: D=%d unsupported", D); return DICP_ERR_UNSUPPORTED;
  }
}

extern "C" int dicp_lddmm_ode_self_bwd_f32(const float* q, const float* p, const float* gv,
                                           const float* gmG, const float* gdiv, int64_t M,
                                           int D, double sigma, double eta, float* gq,
                                           float* gp, void* ws, size_t ws_bytes,
                                           dicp_stream_t stream) {
  dicp::BatchCall batch_call_;  // a call of a launch batch (batch.hpp)
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (M < 0 || (M > 0 && (!q || !p || !gv || !gp)) || !(sigma > 0)) {  // gmG NULL = zero (eta = 0)
    set_error("dicp_lddmm_ode_self_bwd_f32: invalid arguments");
    return DICP_ERR_INVALID;
  }
  switch (D) {
    case 2: return ode_self_bwd_d<2>(q, p, gv, gmG, gdiv, M, sigma, eta, make_outs(gq, gp), ws, ws_bytes, st);
    case 3: return ode_self_bwd_d<3>(q, p, gv, gmG, gdiv, M, sigma, eta, make_outs(gq, gp), ws, ws_bytes, st);
    default: set_error("ode_self_bwd: D=%d unsupported", D); return DICP_ERR_UNSUPPORTED;
  }
}

// One explicit-Euler step of the shooting ODE with the state update fused into the
// reduction's epilogue: q_next = q + dt v(q,p), p_next = p + dt mG(q,p), g rows as in
// dicp_lddmm_ode_self_fwd_f32 (integrators.py:20-33 EulerIntegrator over LDDMM.py:176-227).
extern "C" int dicp_lddmm_euler_step_f32(const float* q, const float* p, int64_t M, int D,
                                         double sigma, double eta, double dt, float* q_next,
                                         float* p_next, float* g, void* ws, size_t ws_bytes,
                                         dicp_stream_t stream) {
  dicp::BatchCall batch_call_;  // a call of a launch batch (batch.hpp)
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (M < 0 || (M > 0 && (!q || !p || !q_next || !p_next)) || !(sigma > 0) ||
      (M > 0 && (q_next == q || q_next == p || p_next == q || p_next == p))) {
    set_error("dicp_lddmm_euler_step_f32: invalid arguments (outputs must not alias inputs)");
    return DICP_ERR_INVALID;
  }
  Outs o = make_outs(q_next, p_next, g, nullptr);
  o.base[0] = q;
  o.base[1] = p;
  o.alpha[0] = o.alpha[1] = (float)dt;
  switch (D) {
    case 2: return ode_self_fwd_d<2>(q, p, M, sigma, eta, o, ws, ws_bytes, st);
    case 3: return ode_self_fwd_d<3>(q, p, M, sigma, eta, o, ws, ws_bytes, st);
    default: set_error("euler_step: D=%d unsupported", D); return DICP_ERR_UNSUPPORTED;
  }
}

// The matching adjoint step (exact discrete adjoint of the Euler step):
//   lq_next = lq + dt * d/dq[lq.v + lp.mG + gdiv sum g] + addq,
//   lp_next = lp + dt * d/dp[...]                        + addp
// (addq / addp: the loss's own cotangent on the state at this time, or NULL).
extern "C" int dicp_lddmm_euler_adjoint_step_zs_f32(const float* q, const float* p, const float* lq,
                                                    const float* lp, const float* gdiv, int64_t M,
                                                    int D, double sigma, double eta, double dt,
                                                    const float* addq, const float* addp,
                                                    const float* zs, float* lq_next, float* lp_next,
                                                    void* ws, size_t ws_bytes, dicp_stream_t stream) {
  dicp::BatchCall batch_call_;  // a call of a launch batch (batch.hpp)
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const float* ins[5] = {q, p, lq, lp, zs};
  bool alias = false;
  for (const float* x : ins) alias = alias || (x && ((lq_next && x == lq_next) || x == lp_next));
  // lq_next may be NULL: only lp_next is produced (the gq half of the eta = 0 symmetric VJP is
  // then never evaluated -- the last adjoint step when the start points need no gradient).
  // lp may be NULL: a zero cotangent on the momenta (the first adjoint step when the loss does
  // not depend on the final momenta; eta = 0), the b terms of the VJP are then skipped.
  // zs may be NULL (no divergence rows).
  if (M < 0 || (M > 0 && (!q || !p || !lq || !lp_next || alias)) || !(sigma > 0)) {
    set_error("dicp_lddmm_euler_adjoint_step_f32: invalid arguments (outputs must not alias inputs)");
    return DICP_ERR_INVALID;
  }
  Outs o = make_outs(lq_next, lp_next);
  o.base[0] = lq;
  o.base[1] = lp;
  o.add[0] = addq;
  o.add[1] = addp;
  o.alpha[0] = o.alpha[1] = (float)dt;
  switch (D) {
    case 2: return ode_self_bwd_d<2>(q, p, lq, lp, gdiv, M, sigma, eta, o, ws, ws_bytes, st, zs, 0, M);
    case 3: return ode_self_bwd_d<3>(q, p, lq, lp, gdiv, M, sigma, eta, o, ws, ws_bytes, st, zs, 0, M);
    default: set_error("euler_adjoint_step: D=%d unsupported", D); return DICP_ERR_UNSUPPORTED;
  }
}

extern "C" int dicp_lddmm_euler_adjoint_step_f32(const float* q, const float* p, const float* lq,
                                                 const float* lp, const float* gdiv, int64_t M,
                                                 int D, double sigma, double eta, double dt,
                                                 const float* addq, const float* addp,
                                                 float* lq_next, float* lp_next, void* ws,
                                                 size_t ws_bytes, dicp_stream_t stream) {
  dicp::BatchCall batch_call_;  // a call of a launch batch (batch.hpp)
  return dicp_lddmm_euler_adjoint_step_zs_f32(q, p, lq, lp, gdiv, M, D, sigma, eta, dt, addq, addp, nullptr,
                                              lq_next, lp_next, ws, ws_bytes, stream);
}

extern "C" int dicp_lddmm_ode_ext_fwd_f32(const float* x, int64_t N, const float* q,
                                          const float* p, int64_t M, int D, double sigma,
                                          double eta, float* vx, float* gx, void* ws,
                                          size_t ws_bytes, dicp_stream_t stream) {
  dicp::BatchCall batch_call_;  // a call of a launch batch (batch.hpp)
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (N < 0 || M < 0 || (N > 0 && (!x || !vx)) || (M > 0 && (!q || !p)) || !(sigma > 0)) {
    set_error("dicp_lddmm_ode_ext_fwd_f32: invalid arguments");
    return DICP_ERR_INVALID;
  }
  switch (D) {
    case 2: return ode_ext_fwd_d<2>(x, N, q, p, M, sigma, eta, vx, gx, ws, ws_bytes, st);
    case 3: return ode_ext_fwd_d<3>(x, N, q, p, M, sigma, eta, vx, gx, ws, ws_bytes, st);
    default: set_error("ode_ext_fwd: D=%d unsupported", D); return DICP_ERR_UNSUPPORTED;
  }
}

extern "C" int dicp_lddmm_ode_ext_bwd_f32(const float* x, int64_t N, const float* q,
                                          const float* p, int64_t M, int D, double sigma,
                                          double eta, const float* gvx, const float* gdiv,
                                          float* gxo, float* gq, float* gp, void* ws,
                                          size_t ws_bytes, dicp_stream_t stream) {
  dicp::BatchCall batch_call_;  // a call of a launch batch (batch.hpp)
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (N < 0 || M < 0 || (N > 0 && (!x || !gvx || !gxo)) || (M > 0 && (!q || !p || !gq || !gp)) ||
      !(sigma > 0)) {
    set_error("dicp_lddmm_ode_ext_bwd_f32: invalid arguments");
    return DICP_ERR_INVALID;
  }
  switch (D) {
    case 2: return ode_ext_bwd_d<2>(x, N, q, p, M, sigma, eta, gvx, gdiv, gxo, gq, gp, ws, ws_bytes, st);
    case 3: return ode_ext_bwd_d<3>(x, N, q, p, M, sigma, eta, gvx, gdiv, gxo, gq, gp, ws, ws_bytes, st);
    default: set_error("ode_ext_bwd: D=%d unsupported", D); return DICP_ERR_UNSUPPORTED;
  }
}

// Row-split (multi-GPU single frame): rows [row0, row0 + nrows) of the fused
// forward against all M columns; outputs address the slice (nrows rows).
extern "C" int dicp_lddmm_ode_self_fwd_rows_f32(const float* q, const float* p, int64_t M,
                                                int64_t row0, int64_t nrows, int D,
                                                double sigma, double eta, float* v, float* mG,
                                                float* g, float* h, void* ws, size_t ws_bytes,
                                                dicp_stream_t stream) {
  dicp::BatchCall batch_call_;  // a call of a launch batch (batch.hpp)
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (M < 0 || row0 < 0 || nrows < 0 || row0 + nrows > M ||
      (nrows > 0 && (!q || !p || !v || !mG)) || !(sigma > 0)) {
    set_error("dicp_lddmm_ode_self_fwd_rows_f32: invalid arguments");
    return DICP_ERR_INVALID;
  }
  if (nrows == 0) return DICP_OK;
  switch (D) {
    case 2: return ode_self_fwd_d<2>(q, p, M, sigma, eta, make_outs(v, mG, g, h), ws, ws_bytes, st, row0, nrows);
    case 3: return ode_self_fwd_d<3>(q, p, M, sigma, eta, make_outs(v, mG, g, h), ws, ws_bytes, st, row0, nrows);
    default: set_error("ode_self_fwd_rows: D=%d unsupported", D); return DICP_ERR_UNSUPPORTED;
  }
}

extern "C" int dicp_lddmm_euler_step_rows_f32(const float* q, const float* p, int64_t M,
                                              int64_t row0, int64_t nrows, int D, double sigma,
                                              double eta, double dt, float* q_next,
                                              float* p_next, float* g, void* ws,
                                              size_t ws_bytes, dicp_stream_t stream) {
  dicp::BatchCall batch_call_;  // a call of a launch batch (batch.hpp)
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (M < 0 || row0 < 0 || nrows < 0 || row0 + nrows > M ||
      (nrows > 0 && (!q || !p || !q_next || !p_next)) || !(sigma > 0)) {
    set_error("dicp_lddmm_euler_step_rows_f32: invalid arguments");
    return DICP_ERR_INVALID;
  }
  if (nrows == 0) return DICP_OK;
  Outs o = make_outs(q_next, p_next, g, nullptr);
  o.base[0] = q + row0 * D;
  o.base[1] = p + row0 * D;
  o.alpha[0] = o.alpha[1] = (float)dt;
  switch (D) {
    case 2: return ode_self_fwd_d<2>(q, p, M, sigma, eta, o, ws, ws_bytes, st, row0, nrows);
    case 3: return ode_self_fwd_d<3>(q, p, M, sigma, eta, o, ws, ws_bytes, st, row0, nrows);
    default: set_error("euler_step_rows: D=%d unsupported", D); return DICP_ERR_UNSUPPORTED;
  }
}

// Ordered forms (rows [row0, row0 + nrows) visited in row_order, or NULL = natural order):
// the general entry points behind the four above.
extern "C" int dicp_lddmm_ode_self_fwd_zs_f32(const float* q, const float* p, int64_t M, int64_t row0,
                                              int64_t nrows, int D, double sigma, double eta,
                                              const int32_t* row_order, float* v, float* mG, float* g,
                                              float* zs, void* ws, size_t ws_bytes, dicp_stream_t stream) {
  dicp::BatchCall batch_call_;  // a call of a launch batch (batch.hpp)
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (M < 0 || row0 < 0 || nrows < 0 || row0 + nrows > M ||
      (nrows > 0 && (!q || !p || !v || !mG || !zs)) || !(sigma > 0)) {
    set_error("dicp_lddmm_ode_self_fwd_zs_f32: invalid arguments");
    return DICP_ERR_INVALID;
  }
  if (nrows == 0) return DICP_OK;
  switch (D) {
    case 2: return ode_self_fwd_d<2>(q, p, M, sigma, eta, make_outs(v, mG, g, nullptr), ws, ws_bytes, st, row0, nrows, row_order, zs);
    case 3: return ode_self_fwd_d<3>(q, p, M, sigma, eta, make_outs(v, mG, g, nullptr), ws, ws_bytes, st, row0, nrows, row_order, zs);
    default: set_error("ode_self_fwd_zs: D=%d unsupported", D); return DICP_ERR_UNSUPPORTED;
  }
}

extern "C" int dicp_lddmm_ode_self_fwd_ord_f32(const float* q, const float* p, int64_t M,
                                               int64_t row0, int64_t nrows, int D, double sigma,
                                               double eta, const int32_t* row_order, float* v,
                                               float* mG, float* g, float* h, void* ws,
                                               size_t ws_bytes, dicp_stream_t stream) {
  dicp::BatchCall batch_call_;  // a call of a launch batch (batch.hpp)
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (M < 0 || row0 < 0 || nrows < 0 || row0 + nrows > M ||
      (nrows > 0 && (!q || !p || !v || !mG)) || !(sigma > 0)) {
    set_error("dicp_lddmm_ode_self_fwd_ord_f32: invalid arguments");
    return DICP_ERR_INVALID;
  }
  if (nrows == 0) return DICP_OK;
  switch (D) {
    case 2: return ode_self_fwd_d<2>(q, p, M, sigma, eta, make_outs(v, mG, g, h), ws, ws_bytes, st, row0, nrows, row_order);
    case 3: return ode_self_fwd_d<3>(q, p, M, sigma, eta, make_outs(v, mG, g, h), ws, ws_bytes, st, row0, nrows, row_order);
    default: set_error("ode_self_fwd_ord: D=%d unsupported", D); return DICP_ERR_UNSUPPORTED;
  }
}

extern "C" int dicp_lddmm_euler_step_zs_f32(const float* q, const float* p, int64_t M, int64_t row0,
                                            int64_t nrows, int D, double sigma, double eta, double dt,
                                            const int32_t* row_order, float* q_next, float* p_next,
                                            float* g, float* zs, void* ws, size_t ws_bytes,
                                            dicp_stream_t stream) {
  dicp::BatchCall batch_call_;  // a call of a launch batch (batch.hpp)
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // p_next may be NULL: the momenta update is not wanted (the packed pass skips its Gs' / Hs /
  // GL' sums); zs may be NULL (no divergence rows)
  if (M < 0 || row0 < 0 || nrows < 0 || row0 + nrows > M ||
      (nrows > 0 && (!q || !p || !q_next)) || !(sigma > 0) ||
      (nrows > 0 && (q_next == q || q_next == p || (p_next && (p_next == q || p_next == p)) ||
                     (zs && (zs == q || zs == p || zs == q_next || zs == p_next))))) {
    set_error("dicp_lddmm_euler_step_ord_f32: invalid arguments (outputs must not alias inputs)");
    return DICP_ERR_INVALID;
  }
  if (nrows == 0) return DICP_OK;
  Outs o = make_outs(q_next, p_next, g, nullptr);
  o.base[0] = q + row0 * D;
  o.base[1] = p + row0 * D;
  o.alpha[0] = o.alpha[1] = (float)dt;
  switch (D) {
    case 2: return ode_self_fwd_d<2>(q, p, M, sigma, eta, o, ws, ws_bytes, st, row0, nrows, row_order, zs);
    case 3: return ode_self_fwd_d<3>(q, p, M, sigma, eta, o, ws, ws_bytes, st, row0, nrows, row_order, zs);
    default: set_error("euler_step_ord: D=%d unsupported", D); return DICP_ERR_UNSUPPORTED;
  }
}

extern "C" int dicp_lddmm_euler_step_ord_f32(const float* q, const float* p, int64_t M,
                                             int64_t row0, int64_t nrows, int D, double sigma,
                                             double eta, double dt, const int32_t* row_order,
                                             float* q_next, float* p_next, float* g, void* ws,
                                             size_t ws_bytes, dicp_stream_t stream) {
  dicp::BatchCall batch_call_;  // a call of a launch batch (batch.hpp)
  return dicp_lddmm_euler_step_zs_f32(q, p, M, row0, nrows, D, sigma, eta, dt, row_order, q_next, p_next, g,
                                      nullptr, ws, ws_bytes, stream);
}

// A row-split Euler step in two column phases (core/shooting.py, RowSplit.overlap): phase 0
// runs the rank's rows against its own slice -- the rows' values, which the rank holds before
// the all-gather of the step's input has landed -- into the first partial slots of `ws`;
// phase 1 runs them against the other M - nrows points (the wrapped column range from
// row0 + nrows) into the remaining slots and merges all slots once, with the Euler epilogue.
// The two calls must see the same sizes, output pointers (which select the pass) and `ws`.
// The pair operators' stores are linear in the column sums, so the result is the one-pass
// step's up to fp32 summation order (and the coordinate origin of each phase: its first
// column point).  Ordered packed passes (fwd_alg 2, 5, 6); zs needs eta = 0.
namespace {
template <class Op>
int step_phase_op(const char* name, int phase, const Args& a0, const Args& a1, const Scal& sc, int64_t nrows,
                  int64_t M, int64_t coff, const Outs& o, void* ws, size_t wsb, hipStream_t st) {
  // phase 0 reads its nrows columns in place (no offset); phase 1 from coff, wrapping at M
  return launch_pk_phase<Op>(name, phase, phase == 0 ? a0 : a1, sc, nrows, nrows, M - nrows,
                             phase == 0 ? 0 : coff, phase == 0 ? nrows : M, o, ws, wsb, st);
}

struct PhaseGo {
  int phase;
  const Args &a0, &a1;
  const Scal& sc;
  int64_t nrows, M, coff;
  const Outs& o;
  void* ws;
  size_t wsb;
  hipStream_t st;
  template <class OpS, class OpR>
  int run(bool raw) const {
    return raw ? step_phase_op<OpR>("ode_self_fwd(pk, phase)", phase, a0, a1, sc, nrows, M, coff, o, ws, wsb, st)
               : step_phase_op<OpS>("ode_self_fwd(pk, phase)", phase, a0, a1, sc, nrows, M, coff, o, ws, wsb, st);
  }
};

// the pass (and its raw-coordinate twin) for these outputs: f.run<OpScaled, OpRaw>(raw)
template <int D, class F>
int step_phase_pick(bool raw, bool zs, bool eta, bool mg, bool div, const F& f) {
  if (zs)
    return mg ? f.template run<OpOdeSelfFwdPk<D, true, false, true, true>, OpOdeSelfFwdPk<D, true, false, true, true, true>>(raw)
              : f.template run<OpOdeSelfFwdPk<D, true, false, false, true>, OpOdeSelfFwdPk<D, true, false, false, true, true>>(raw);
  if (eta)
    return mg ? f.template run<OpOdeSelfFwdPk<D, true, true>, OpOdeSelfFwdPk<D, true, true, true, false, true>>(raw)
              : f.template run<OpOdeSelfFwdPk<D, true, true, false>, OpOdeSelfFwdPk<D, true, true, false, false, true>>(raw);
  if (!mg)
    return div ? f.template run<OpOdeSelfFwdPk<D, true, false, false>, OpOdeSelfFwdPk<D, true, false, false, false, true>>(raw)
               : f.template run<OpOdeSelfFwdPk<D, false, false, false>, OpOdeSelfFwdPk<D, false, false, false, false, true>>(raw);
  return div ? f.template run<OpOdeSelfFwdPk<D, true>, OpOdeSelfFwdPk<D, true, false, true, false, true>>(raw)
             : f.template run<OpOdeSelfFwdPk<D, false>, OpOdeSelfFwdPk<D, false, false, true, false, true>>(raw);
}

template <int D>
int euler_step_phase_d(int phase, const float* q_loc, const float* p_loc, const float* q, const float* p, int64_t M,
                       int64_t row0, int64_t nrows, double sigma, double eta, const Outs& o, void* ws, size_t wsb,
                       hipStream_t st) {
  Scal sc0 = make_scal(sigma, eta), sc1 = sc0;
  // phase 0: rows = columns = the local slice; phase 1: rows = the slice of (q, p), columns =
  // all of (q, p) read from row0 + nrows on (wrapping), M - nrows of them
  Args a0 = {q_loc, p_loc, nullptr, nullptr, q_loc, p_loc, nullptr, nullptr, 0.f};
  Args a1 = {q ? q + row0 * D : nullptr, p ? p + row0 * D : nullptr, nullptr, nullptr, q, p, nullptr, nullptr, 0.f};
  const bool raw = tl_coord_raw != 0;
  scale_coords(a0, sc0, sigma);
  scale_coords(a1, sc1, sigma);
  if (raw) {
    raw_coords(a0, sc0);
    raw_coords(a1, sc1);
  }
  const Scal& sc = phase == 0 ? sc0 : sc1;
  const int64_t coff = row0 + nrows < M ? row0 + nrows : 0;
  const PhaseGo go{phase, a0, a1, sc, nrows, M, coff, o, ws, wsb, st};
  return step_phase_pick<D>(raw, o.ptr[3] != nullptr, eta != 0.0, o.ptr[1] != nullptr, o.ptr[2] != nullptr, go);
}

template <int D>
size_t euler_step_phase_ws(int64_t nrows, int64_t M) {
  size_t m = 0;
  for (size_t v : {pk_phase_ws_bytes<OpOdeSelfFwdPk<D, true, false, true, true>>(nrows, nrows, M - nrows),
                   pk_phase_ws_bytes<OpOdeSelfFwdPk<D, true, false, true, true, true>>(nrows, nrows, M - nrows),
                   pk_phase_ws_bytes<OpOdeSelfFwdPk<D, true, false, false, true>>(nrows, nrows, M - nrows),
                   pk_phase_ws_bytes<OpOdeSelfFwdPk<D, true, false, false, true, true>>(nrows, nrows, M - nrows),
                   pk_phase_ws_bytes<OpOdeSelfFwdPk<D, true, true>>(nrows, nrows, M - nrows),
                   pk_phase_ws_bytes<OpOdeSelfFwdPk<D, true, true, true, false, true>>(nrows, nrows, M - nrows),
                   pk_phase_ws_bytes<OpOdeSelfFwdPk<D, true, true, false>>(nrows, nrows, M - nrows),
                   pk_phase_ws_bytes<OpOdeSelfFwdPk<D, true, true, false, false, true>>(nrows, nrows, M - nrows),
                   pk_phase_ws_bytes<OpOdeSelfFwdPk<D, true, false, false>>(nrows, nrows, M - nrows),
                   pk_phase_ws_bytes<OpOdeSelfFwdPk<D, true, false, false, false, true>>(nrows, nrows, M - nrows),
                   pk_phase_ws_bytes<OpOdeSelfFwdPk<D, false, false, false>>(nrows, nrows, M - nrows),
                   pk_phase_ws_bytes<OpOdeSelfFwdPk<D, false, false, false, false, true>>(nrows, nrows, M - nrows),
                   pk_phase_ws_bytes<OpOdeSelfFwdPk<D, true>>(nrows, nrows, M - nrows),
                   pk_phase_ws_bytes<OpOdeSelfFwdPk<D, true, false, true, false, true>>(nrows, nrows, M - nrows),
                   pk_phase_ws_bytes<OpOdeSelfFwdPk<D, false>>(nrows, nrows, M - nrows),
                   pk_phase_ws_bytes<OpOdeSelfFwdPk<D, false, false, true, false, true>>(nrows, nrows, M - nrows)})
    m = v > m ? v : m;
  return m;
}
}  // namespace

extern "C" int dicp_lddmm_euler_step_phase_f32(int phase, const float* q_loc, const float* p_loc, const float* q,
                                               const float* p, int64_t M, int64_t row0, int64_t nrows, int D,
                                               double sigma, double eta, double dt, float* q_next, float* p_next,
                                               float* g, float* zs, void* ws, size_t ws_bytes,
                                               dicp_stream_t stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  auto overlaps = [](const float* out, int64_t n_out, const float* in, int64_t n_in) {
    return out && in && out < in + n_in && in < out + n_out;
  };
  bool bad = (phase != 0 && phase != 1) || M < 0 || row0 < 0 || nrows < 0 || row0 + nrows > M ||
             (nrows > 0 && nrows == M) || !(sigma > 0) || (nrows > 0 && !q_next) || (zs && eta != 0.0) ||
             (nrows > 0 && phase == 0 && (!q_loc || !p_loc)) || (nrows > 0 && phase == 1 && (!q || !p));
  // outputs (phase 1 writes them) must not overlap (q, p); they may be the local slice's
  // buffers, which only phase 0 reads
  const float* outs_[4] = {q_next, p_next, g, zs};
  const int64_t w_[4] = {D, D, 1, D};
  for (int k = 0; k < 4 && !bad && phase == 1; ++k) {
    const int64_t n = nrows * w_[k];
    bad = overlaps(outs_[k], n, q, M * D) || overlaps(outs_[k], n, p, M * D);
  }
  if (bad) {
    set_error("dicp_lddmm_euler_step_phase_f32: invalid arguments (phase 0/1, 0 <= nrows < M, outputs must "
              "not overlap the inputs, zs needs eta = 0)");
    return DICP_ERR_INVALID;
  }
  if (!packed_fwd_alg()) {
    set_error("dicp_lddmm_euler_step_phase_f32: needs an ordered packed forward (fwd_alg 2, 5 or 6)");
    return DICP_ERR_UNSUPPORTED;
  }
  if (nrows == 0) return DICP_OK;
  Outs o = make_outs(q_next, p_next, g, zs);
  o.alpha[0] = o.alpha[1] = (float)dt;
  if (phase == 1) {
    o.base[0] = q + row0 * D;
    o.base[1] = p_next ? p + row0 * D : nullptr;
  }
  switch (D) {
    case 2: return euler_step_phase_d<2>(phase, q_loc, p_loc, q, p, M, row0, nrows, sigma, eta, o, ws, ws_bytes, st);
    case 3: return euler_step_phase_d<3>(phase, q_loc, p_loc, q, p, M, row0, nrows, sigma, eta, o, ws, ws_bytes, st);
    default: set_error("euler_step_phase: D=%d unsupported", D); return DICP_ERR_UNSUPPORTED;
  }
}

extern "C" int dicp_lddmm_ode_self_bwd_part_zs_f32(const float* q, const float* p, const float* gv,
                                                   const float* gmG, const float* gdiv, int64_t M,
                                                   int D, double sigma, double eta, int part,
                                                   int nparts, const float* zs, int64_t zrow0,
                                                   int64_t znrows, float* gq, float* gp, void* ws,
                                                   size_t ws_bytes, dicp_stream_t stream) {
  dicp::BatchCall batch_call_;  // a call of a launch batch (batch.hpp)
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (M < 0 || nparts < 1 || part < 0 || part >= nparts ||
      (M > 0 && (!q || !p || !gv || !gp)) || !(sigma > 0) ||  // gq may be NULL (gp only), gmG NULL = 0
      (zs && (zrow0 < 0 || znrows < 0 || zrow0 + znrows > M))) {
    set_error("dicp_lddmm_ode_self_bwd_part_f32: invalid arguments");
    return DICP_ERR_INVALID;
  }
  if (M == 0) return DICP_OK;
  switch (D) {
    case 2: return ode_self_bwd_part_d<2>(q, p, gv, gmG, gdiv, M, sigma, eta, part, nparts, gq, gp, ws, ws_bytes, st, zs, zrow0, znrows);
    case 3: return ode_self_bwd_part_d<3>(q, p, gv, gmG, gdiv, M, sigma, eta, part, nparts, gq, gp, ws, ws_bytes, st, zs, zrow0, znrows);
    default: set_error("ode_self_bwd_part: D=%d unsupported", D); return DICP_ERR_UNSUPPORTED;
  }
}

extern "C" int dicp_lddmm_ode_self_bwd_part_f32(const float* q, const float* p, const float* gv,
                                                const float* gmG, const float* gdiv, int64_t M,
                                                int D, double sigma, double eta, int part,
                                                int nparts, float* gq, float* gp, void* ws,
                                                size_t ws_bytes, dicp_stream_t stream) {
  dicp::BatchCall batch_call_;  // a call of a launch batch (batch.hpp)
  return dicp_lddmm_ode_self_bwd_part_zs_f32(q, p, gv, gmG, gdiv, M, D, sigma, eta, part, nparts, nullptr, 0, 0,
                                             gq, gp, ws, ws_bytes, stream);
}

// Workspace sizes for the LDDMM entries (the GMM ones live in gmm.hip).
size_t dicp_lddmm_ws(int kind, int64_t M, int64_t N, int D) {
  if (!supported_dim(D)) return 0;
  switch (kind) {
    case DICP_WS_RED: {
      size_t m = 0;
      size_t c[] = {red_ws<OpKBase>(D, M, N), red_ws<OpKRed>(D, M, N), red_ws<OpGradK>(D, M, N),
                    red_ws<OpGenDK>(D, M, N), red_ws<OpHessK>(D, M, N), red_ws<OpLapK>(D, M, N),
                    red_ws<OpGradLapKPlain>(D, M, N), red_ws<OpGradKScal>(D, M, N),
                    red_ws<OpMinSqDist>(D, M, N), red_ws<OpZDotB>(D, M, N),
                    red_ws<OpDDK>(D, M, N), red_ws<OpKRedScal>(D, M, N),
                    red_ws<OpGradLapKScal>(D, M, N), red_ws<OpMinSqDistOther>(D, M, N),
                    red_ws<OpRadiusCount>(D, M, N),
                    D == 2 ? rowred_pk_ws_bytes<OpExtFwdPk<2, false, false>>(M, N)
                           : rowred_pk_ws_bytes<OpExtFwdPk<3, false, false>>(M, N)};
      for (size_t v : c) m = v > m ? v : m;
      if (cx_eligible(M, N) || (M == N && sym_red() == 2)) {   // (sym_red 2: x = y forced)
        const size_t v = cx_red_ws(M, N, D);
        m = v > m ? v : m;
      }
      return m;
    }
    case DICP_WS_ODE_SELF_FWD: return D == 2 ? ode_self_fwd_ws<2>(M) : ode_self_fwd_ws<3>(M);
    case DICP_WS_ODE_SELF_BWD:
    {
      size_t a = D == 2 ? ws_r<OpOdeSelfBwd<2>>(r_bwd(), M, M) : ws_r<OpOdeSelfBwd<3>>(r_bwd(), M, M);
      size_t b = D == 2 ? ws_r<OpOdeSelfBwdEta<2>>(r_bwd(), M, M) : ws_r<OpOdeSelfBwdEta<3>>(r_bwd(), M, M);
      size_t c = D == 2 ? ws_r<OpOdeSelfBwd2<2>>(r_bwd(), M, M) : ws_r<OpOdeSelfBwd2<3>>(r_bwd(), M, M);
      a = a > b ? a : b;
      a = a > c ? a : c;
      const size_t d = sym_ws_bytes(M, 2 * D);  // SymBwd and SymBwdEta: W = 2D
      return a > d ? a : d;
    }
    case DICP_WS_ODE_EXT_FWD: return D == 2 ? ode_ext_fwd_ws<2>(N, M) : ode_ext_fwd_ws<3>(N, M);
    case DICP_WS_ODE_EXT_BWD: return D == 2 ? ode_ext_bwd_ws<2>(N, M) : ode_ext_bwd_ws<3>(N, M);
    case DICP_WS_ODE_SELF_FWD_ROWS:
      return D == 2 ? ode_self_fwd_rows_ws<2>(M, N) : ode_self_fwd_rows_ws<3>(M, N);
    case DICP_WS_ODE_SELF_FWD_PHASED:
      if (M <= 0 || M >= N) return 0;
      return D == 2 ? euler_step_phase_ws<2>(M, N) : euler_step_phase_ws<3>(M, N);
    case DICP_WS_ODE_SELF_BWD_PART: {
      const int np = N < 1 ? 1 : (int)N;
      return D == 2 ? ode_self_bwd_part_ws<2>(M, np) : ode_self_bwd_part_ws<3>(M, np);
    }
    default: return 0;
  }
}

int dicp_lddmm_splits(int kind, int64_t M, int64_t N) {
  switch (kind) {
    case DICP_WS_ODE_SELF_BWD:
      if (g_bwd_alg == 1)
        return r_bwd() == 1 ? rowred_splits<OpOdeSelfBwd2<3>, 1>(M, M)
             : r_bwd() == 2 ? rowred_splits<OpOdeSelfBwd2<3>, 2>(M, M)
                            : rowred_splits<OpOdeSelfBwd2<3>, 4>(M, M);
      return r_bwd() == 1 ? rowred_splits<OpOdeSelfBwd<3>, 1>(M, M)
           : r_bwd() == 2 ? rowred_splits<OpOdeSelfBwd<3>, 2>(M, M)
                          : rowred_splits<OpOdeSelfBwd<3>, 4>(M, M);
    case DICP_WS_ODE_SELF_FWD:
      return r_fwd() == 1 ? rowred_splits<OpOdeSelfFwd<3, false, true>, 1>(M, M)
           : r_fwd() == 2 ? rowred_splits<OpOdeSelfFwd<3, false, true>, 2>(M, M)
                          : rowred_splits<OpOdeSelfFwd<3, false, true>, 4>(M, M);
    default: return rowred_splits<OpKRed<3>, kR>(M, N);
  }
}
