// C-ABI entry points of the Gaussian-kernel reductions (GenKernel, kernel.py:58-337) and of
// the fused LDDMM geodesic-shooting ODE (LDDMMModel.ODE, LDDMM.py:176-227) for gfx950.
#include "launch.hpp"
#include "lddmm_ops.hpp"

using namespace dicp;

namespace {

constexpr int kR = 2;       // rows per thread for the light reductions / fused forward
constexpr int kRBwd = 1;    // rows per thread for the (register-heavy) fused backward

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

}  // namespace

extern "C" int dicp_supports_dim(int D) { return supported_dim(D) ? 1 : 0; }

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
    default: set_error("dicp_gauss_red_f32: unknown op %d", op); return DICP_ERR_UNSUPPORTED;
  }
}

// ---------------------------------------------------------------------------------------
// Fused ODE
// ---------------------------------------------------------------------------------------
namespace {

template <int D>
int ode_self_fwd_d(const float* q, const float* p, int64_t M, double sigma, double eta, float* v,
                   float* mG, float* g, float* h, void* ws, size_t wsb, hipStream_t st) {
  const Args a = {q, p, nullptr, nullptr, q, p, nullptr, nullptr};
  const Scal sc = make_scal(sigma, eta);
  const Outs o = make_outs(v, mG, g, h);
  if (eta != 0.0)
    return launch_rowred<OpOdeSelfFwd<D, true, true>, kR>("ode_self_fwd", a, sc, M, M, o, ws, wsb, st);
  if (g != nullptr)
    return launch_rowred<OpOdeSelfFwd<D, false, true>, kR>("ode_self_fwd", a, sc, M, M, o, ws, wsb, st);
  return launch_rowred<OpOdeSelfFwd<D, false, false>, kR>("ode_self_fwd", a, sc, M, M, o, ws, wsb, st);
}

template <int D>
size_t ode_self_fwd_ws(int64_t M) {
  size_t a = rowred_ws_bytes<OpOdeSelfFwd<D, true, true>, kR>(M, M);
  size_t b = rowred_ws_bytes<OpOdeSelfFwd<D, false, true>, kR>(M, M);
  return a > b ? a : b;
}

template <int D>
int ode_self_bwd_d(const float* q, const float* p, const float* gv, const float* gmG,
                   const float* gdiv, int64_t M, double sigma, float* gq, float* gp, void* ws,
                   size_t wsb, hipStream_t st) {
  const Args a = {q, p, gv, gmG, q, p, gv, gmG};
  Scal sc = make_scal(sigma, 0.0);
  sc.dev0 = gdiv;  // nullptr -> aux0 = 0
  const Outs o = make_outs(gq, gp);
  return launch_rowred<OpOdeSelfBwd<D>, kRBwd>("ode_self_bwd", a, sc, M, M, o, ws, wsb, st);
}

template <int D>
int ode_ext_fwd_d(const float* x, int64_t N, const float* q, const float* p, int64_t M,
                  double sigma, double eta, float* vx, float* gx, void* ws, size_t wsb,
                  hipStream_t st) {
  const Args a = {x, nullptr, nullptr, nullptr, q, p, nullptr, nullptr};
  const Scal sc = make_scal(sigma, eta);
  const Outs o = make_outs(vx, gx);
  if (eta != 0.0) {
    if (gx) return launch_rowred<OpOdeExtFwd<D, true, true>, kR>("ode_ext_fwd", a, sc, N, M, o, ws, wsb, st);
    return launch_rowred<OpOdeExtFwd<D, true, false>, kR>("ode_ext_fwd", a, sc, N, M, o, ws, wsb, st);
  }
  if (gx) return launch_rowred<OpOdeExtFwd<D, false, true>, kR>("ode_ext_fwd", a, sc, N, M, o, ws, wsb, st);
  return launch_rowred<OpOdeExtFwd<D, false, false>, kR>("ode_ext_fwd", a, sc, N, M, o, ws, wsb, st);
}

template <int D>
size_t ode_ext_fwd_ws(int64_t N, int64_t M) {
  size_t a = rowred_ws_bytes<OpOdeExtFwd<D, true, true>, kR>(N, M);
  size_t b = rowred_ws_bytes<OpOdeExtFwd<D, false, true>, kR>(N, M);
  return a > b ? a : b;
}

template <int D>
int ode_ext_bwd_d(const float* x, int64_t N, const float* q, const float* p, int64_t M,
                  double sigma, const float* gvx, const float* gdiv, float* gxo, float* gq,
                  float* gp, void* ws, size_t wsb, hipStream_t st) {
  Scal sc = make_scal(sigma, 0.0);
  sc.dev0 = gdiv;
  // rows x: gradient w.r.t. the carried points
  {
    const Args a = {x, gvx, nullptr, nullptr, q, p, nullptr, nullptr};
    const Outs o = make_outs(gxo);
    int rc = launch_rowred<OpOdeExtBwdX<D>, kR>("ode_ext_bwd_x", a, sc, N, M, o, ws, wsb, st);
    if (rc) return rc;
  }
  // rows q: gradient w.r.t. support points and momenta (accumulated)
  {
    const Args a = {q, p, nullptr, nullptr, x, gvx, nullptr, nullptr};
    Outs o = make_outs(gq, gp);
    o.accumulate[0] = o.accumulate[1] = 1;
    return launch_rowred<OpOdeExtBwdQ<D>, kR>("ode_ext_bwd_q", a, sc, M, N, o, ws, wsb, st);
  }
}

template <int D>
size_t ode_ext_bwd_ws(int64_t N, int64_t M) {
  size_t a = rowred_ws_bytes<OpOdeExtBwdX<D>, kR>(N, M);
  size_t b = rowred_ws_bytes<OpOdeExtBwdQ<D>, kR>(M, N);
  return a > b ? a : b;
}

}  // namespace

extern "C" int dicp_lddmm_ode_self_fwd_f32(const float* q, const float* p, int64_t M, int D,
                                           double sigma, double eta, float* v, float* mG,
                                           float* g, float* h, void* ws, size_t ws_bytes,
                                           dicp_stream_t stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (M < 0 || (M > 0 && (!q || !p || !v || !mG)) || !(sigma > 0)) {
    set_error("dicp_lddmm_ode_self_fwd_f32: invalid arguments");
    return DICP_ERR_INVALID;
  }
  switch (D) {
    case 2: return ode_self_fwd_d<2>(q, p, M, sigma, eta, v, mG, g, h, ws, ws_bytes, st);
    case 3: return ode_self_fwd_d<3>(q, p, M, sigma, eta, v, mG, g, h, ws, ws_bytes, st);
    default: set_error("ode_self_fwd: D=%d unsupported", D); return DICP_ERR_UNSUPPORTED;
  }
}

extern "C" int dicp_lddmm_ode_self_bwd_f32(const float* q, const float* p, const float* gv,
                                           const float* gmG, const float* gdiv, int64_t M,
                                           int D, double sigma, double eta, float* gq,
                                           float* gp, void* ws, size_t ws_bytes,
                                           dicp_stream_t stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (M < 0 || (M > 0 && (!q || !p || !gv || !gmG || !gq || !gp)) || !(sigma > 0)) {
    set_error("dicp_lddmm_ode_self_bwd_f32: invalid arguments");
    return DICP_ERR_INVALID;
  }
  if (eta != 0.0) {
    set_error("ode_self_bwd: eta != 0 (gradcomponent=True) backward not compiled in yet");
    return DICP_ERR_UNSUPPORTED;
  }
  switch (D) {
    case 2: return ode_self_bwd_d<2>(q, p, gv, gmG, gdiv, M, sigma, gq, gp, ws, ws_bytes, st);
    case 3: return ode_self_bwd_d<3>(q, p, gv, gmG, gdiv, M, sigma, gq, gp, ws, ws_bytes, st);
    default: set_error("ode_self_bwd: D=%d unsupported", D); return DICP_ERR_UNSUPPORTED;
  }
}

extern "C" int dicp_lddmm_ode_ext_fwd_f32(const float* x, int64_t N, const float* q,
                                          const float* p, int64_t M, int D, double sigma,
                                          double eta, float* vx, float* gx, void* ws,
                                          size_t ws_bytes, dicp_stream_t stream) {
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
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (N < 0 || M < 0 || (N > 0 && (!x || !gvx || !gxo)) || (M > 0 && (!q || !p || !gq || !gp)) ||
      !(sigma > 0)) {
    set_error("dicp_lddmm_ode_ext_bwd_f32: invalid arguments");
    return DICP_ERR_INVALID;
  }
  if (eta != 0.0) {
    set_error("ode_ext_bwd: eta != 0 (gradcomponent=True) backward not compiled in yet");
    return DICP_ERR_UNSUPPORTED;
  }
  switch (D) {
    case 2: return ode_ext_bwd_d<2>(x, N, q, p, M, sigma, gvx, gdiv, gxo, gq, gp, ws, ws_bytes, st);
    case 3: return ode_ext_bwd_d<3>(x, N, q, p, M, sigma, gvx, gdiv, gxo, gq, gp, ws, ws_bytes, st);
    default: set_error("ode_ext_bwd: D=%d unsupported", D); return DICP_ERR_UNSUPPORTED;
  }
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
                    red_ws<OpGradLapKScal>(D, M, N)};
      for (size_t v : c) m = v > m ? v : m;
      return m;
    }
    case DICP_WS_ODE_SELF_FWD: return D == 2 ? ode_self_fwd_ws<2>(M) : ode_self_fwd_ws<3>(M);
    case DICP_WS_ODE_SELF_BWD:
      return D == 2 ? rowred_ws_bytes<OpOdeSelfBwd<2>, kRBwd>(M, M)
                    : rowred_ws_bytes<OpOdeSelfBwd<3>, kRBwd>(M, M);
    case DICP_WS_ODE_EXT_FWD: return D == 2 ? ode_ext_fwd_ws<2>(N, M) : ode_ext_fwd_ws<3>(N, M);
    case DICP_WS_ODE_EXT_BWD: return D == 2 ? ode_ext_bwd_ws<2>(N, M) : ode_ext_bwd_ws<3>(N, M);
    default: return 0;
  }
}

int dicp_lddmm_splits(int kind, int64_t M, int64_t N) {
  switch (kind) {
    case DICP_WS_ODE_SELF_BWD: return num_splits(M, M, kRBwd);
    case DICP_WS_ODE_SELF_FWD: return num_splits(M, M, kR);
    default: return num_splits(M, N, kR);
  }
}
