// C-ABI entry of the gradient reductions (grad_ops.hpp): the backward passes of the
// Gaussian-kernel reductions GenDKRed, HessKRed, GradLapKRed, DDKRed and GradKRed_rev that
// the reference gets from KeOps / torch autodiff (kernel.py:147-168, :194-207, :284-292).
#include "grad_ops.hpp"
#include "launch.hpp"

using namespace dicp;

namespace {

template <int D, int KIND>
int grad_launch(const Args& a, const Scal& sc, int64_t M, int64_t N, float* out, void* ws, size_t wsb,
                hipStream_t st) {
  return launch_rowred<OpGrad<D, KIND>, 2>("gauss_red_grad", a, sc, M, N, make_outs(out), ws, wsb, st);
}

template <int D>
int grad_dispatch(int kind, const Args& a, const Scal& sc, int64_t M, int64_t N, float* out, void* ws,
                  size_t wsb, hipStream_t st) {
  switch (kind) {
    case DICP_GRAD_HESSW: return grad_launch<D, kHessW>(a, sc, M, N, out, ws, wsb, st);
    case DICP_GRAD_HESSWP: return grad_launch<D, kHessWP>(a, sc, M, N, out, ws, wsb, st);
    case DICP_GRAD_ZDOTV: return grad_launch<D, kZDotV>(a, sc, M, N, out, ws, wsb, st);
    case DICP_GRAD_HESS3: return grad_launch<D, kHess3>(a, sc, M, N, out, ws, wsb, st);
    case DICP_GRAD_GRADLAP3: return grad_launch<D, kGradLap3>(a, sc, M, N, out, ws, wsb, st);
    default: set_error("dicp_gauss_red_grad_f32: unknown kind %d", kind); return DICP_ERR_UNSUPPORTED;
  }
}

template <int D>
size_t grad_ws_d(int64_t M, int64_t N) {
  size_t m = 0;
  for (size_t v : {rowred_ws_bytes<OpGrad<D, kHessW>, 2>(M, N), rowred_ws_bytes<OpGrad<D, kHessWP>, 2>(M, N),
                   rowred_ws_bytes<OpGrad<D, kZDotV>, 2>(M, N), rowred_ws_bytes<OpGrad<D, kHess3>, 2>(M, N),
                   rowred_ws_bytes<OpGrad<D, kGradLap3>, 2>(M, N)})
    m = v > m ? v : m;
  return m;
}

}  // namespace

size_t dicp_grad_ws(int64_t M, int64_t N, int D) {
  return D == 2 ? grad_ws_d<2>(M, N) : D == 3 ? grad_ws_d<3>(M, N) : 0;
}

extern "C" int dicp_gauss_red_grad_f32(int kind, const float* x, int64_t M, const float* y, int64_t N, int D,
                                       const float* r1, const float* r2, const float* c1, const float* c2,
                                       const float* cw, double sigma, float* out, void* ws, size_t ws_bytes,
                                       dicp_stream_t stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (M < 0 || N < 0 || (M > 0 && (!x || !out)) || (N > 0 && !y) || !(sigma > 0)) {
    set_error("dicp_gauss_red_grad_f32: invalid arguments");
    return DICP_ERR_INVALID;
  }
  if (M == 0) return DICP_OK;
  if (N == 0) {  // empty sum
    if (hipMemsetAsync(out, 0, (size_t)M * D * sizeof(float), st) != hipSuccess) {
      set_error("dicp_gauss_red_grad_f32: hipMemsetAsync failed");
      return DICP_ERR_HIP;
    }
    return DICP_OK;
  }
  const Args a = {x, r1, r2, nullptr, y, c1, c2, cw, 0.f};
  const Scal sc = make_scal(sigma, 0.0);
  switch (D) {
    case 2: return grad_dispatch<2>(kind, a, sc, M, N, out, ws, ws_bytes, st);
    case 3: return grad_dispatch<3>(kind, a, sc, M, N, out, ws, ws_bytes, st);
    default: set_error("gauss_red_grad: D=%d not compiled in (supported: 2, 3)", D); return DICP_ERR_UNSUPPORTED;
  }
}
