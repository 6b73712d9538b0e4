// Kernel ridge solve (K(x,x) + alpha I) b = v on the device by conjugate gradients, the
// mat-vec being the KRed reduction (lddmm_ops.hpp OpKRed).  Replaces the dense host solves
// the reference uses to convert speeds into momenta (LDDMMModel.v2p, LDDMM.py:235-253):
// KridgeSolve_keops (kernel.py:239-241, KeOps LazyTensor.solve = CG on the flattened (M,D)
// system with ridge alpha) and KridgeSolve_torch (kernel.py:234-237, dense torch.linalg.solve).
//
// Structure (MI355X-first): each CG iteration is two launches on the caller's stream --
//   1. the O(M^2) mat-vec  Kp = KRed(x, x, p)            (tiled rowred kernel, all CUs)
//   2. one single-workgroup update kernel (O(M D) work): pAp = <p, Kp + alpha p>,
//      b += a p, r -= a (Kp + alpha p), rr' = <r, r>, p = r + (rr'/rr) p, convergence test
//      (fixed-order tree sums: deterministic, no atomics).
// A device flag `done` makes every later launch of the chunk a no-op once the residual test
// passes, so the host launches `iters` iterations ahead without synchronising and reads the
// 16-byte status block only between chunks.
#include "launch.hpp"
#include "lddmm_ops.hpp"

#include <cmath>

using namespace dicp;

namespace {

constexpr int kUpdBlock = 1024;  // threads of the single-workgroup update kernel

// State block at the head of the workspace (device):
//   status[0] = done flag (int), status[1] = iterations performed (int),
//   f[2] = <r,r> (current), f[3] = convergence threshold delta
struct CgState {
  int done;
  int iters;
  float rr;
  float delta;
  float fdone;  // done as a float: the mat-vec's skip flag (OpKRedCg, Scal::dev0)
};

// KRed mat-vec that turns into a no-op once the solver has converged (common.hpp
// skip_on_aux0: the rowred kernel returns when the device scalar dev0 is nonzero).
template <int D>
struct OpKRedCg : OpKRed<D> {
  static constexpr bool kSkipOnAux0 = true;
};

constexpr size_t kStateBytes = 256;

size_t align256(size_t b) { return (b + 255) / 256 * 256; }

// Fixed-order block sum of one float per thread (kUpdBlock threads).
__device__ float block_sum(float v, float* sh) {
  const int t = threadIdx.x;
  sh[t] = v;
  __syncthreads();
#pragma unroll
  for (int s = kUpdBlock / 2; s > 0; s >>= 1) {
    if (t < s) sh[t] += sh[t + s];
    __syncthreads();
  }
  const float r = sh[0];
  __syncthreads();
  return r;
}

// b = 0, r = v, p = v, rr = <v,v>, delta = n * eps^2 (KeOps ConjugateGradientSolver
// stopping rule: |r|^2 < size(b) eps^2); done if rr < delta already (returns b = 0).
__global__ __launch_bounds__(kUpdBlock) void cg_init_kernel(const float* __restrict__ v, int64_t n,
                                                            float eps, float* __restrict__ b,
                                                            float* __restrict__ r, float* __restrict__ p,
                                                            CgState* st) {
  __shared__ float sh[kUpdBlock];
  float acc = 0.f;
  for (int64_t e = threadIdx.x; e < n; e += kUpdBlock) {
    const float x = v[e];
    b[e] = 0.f;
    r[e] = x;
    p[e] = x;
    acc = fmaf(x, x, acc);
  }
  const float rr = block_sum(acc, sh);
  if (threadIdx.x == 0) {
    st->rr = rr;
    st->delta = (float)n * eps * eps;
    st->iters = 0;
    st->done = !(rr >= st->delta);  // also stops on NaN input
    st->fdone = st->done ? 1.f : 0.f;
  }
}

__global__ __launch_bounds__(kUpdBlock) void cg_update_kernel(const float* __restrict__ kp,
                                                              float alpha, int64_t n,
                                                              float* __restrict__ b,
                                                              float* __restrict__ r,
                                                              float* __restrict__ p, CgState* st) {
  __shared__ float sh[kUpdBlock];
  if (st->done) return;
  // <p, (K + alpha I) p>
  float acc = 0.f;
  for (int64_t e = threadIdx.x; e < n; e += kUpdBlock) {
    const float pe = p[e];
    acc = fmaf(pe, fmaf(alpha, pe, kp[e]), acc);
  }
  const float pap = block_sum(acc, sh);
  const float rr = st->rr;
  if (!(pap > 0.f)) {  // breakdown (K + alpha I is SPD: only from round-off / NaN)
    if (threadIdx.x == 0) st->done = 2, st->fdone = 1.f;
    return;
  }
  const float a = rr / pap;
  acc = 0.f;
  for (int64_t e = threadIdx.x; e < n; e += kUpdBlock) {
    const float pe = p[e];
    b[e] = fmaf(a, pe, b[e]);
    const float re = fmaf(-a, fmaf(alpha, pe, kp[e]), r[e]);
    r[e] = re;
    acc = fmaf(re, re, acc);
  }
  const float rrn = block_sum(acc, sh);
  const bool conv = rrn < st->delta;
  if (!conv) {
    const float beta = rrn / rr;
    for (int64_t e = threadIdx.x; e < n; e += kUpdBlock) p[e] = fmaf(beta, p[e], r[e]);
  }
  if (threadIdx.x == 0) {
    st->rr = rrn;
    st->iters += 1;
    if (conv) st->done = 1, st->fdone = 1.f;
  }
}

template <int D>
size_t cg_ws(int64_t M) {
  const size_t vec = align256((size_t)M * D * sizeof(float));
  return kStateBytes + 3 * vec + rowred_ws_bytes<OpKRedCg<D>, 2>(M, M);
}

template <int D>
int cg_run(const float* x, int64_t M, double sigma, double alpha, double eps, const float* v,
           float* b, int start, int iters, void* ws, size_t wsb, hipStream_t stream) {
  const size_t need = cg_ws<D>(M);
  if (ws == nullptr || wsb < need) {
    set_error("dicp_kernel_ridge_cg_f32: workspace too small (%zu < %zu bytes)", wsb, need);
    return DICP_ERR_WORKSPACE;
  }
  const int64_t n = M * D;
  char* w = reinterpret_cast<char*>(ws);
  CgState* st = reinterpret_cast<CgState*>(w);
  const size_t vec = align256((size_t)n * sizeof(float));
  float* r = reinterpret_cast<float*>(w + kStateBytes);
  float* p = reinterpret_cast<float*>(w + kStateBytes + vec);
  float* kp = reinterpret_cast<float*>(w + kStateBytes + 2 * vec);
  void* rws = w + kStateBytes + 3 * vec;
  const size_t rwsb = wsb - (kStateBytes + 3 * vec);
  if (start) {
    cg_init_kernel<<<1, kUpdBlock, 0, stream>>>(v, n, (float)eps, b, r, p, st);
    const int rc = check_launch("kernel_ridge_cg(init)");
    if (rc) return rc;
  }
  Args a = {x, nullptr, nullptr, nullptr, x, p, nullptr, nullptr, 0.f};
  Scal sc = make_scal(sigma, 0.0);
  sc.dev0 = &st->fdone;
  const Outs o = make_outs(kp);
  for (int it = 0; it < iters; ++it) {
    int rc = launch_rowred<OpKRedCg<D>, 2>("kernel_ridge_cg(matvec)", a, sc, M, M, o, rws, rwsb, stream);
    if (rc) return rc;
    cg_update_kernel<<<1, kUpdBlock, 0, stream>>>(kp, (float)alpha, n, b, r, p, st);
    rc = check_launch("kernel_ridge_cg(update)");
    if (rc) return rc;
  }
  return DICP_OK;
}

}  // namespace

extern "C" int dicp_kernel_ridge_cg_f32(const float* x, int64_t M, int D, double sigma,
                                        double alpha, double eps, const float* v, float* b,
                                        int start, int iters, void* ws, size_t ws_bytes,
                                        dicp_stream_t stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (M <= 0 || !x || !v || !b || !(sigma > 0) || !(alpha >= 0) || !(eps > 0) || iters < 0 ||
      M * D > INT32_MAX) {
    set_error("dicp_kernel_ridge_cg_f32: invalid arguments");
    return DICP_ERR_INVALID;
  }
  switch (D) {
    case 2: return cg_run<2>(x, M, sigma, alpha, eps, v, b, start, iters, ws, ws_bytes, st);
    case 3: return cg_run<3>(x, M, sigma, alpha, eps, v, b, start, iters, ws, ws_bytes, st);
    default: set_error("dicp_kernel_ridge_cg_f32: D=%d unsupported", D); return DICP_ERR_UNSUPPORTED;
  }
}

size_t dicp_solve_ws(int kind, int64_t M, int D) {
  (void)kind;
  if (D == 2) return cg_ws<2>(M);
  if (D == 3) return cg_ws<3>(M);
  return 0;
}
