// Host-side launch helpers: split-column choice, workspace carving, error reporting.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>
#include <stdio.h>
#include <string>

#include "../../include/difficp_hip.h"
#include "common.hpp"

namespace dicp {

void set_error(const char* fmt, ...);

// Workgroups we aim for per pass: 256 CUs x ~8 resident workgroups, so that the tail of
// an unevenly-clocked chip (8 XCDs) stays short.
constexpr int64_t kTargetBlocks = 2048;
constexpr int64_t kMinChunk = 2 * kTile;

// Number of column chunks (gridDim.y) for an M-row, N-column pass with R rows per thread.
inline int num_splits(int64_t M, int64_t N, int R) {
  if (M <= 0 || N <= 0) return 1;
  const int64_t bx = (M + (int64_t)kBlock * R - 1) / ((int64_t)kBlock * R);
  int64_t S = (kTargetBlocks + bx - 1) / bx;
  const int64_t smax = (N + kMinChunk - 1) / kMinChunk;
  if (S > smax) S = smax;
  if (S < 1) S = 1;
  // chunk rounded up to whole tiles; recompute S so no chunk is empty
  int64_t chunk = (N + S - 1) / S;
  chunk = (chunk + kTile - 1) / kTile * kTile;
  S = (N + chunk - 1) / chunk;
  return (int)S;
}

inline int64_t chunk_of(int64_t N, int S) {
  int64_t chunk = (N + S - 1) / S;
  return (chunk + kTile - 1) / kTile * kTile;
}

inline int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: HIP launch failed: %s", what, hipGetErrorString(e));
    return DICP_ERR_HIP;
  }
  return DICP_OK;
}

template <class Op>
constexpr int total_out_width() {
  return Op::kOutW[0] + Op::kOutW[1] + Op::kOutW[2] + Op::kOutW[3];
}

template <class Op, int R>
size_t rowred_ws_bytes(int64_t M, int64_t N) {
  const int S = num_splits(M, N, R);
  if (S <= 1) return 0;
  return (size_t)S * (size_t)M * (size_t)total_out_width<Op>() * sizeof(float);
}

// Launch Op over rows [0,M) x columns [0,N).  `fin` holds the final output pointers and
// accumulate flags.  Split partial slabs are carved from ws and merged in chunk order.
template <class Op, int R>
int launch_rowred(const char* name, const Args& a, const Scal& sc, int64_t M, int64_t N,
                  const Outs& fin, void* ws, size_t ws_bytes, hipStream_t st) {
  if (M <= 0) return DICP_OK;
  const int S = num_splits(M, N, R);
  const int64_t chunk = N > 0 ? chunk_of(N, S) : 0;
  const int64_t bx = (M + (int64_t)kBlock * R - 1) / ((int64_t)kBlock * R);
  if (bx > 0x7fffffff) {
    set_error("%s: too many rows (%lld)", name, (long long)M);
    return DICP_ERR_INVALID;
  }
  dim3 grid((unsigned)bx, (unsigned)S, 1), block(kBlock, 1, 1);
  if (S == 1) {
    rowred_kernel<Op, R><<<grid, block, 0, st>>>(a, sc, M, N, chunk, fin);
    return check_launch(name);
  }
  const size_t need = rowred_ws_bytes<Op, R>(M, N);
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
  rowred_kernel<Op, R><<<grid, block, 0, st>>>(a, sc, M, N, chunk, part);
  int rc = check_launch(name);
  if (rc) return rc;
  for (int k = 0; k < Op::kNOut; ++k) {
    if (!fin.ptr[k]) continue;
    const int64_t n = M * Op::kOutW[k];
    const int64_t nb = (n + kBlock - 1) / kBlock;
    merge_slabs_kernel<Op::kMin><<<dim3((unsigned)nb), dim3(kBlock), 0, st>>>(
        part.ptr[k], n, S, fin.ptr[k], fin.accumulate[k]);
    rc = check_launch(name);
    if (rc) return rc;
  }
  return DICP_OK;
}

inline Scal make_scal(double sigma, double eta) {
  Scal sc;
  const double s = 1.0 / (sigma * sigma);
  sc.nc = (float)(-1.4426950408889634 * 0.5 * s);
  sc.s = (float)s;
  sc.eta = (float)eta;
  sc.aux0 = 0.f;
  sc.aux1 = 0.f;
  sc.dev0 = nullptr;
  return sc;
}

inline Outs make_outs(float* p0, float* p1 = nullptr, float* p2 = nullptr, float* p3 = nullptr) {
  Outs o;
  o.ptr[0] = p0;
  o.ptr[1] = p1;
  o.ptr[2] = p2;
  o.ptr[3] = p3;
  for (int k = 0; k < 4; ++k) o.accumulate[k] = 0;
  return o;
}

}  // namespace dicp
