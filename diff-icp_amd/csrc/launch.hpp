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

constexpr int64_t kMinChunk = 256;  // smallest column chunk of a split

// Resident-workgroup capacity of the device for a kernel: CUs x blocks per CU (occupancy
// query, cached per kernel by the caller).  Falls back to 256 x 4 without a device.
inline int device_cus() {
  static int cus = -1;
  if (cus < 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
      cus = n;
    else
      cus = 256;
  }
  return cus;
}

// Resident 256-thread workgroups per CU from the kernel's resources (MI355X_MICROARCH.md
// "Register files": waves/SIMD = min(8, 512 / alloc(VGPR+AGPR, granule 8)); one wave of a
// 4-wave workgroup per SIMD; LDS 160 KiB per CU).  hipOccupancyMaxActiveBlocksPerMultiprocessor
// under-reports on gfx950 (it assumes a smaller LDS), which made the split model leave
// CUs idle.
template <class K>
int blocks_per_cu(K kernel) {
  hipFuncAttributes at;
  if (hipFuncGetAttributes(&at, reinterpret_cast<const void*>(kernel)) != hipSuccess) {
    (void)hipGetLastError();
    return 4;
  }
  const int vg = at.numRegs > 0 ? ((at.numRegs + 7) / 8) * 8 : 64;
  int waves = 512 / vg;
  if (waves > 8) waves = 8;
  if (waves < 1) waves = 1;
  int b = waves;  // blocks per CU limited by waves per SIMD (1 wave / SIMD / block)
  const size_t lds = at.sharedSizeBytes;
  if (lds > 0) {
    const int bl = (int)((160 * 1024) / lds);
    if (bl < b) b = bl;
  }
  return b < 1 ? 1 : b;
}

// Column split of an M-row x N-column pass, R rows per thread, `cap` resident workgroups.
// The pair loops are latency-bound per wave (long dependent chains through the exp), so the
// chip needs all its wave slots filled: aim at ~g_split_rounds x cap workgroups (chunk
// granularity kChunkGran columns).  Deterministic for given (M, N, R, cap, knob).
constexpr int64_t kChunkGran = 64;
// 0 = automatic: rounds = clamp(M / round_rows, 1, max_rounds), round_rows = 16000 rows for
// the light passes (ODE forward, E-step: 20k rows -> 1, 50k -> 3, 100k -> 6, 200k -> 12) and
// 5000 for the VJP (20k -> 4, 50k -> 10, 100k -> 20, 200k -> 24), from the sweep of
// tools/ab_tune.py --mode rounds on MI355X; > 0 forces a value (dicp_set_option).
// Many short blocks let the dispatcher balance the chip (uneven finish times across CUs /
// XCDs) at the price of S x M partial-slab traffic, which stays far below HBM bandwidth.
inline int& split_rounds() {
  static int r = 0;
  return r;
}
inline int64_t rounds_for(int64_t M, int64_t round_rows, int64_t max_rounds) {
  if (split_rounds() > 0) return split_rounds();
  int64_t r = M / round_rows;
  return r < 1 ? 1 : (r > max_rounds ? max_rounds : r);
}

// Ops may set kRoundRows / kMaxRounds (per-pair-heavy passes want more, shorter blocks).
template <class T, class = void>
struct round_rows_of { static constexpr int64_t rows = 16000, max = 16; };
template <class T>
struct round_rows_of<T, std::void_t<decltype(T::kRoundRows)>> {
  static constexpr int64_t rows = T::kRoundRows, max = T::kMaxRounds;
};

inline int64_t round_chunk(int64_t N, int64_t S) {
  int64_t chunk = (N + S - 1) / S;
  return (chunk + kChunkGran - 1) / kChunkGran * kChunkGran;
}

// Experiment knob (dicp_set_option "force_splits"): > 0 forces the split count.
// dicp_set_option "min_chunk": the smallest column chunk of a split; 0 (default) = kMinChunk.
// At a few thousand columns the 256 floor caps the split count, hence the grid (2k points: 8
// splits x 4 row blocks = 32 workgroups, ~20 us per fused forward pass); 64 measured 27.7 ->
// 26.7 ms per 2k PSR iteration (tools/probes/min_chunk_ab.py), but the changed summation split
// moved a 400-point logdet Ralston gradient to 2.17e-5 of float64 against its 2e-5 bound
// (tests/test_gpu_model.py), so the default stays 256 (forced only)
inline int64_t& min_chunk() {
  static int64_t s = 0;
  return s;
}
inline int64_t min_chunk_for(int64_t) { return min_chunk() > 0 ? min_chunk() : kMinChunk; }

inline int& force_splits() {
  static int s = 0;
  return s;
}

inline int num_splits_cap(int64_t M, int64_t N, int R, int64_t cap, int64_t round_rows = 16000,
                          int64_t max_rounds = 16) {
  if (M <= 0 || N <= 0) return 1;
  const int64_t bx = (M + (int64_t)kBlock * R - 1) / ((int64_t)kBlock * R);
  int64_t S = (rounds_for(M, round_rows, max_rounds) * cap + bx - 1) / bx;
  if (force_splits() > 0) S = force_splits();
  const int64_t mc = min_chunk_for(N);
  int64_t smax = (N + mc - 1) / mc;
  if (smax < 1) smax = 1;
  if (S > smax) S = smax;
  if (S < 1) S = 1;
  const int64_t chunk = round_chunk(N, S);
  return (int)((N + chunk - 1) / chunk);
}

inline int64_t chunk_of(int64_t N, int S) { return round_chunk(N, S); }

template <class Op, int R>
__global__ __launch_bounds__(kBlock) void rowred_kernel(Args, Scal, int64_t, int64_t, int64_t, Outs);

template <class Op, int R>
int64_t rowred_capacity() {
  static int64_t cap = -1;
  if (cap < 0) cap = (int64_t)device_cus() * blocks_per_cu(rowred_kernel<Op, R>);
  return cap;
}

template <class Op, int R>
int rowred_splits(int64_t M, int64_t N) {
  return num_splits_cap(M, N, R, rowred_capacity<Op, R>(), round_rows_of<Op>::rows,
                        round_rows_of<Op>::max);
}

inline int check_launch(const char* what) {
  if (batching()) return batch_check(what);
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
  const int S = rowred_splits<Op, R>(M, N);
  if (S <= 1) return 0;
  return (size_t)S * (size_t)M * (size_t)total_out_width<Op>() * sizeof(float);
}

// Launch Op over rows [0,M) x columns [0,N).  `fin` holds the final output pointers and
// accumulate flags.  Split partial slabs are carved from ws and merged in chunk order.
template <class Op, int R>
int launch_rowred(const char* name, const Args& a, const Scal& sc, int64_t M, int64_t N,
                  const Outs& fin, void* ws, size_t ws_bytes, hipStream_t st) {
  if (int rc = no_batch("rowred (scalar rows)")) return rc;
  if (M <= 0) return DICP_OK;
  const int S = rowred_splits<Op, R>(M, N);
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
    merge_slabs_kernel<Op::kMin><<<dim3((unsigned)nb, (unsigned)nk), dim3(kBlock), 0, st>>>(ms, fin, S);
    rc = check_launch(name);
    if (rc) return rc;
  }
  return DICP_OK;
}

// Centred-expansion reductions (centred.hpp / centred.hip).  red_alg: 0 = never (generic
// skeleton), 1 = automatic (large enough passes), 2 = always; cx_rho_x100: sub-tile radius (in
// scaled units x 100) up to which the expanded exponent is used.
int& red_alg();
// pair-once centred sums when the rows are the columns (sym_cx.hpp): 0 off, 1 auto, 2 always
int& sym_red();
int& sym_red_rows();   // rows per lane of the pair-once sums: 0 auto, 4, 8
int& lse_adapt();      // E / M passes: eventful tiles before the per-pair re-reference test
int& lse_bound();      // many-component E-step: 1 the bound shift + exact re-sum of listed rows
int& lse_pk();         // E / M passes: 1 packed row pairs (v_pk_*), 0 scalar rows
int& cx_rho_x100();
// rows M, columns N; ext: the external-point forward (its non-centred kernel is the packed one)
bool cx_eligible(int64_t M, int64_t N, bool ext = false);
bool scx_eligible(int op, const float* x, int64_t M, const float* y, int64_t N);
bool cx_has_op(int op);
int cx_gauss_red(int op, const float* x, int64_t M, const float* y, int64_t N, int D, const float* b,
                 double sigma, float* out, void* ws, size_t wsb, hipStream_t st);
int cx_ext_fwd(const float* x, int64_t N, const float* q, const float* p, int64_t M, int D, double sigma,
               double eta, float* vx, float* gx, void* ws, size_t wsb, hipStream_t st);
size_t cx_red_ws(int64_t M, int64_t N, int D);
size_t cx_ext_ws(int64_t N, int64_t M, int D);

// sigma and eta of the calling thread's latest make_scal, in double: the launch constants the
// eta != 0 forward forms in double on the host (packed.hpp eta_consts) read them
inline thread_local double tl_launch_sigma = 1.0;
inline thread_local double tl_launch_eta = 0.0;

inline Scal make_scal(double sigma, double eta) {
  tl_launch_sigma = sigma;
  tl_launch_eta = eta;
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
  for (int k = 0; k < 4; ++k) {
    o.accumulate[k] = 0;
    o.base[k] = nullptr;
    o.add[k] = nullptr;
    o.alpha[k] = 1.f;
  }
  return o;
}

}  // namespace dicp
