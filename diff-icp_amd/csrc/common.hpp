// Shared machinery of the diff-ICP gfx950 kernels: the tiled "row reduction over column
// tiles staged in LDS" skeleton that every N x M pass (Gaussian-kernel sums, fused LDDMM
// ODE, GMM E/M/targets passes) is built from, plus the deterministic split-column merge.
//
// Design (MI355X-first):
//  * one workgroup = 256 threads = 4 wave64; each thread owns R target rows held in VGPRs;
//  * the column range [j0, j1) of this workgroup is swept in tiles of 256 column records
//    staged in LDS (one record per thread, float4-packed); every lane of a wave reads the
//    SAME record address -> LDS broadcast, conflict-free; each record read serves R rows;
//  * per-tile partial accumulators are folded into running totals once per tile
//    (two-level summation: fp32 error ~ (sqrt(256)+sqrt(N/256)) ulp instead of ~sqrt(N));
//  * when M alone cannot fill 256 CUs x several waves, the column range is split over
//    gridDim.y chunks; each chunk writes its own partial slab and a second tiny kernel
//    sums the slabs in chunk order: no float atomics, bitwise-deterministic results;
//  * the Gaussian exponential is one v_exp_f32 (exp2) with log2(e)/(2 sigma^2) folded
//    into a single multiplier.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "batch.hpp"

namespace dicp {

#ifndef DICP_STAGE_EARLY
#define DICP_STAGE_EARLY 1
#endif
#ifndef DICP_PAIR_UNROLL
#define DICP_PAIR_UNROLL 2
#endif
#ifdef DICP_WAVES_PER_EU
#define DICP_KERNEL_ATTR __attribute__((amdgpu_waves_per_eu(DICP_WAVES_PER_EU)))
#else
#define DICP_KERNEL_ATTR
#endif

constexpr int kBlock = 256;       // threads per workgroup (4 waves)
#ifndef DICP_TILE
#define DICP_TILE 256
#endif
constexpr int kTile = DICP_TILE;  // column records per LDS tile (<= kBlock, one per staging thread)
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float fast_log2(float x) { return __builtin_amdgcn_logf(x); }

// Scalars every pair op may need.  nc = -log2(e)/(2 sigma^2): K = exp2(nc * |z|^2).
struct Scal {
  float nc;    // exp2 multiplier
  float s;     // 1/sigma^2
  float eta;   // gradcomponent weight (0 or 1/lambda)
  float aux0;  // op-specific
  float aux1;  // op-specific
  const float* dev0;  // op-specific device scalar (e.g. cotangent of the divergence sum)
};

// Row / column pointers of one pass (meaning fixed per op).
struct Args {
  const float* r0;
  const float* r1;
  const float* r2;
  const float* r3;
  const float* c0;
  const float* c1;
  const float* c2;
  const float* c3;
  // coordinate pre-scale alpha = sqrt(log2(e) / (2 sigma^2)) for ops that work in scaled
  // coordinates (K = exp2(-|alpha z|^2) needs no per-pair multiply); 0 when unused
  float scale;
  // origin of the scaled coordinates q' = alpha (q - shift): a device D-vector (the first
  // support point) or NULL (0).  Pair terms only see differences, so the shift changes no
  // result in exact arithmetic; it keeps |q'| at the cloud's extent over sigma whatever the
  // offset of the coordinates, so the rounding of q' does not grow with that offset.
  const float* shift;
};

template <int D>
__device__ __forceinline__ void load_shift(const Args& a, float* c) {
#pragma unroll
  for (int d = 0; d < D; ++d) c[d] = a.shift ? a.shift[d] : 0.f;
}
// scaled coordinates of point i of p (D floats): alpha (p_i - shift)
template <int D>
__device__ __forceinline__ void ld_coord(const Args& a, const float* __restrict__ p, int64_t i, float* dst) {
  float c[D];
  load_shift<D>(a, c);
#pragma unroll
  for (int d = 0; d < D; ++d) dst[d] = a.scale * (p[i * D + d] - c[d]);
}

// Output descriptor: up to 4 output arrays, each (rows, width) row-major.
// In split mode the kernel writes partial slab `blockIdx.y` of each output at
// out[k] + blockIdx.y * rows * width[k] and the merge applies the epilogue; otherwise the
// kernel applies it.  Epilogue per element e of output k (the reduced value a):
//   out[k][e] = (base[k] ? base[k][e] : 0) + alpha[k] * a + (add[k] ? add[k][e] : 0)
//               (+ out[k][e] first if accumulate[k])
// which fuses integrator updates such as q_next = q + dt v into the reduction.
struct Outs {
  float* ptr[4];
  int accumulate[4];
  const float* base[4];
  const float* add[4];
  float alpha[4];
};

__device__ __forceinline__ float epilogue(const Outs& o, int k, int64_t e, float a) {
  float v = o.alpha[k] * a;
  if (o.base[k]) v += o.base[k][e];
  if (o.add[k]) v += o.add[k][e];
  if (o.accumulate[k]) v += o.ptr[k][e];
  return v;
}

// Ops may define load_row_s / load_col_s, which also see the launch scalars (e.g. to stage
// a scalar-premultiplied copy of a column field in LDS once per column instead of
// multiplying once per pair).
template <class T, class = void>
struct has_row_s : std::false_type {};
template <class T>
struct has_row_s<T, std::void_t<decltype(&T::load_row_s)>> : std::true_type {};
template <class T, class = void>
struct has_col_s : std::false_type {};
template <class T>
struct has_col_s<T, std::void_t<decltype(&T::load_col_s)>> : std::true_type {};

template <class T, class = void>
struct skip_on_aux0 : std::false_type {};
template <class T>
struct skip_on_aux0<T, std::void_t<decltype(T::kSkipOnAux0)>> : std::bool_constant<T::kSkipOnAux0> {};

template <class Op>
__device__ __forceinline__ void op_load_row(const Args& a, const Scal& sc, int64_t i,
                                            typename Op::Row& r) {
  if constexpr (has_row_s<Op>::value) Op::load_row_s(a, sc, i, r);
  else Op::load_row(a, i, r);
}
template <class Op>
__device__ __forceinline__ void op_load_col(const Args& a, const Scal& sc, int64_t j, float* rec) {
  if constexpr (has_col_s<Op>::value) Op::load_col_s(a, sc, j, rec);
  else Op::load_col(a, j, rec);
}

template <int W>
struct Vec {
  float v[W];
};

// ------------------------------------------------------------------------------------
// Generic tiled row-reduction kernel.
//   Op::D, Op::CW4 (float4 per column record), Op::NACC (accumulators per row)
//   Op::Row                        -- per-row state (registers)
//   Op::load_row(args, i, Row&)    -- read row i
//   Op::load_col(args, j, float* rec)  -- write column j's record (CW4*4 floats) into LDS
//   Op::pair(const Scal&, const Row&, const float* rec, float* acc)
//   Op::store(const Scal&, const Row&, const float* tot, float* vals) -> per-output values;
//       vals laid out as the concatenation of the outputs' widths Op::kOutW[0..kNOut).
//   Op::kMin -> accumulate by min instead of sum.
// ------------------------------------------------------------------------------------
template <class Op, int R>
__global__ __launch_bounds__(kBlock) DICP_KERNEL_ATTR void rowred_kernel(Args args, Scal sc,
                                                        int64_t M, int64_t N, int64_t chunk,
                                                        Outs outs) {
  constexpr int CW4 = Op::CW4;
  constexpr int NACC = Op::NACC;
  constexpr bool MIN = Op::kMin;
  // double-buffered column tiles: the global loads of tile t+1 are in flight while tile t
  // is consumed from LDS; one barrier per tile.
  __shared__ float4 lds[2][kTile * CW4];
  if (sc.dev0 != nullptr) sc.aux0 = sc.dev0[0];  // device-resident scalar (no host sync)
  // ops flagged kSkipOnAux0 treat that device scalar as a "skip this launch" flag (iterative
  // solvers launch ahead of their convergence test).  Kept out of Scal on purpose: one more
  // kernel argument changed the register allocation of unrelated kernels (~12% on the VJP).
  if constexpr (skip_on_aux0<Op>::value) {
    if (sc.aux0 != 0.f) return;
  }

  const int tid = threadIdx.x;
  const int64_t ibase = (int64_t)blockIdx.x * (kBlock * R) + tid;

  typename Op::Row row[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    int64_t i = ibase + (int64_t)r * kBlock;
    if (i >= M) i = M - 1;
    op_load_row<Op>(args, sc, i, row[r]);
  }

  float tot[R][NACC];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int k = 0; k < NACC; ++k) tot[r][k] = MIN ? __builtin_huge_valf() : 0.f;

  const int64_t j0 = (int64_t)blockIdx.y * chunk;
  int64_t j1 = j0 + chunk;
  if (j1 > N) j1 = N;

  float pre[CW4 * 4];
  int cnt = (int)((j1 - j0) < kTile ? (j1 - j0) : kTile);
  if (cnt > 0 && tid < cnt) {
    op_load_col<Op>(args, sc, j0 + tid, pre);
#pragma unroll
    for (int k = 0; k < CW4; ++k)
      lds[0][tid * CW4 + k] = make_float4(pre[4 * k], pre[4 * k + 1], pre[4 * k + 2], pre[4 * k + 3]);
  }
  __syncthreads();
  int buf = 0;
  for (int64_t jt = j0; jt < j1; jt += kTile) {
    const int64_t jn = jt + kTile;
    const int cntn = jn < j1 ? (int)((j1 - jn) < kTile ? (j1 - jn) : kTile) : 0;
#if DICP_STAGE_EARLY
    // stage the next tile straight into the free LDS buffer (its previous contents were
    // consumed before the last barrier): the staging registers die before the pair loop,
    // which lowers the loop's VGPR peak; the global-load latency is exposed once per tile
    // per wave and overlapped by the other resident waves.
    if (tid < cntn) {
      op_load_col<Op>(args, sc, jn + tid, pre);
#pragma unroll
      for (int k = 0; k < CW4; ++k)
        lds[buf ^ 1][tid * CW4 + k] =
            make_float4(pre[4 * k], pre[4 * k + 1], pre[4 * k + 2], pre[4 * k + 3]);
    }
#else
    if (tid < cntn) op_load_col<Op>(args, sc, jn + tid, pre);  // prefetch next tile (registers)
#endif

    float acc[R][NACC];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int k = 0; k < NACC; ++k) acc[r][k] = MIN ? __builtin_huge_valf() : 0.f;
    const float4* tile = lds[buf];
#pragma unroll DICP_PAIR_UNROLL
    for (int t = 0; t < cnt; ++t) {
      float rec[CW4 * 4];
#pragma unroll
      for (int k = 0; k < CW4; ++k) {
        const float4 q = tile[t * CW4 + k];
        rec[4 * k + 0] = q.x;
        rec[4 * k + 1] = q.y;
        rec[4 * k + 2] = q.z;
        rec[4 * k + 3] = q.w;
      }
#pragma unroll
      for (int r = 0; r < R; ++r) Op::pair(sc, row[r], rec, acc[r]);
    }
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int k = 0; k < NACC; ++k)
        tot[r][k] = MIN ? fminf(tot[r][k], acc[r][k]) : tot[r][k] + acc[r][k];
#if !DICP_STAGE_EARLY
    if (tid < cntn) {
#pragma unroll
      for (int k = 0; k < CW4; ++k)
        lds[buf ^ 1][tid * CW4 + k] =
            make_float4(pre[4 * k], pre[4 * k + 1], pre[4 * k + 2], pre[4 * k + 3]);
    }
#endif
    __syncthreads();
    buf ^= 1;
    cnt = cntn;
  }

  const bool split = gridDim.y > 1;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int64_t i = ibase + (int64_t)r * kBlock;
    if (i >= M) continue;
    float vals[Op::kOutW[0] + Op::kOutW[1] + Op::kOutW[2] + Op::kOutW[3]];
    Op::store(sc, row[r], tot[r], vals);
    int off = 0;
#pragma unroll
    for (int k = 0; k < Op::kNOut; ++k) {
      const int w = Op::kOutW[k];
      float* base = outs.ptr[k];
      if (base != nullptr) {
        if (split) {
          float* dst = base + (int64_t)blockIdx.y * M * w + i * w;
#pragma unroll
          for (int e = 0; e < w; ++e) dst[e] = vals[off + e];
        } else {
#pragma unroll
          for (int e = 0; e < w; ++e) base[i * w + e] = epilogue(outs, k, i * w + e, vals[off + e]);
        }
      }
      off += w;
    }
  }
}

// Fixed-order merge of split partial slabs, a = sum_{s<S} slab[s][e] (or min), then the
// Outs epilogue, for up to 4 outputs in ONE launch (blockIdx.y = output index k; the
// slab of output k starts at slab[k]).
struct MergeSet {
  const float* slab[4];
  int64_t n[4];
  int k[4];  // output index in Outs
};

template <bool MIN>
__device__ __forceinline__ void merge_slabs_body(const MergeSet& m, const Outs& o, int S, unsigned bx, unsigned by) {
  const int j = by;
  const int64_t n = m.n[j];
  const int64_t e = (int64_t)bx * kBlock + threadIdx.x;
  if (e >= n) return;
  const float* __restrict__ slab = m.slab[j];
  float a = slab[e];
  for (int s = 1; s < S; ++s) {
    const float b = slab[(int64_t)s * n + e];
    a = MIN ? fminf(a, b) : a + b;
  }
  const int k = m.k[j];
  o.ptr[k][e] = epilogue(o, k, e, a);
}

template <bool MIN>
__global__ __launch_bounds__(kBlock) void merge_slabs_kernel(MergeSet m, Outs o, int S) {
  merge_slabs_body<MIN>(m, o, S, blockIdx.x, blockIdx.y);
}

// Slabs of double partials (the eta != 0 forward's, packed.hpp rowred_pk_body_f64): summed in
// double in slab order, the epilogue formed in double, rounded once.
__device__ __forceinline__ void merge_slabs_f64_body(const MergeSet& m, const Outs& o, int S, unsigned bx, unsigned by) {
  const int j = by;
  const int64_t n = m.n[j];
  const int64_t e = (int64_t)bx * kBlock + threadIdx.x;
  if (e >= n) return;
  const double* __restrict__ slab = reinterpret_cast<const double*>(m.slab[j]);
  double a = slab[e];
  for (int s = 1; s < S; ++s) a += slab[(int64_t)s * n + e];
  const int k = m.k[j];
  double v = (double)o.alpha[k] * a;
  if (o.base[k]) v += (double)o.base[k][e];
  if (o.add[k]) v += (double)o.add[k][e];
  if (o.accumulate[k]) v += (double)o.ptr[k][e];
  o.ptr[k][e] = (float)v;
}

template <int I = 0>   // a template: defined in a header included by several objects
__global__ __launch_bounds__(kBlock) void merge_slabs_f64_kernel(MergeSet m, Outs o, int S) {
  merge_slabs_f64_body(m, o, S, blockIdx.x, blockIdx.y);
}

// batched form (batch.hpp): blockIdx.z = the recorded call
struct MergeEntry {
  MergeSet m;
  Outs o;
  int S;
  unsigned gx, gy;
  int f64;   // double slabs (merge_slabs_f64_body)
};
template <bool MIN>
__global__ __launch_bounds__(kBlock) void merge_slabs_batch_kernel(BatchTab<MergeEntry> t) {
  const MergeEntry& e = t.e[blockIdx.z];
  if (blockIdx.x >= e.gx || blockIdx.y >= e.gy) return;
  if (e.f64)
    merge_slabs_f64_body(e.m, e.o, e.S, blockIdx.x, blockIdx.y);
  else
    merge_slabs_body<MIN>(e.m, e.o, e.S, blockIdx.x, blockIdx.y);
}
inline int merge_slabs_batch_flush(const std::vector<const void*>& es, hipStream_t st) {
  return batch_launch<MergeEntry>(merge_slabs_batch_kernel<false>, es, st, "merge_slabs");
}

}  // namespace dicp
