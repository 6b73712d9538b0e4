// Launch batching (dicp_batch_begin / dicp_batch_end, include/difficp_hip.h): between the two
// calls, the batchable entry points of the calling host thread record their kernel launches
// instead of issuing them; dicp_batch_end issues them grouped -- all calls' first launches
// (their main pair kernels), then all second launches (their merges), ... -- with one batched
// launch per kernel instantiation, blockIdx.z indexing the calls (up to kBatchMax per launch).
//
// Why: the groupwise atlas optimises many independent frames of ~20k points (PSR.py:528-569);
// one frame's pass is too small to keep 256 CUs busy to the end (tails, launch gaps).  A
// batched launch is one grid over all the frames' blocks.  Every call keeps its own geometry
// (splits, column groups, rows per thread), arguments and workspace, so each call computes
// bitwise what it computes alone.
//
// Contract: the calls recorded in one batch must be independent (no call reads what another
// writes); each call's own launches keep their order (stage by stage).  A call whose path
// launches a kernel that has no batched form fails the batch (dicp_batch_end returns
// DICP_ERR_UNSUPPORTED and nothing of the batch runs).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <memory>
#include <vector>

#include "../../include/difficp_hip.h"

namespace dicp {

void set_error(const char* fmt, ...);

constexpr int kBatchMax = 12;   // calls per batched launch (kernel-argument table <= ~3.3 KB)

// A kernel-argument table: the per-call entries of one batched launch.
template <class E>
struct BatchTab {
  E e[kBatchMax];
  int n;
};

using BatchFlush = int (*)(const std::vector<const void*>& entries, hipStream_t st);

struct BatchItem {
  BatchFlush flush;               // batched launcher of this kernel instantiation (group key)
  std::shared_ptr<void> entry;    // its argument entry
};

struct Recorder {
  std::vector<std::vector<BatchItem>> calls;   // per recorded entry-point call: its launches
  int depth = 0;                               // nesting of entry points (outermost = a call)
  int unchecked = 0;                           // launches recorded since the last check_launch
  bool failed = false;
};

extern thread_local Recorder* tl_batch;

// PER HOST THREAD geometry hint (dicp_set_option "batch_share", default 1): the number of
// equal-sized calls a launch shares the device with (the frames of a lockstep batch).  The
// geometry rules then size each call for 1/share of the chip -- fewer column splits, more
// column groups per workgroup, the 4-row forms where the BATCH is large enough -- which
// changes only the fp32 summation order (a call made with the same share alone computes the
// same bits).  Workspace sizes are always those of share 1 (the largest).
extern thread_local int tl_batch_share;
inline int batch_share() { return tl_batch_share > 1 ? tl_batch_share : 1; }

// Entry-point guard: the outermost batchable entry point of a call opens a new lane.
struct BatchCall {
  BatchCall() {
    if (tl_batch && tl_batch->depth++ == 0) tl_batch->calls.emplace_back();
  }
  ~BatchCall() {
    if (tl_batch) --tl_batch->depth;
  }
};

inline bool batching() { return tl_batch != nullptr; }

template <class E>
int batch_record(BatchFlush flush, const E& e) {
  if (tl_batch->calls.empty() || tl_batch->depth == 0) {
    tl_batch->failed = true;
    set_error("dicp batch: a launch outside a batchable entry point");
    return DICP_ERR_UNSUPPORTED;
  }
  tl_batch->calls.back().push_back(BatchItem{flush, std::make_shared<E>(e)});
  ++tl_batch->unchecked;
  return DICP_OK;
}

// check_launch inside a batch: every launch must have been recorded -- a kernel launched
// directly (a path without a batched form) fails the batch
inline int batch_check(const char* what) {
  if (tl_batch->unchecked > 0) {
    tl_batch->unchecked = 0;
    return DICP_OK;
  }
  tl_batch->failed = true;
  set_error("%s: no batched form of this launch (dicp batch)", what);
  return DICP_ERR_UNSUPPORTED;
}

// A launch helper without a batched form, called inside a batch: fail the batch before
// launching anything (nothing of the batch is issued).
inline int no_batch(const char* what) {
  if (tl_batch == nullptr) return DICP_OK;
  tl_batch->failed = true;
  set_error("%s: no batched form of this launch (dicp batch)", what);
  return DICP_ERR_UNSUPPORTED;
}

// Launch `kernel` over the entries in tables of kBatchMax; the grid covers the largest entry
// (gx, gy fields), blocks beyond an entry's own grid return at once.
template <class E, class K>
int batch_launch(K kernel, const std::vector<const void*>& entries, hipStream_t st, const char* what) {
  for (size_t i0 = 0; i0 < entries.size(); i0 += kBatchMax) {
    BatchTab<E> t;
    memset(&t, 0, sizeof(t));
    t.n = (int)((entries.size() - i0) < (size_t)kBatchMax ? entries.size() - i0 : kBatchMax);
    unsigned gx = 1, gy = 1;
    for (int j = 0; j < t.n; ++j) {
      t.e[j] = *static_cast<const E*>(entries[i0 + j]);
      gx = t.e[j].gx > gx ? t.e[j].gx : gx;
      gy = t.e[j].gy > gy ? t.e[j].gy : gy;
    }
    kernel<<<dim3(gx, gy, (unsigned)t.n), dim3(256), 0, st>>>(t);
    const hipError_t err = hipGetLastError();
    if (err != hipSuccess) {
      set_error("%s (batched): %s", what, hipGetErrorString(err));
      return DICP_ERR_HIP;
    }
  }
  return DICP_OK;
}

}  // namespace dicp
