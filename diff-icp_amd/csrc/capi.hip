// C-ABI glue: thread-local error message, workspace sizing, version.
#include <stdarg.h>
#include <stdio.h>

#include <memory>
#include <utility>
#include <vector>

#include "launch.hpp"

size_t dicp_lddmm_ws(int kind, int64_t M, int64_t N, int D);
int dicp_lddmm_splits(int kind, int64_t M, int64_t N);
size_t dicp_gmm_ws(int kind, int64_t M, int64_t N, int D);
size_t dicp_solve_ws(int kind, int64_t M, int D);
size_t dicp_grad_ws(int64_t M, int64_t N, int D);

namespace {
thread_local char g_err[512] = "";
}

namespace dicp {
thread_local Recorder* tl_batch = nullptr;
thread_local int tl_batch_share = 1;

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace dicp

extern "C" const char* dicp_last_error(void) { return g_err; }

extern "C" const char* dicp_version(void) {
  return "difficp_hip 0.1 (gfx950; ops: gauss_red x13 (centred / packed KRed), ode_self fwd/bwd, "
         "ode_ext fwd/bwd (centred / packed), gmm estep/mstep/targets, kernel ridge CG, "
         "reduction gradients x5)";
}

extern "C" size_t dicp_workspace_bytes(int kind, int64_t M, int64_t N, int D) {
  // sized for share 1: the most splits / slots any geometry hint can ask for
  struct ShareOne {
    int saved = dicp::tl_batch_share;
    ShareOne() { dicp::tl_batch_share = 1; }
    ~ShareOne() { dicp::tl_batch_share = saved; }
  } one;
  size_t b = 0;
  if (kind == DICP_WS_GRAD)
    b = dicp_grad_ws(M, N, D);
  else if (kind == DICP_WS_RIDGE_CG)
    b = dicp_solve_ws(kind, M, D);
  else if (kind >= DICP_WS_GMM_ESTEP && kind <= DICP_WS_GMM_TARGETS)
    b = dicp_gmm_ws(kind, M, N, D);
  else
    b = dicp_lddmm_ws(kind, M, N, D);
  // 256-byte granule so callers can cache by size class
  return (b + 255) / 256 * 256;
}

extern "C" int dicp_num_splits(int kind, int64_t M, int64_t N) {
  return dicp_lddmm_splits(kind, M, N);
}

// Launch batching (batch.hpp): record the calling thread's batchable launches ...
extern "C" int dicp_batch_begin(void) {
  if (dicp::tl_batch != nullptr) {
    dicp::set_error("dicp_batch_begin: a batch is already open on this thread");
    return DICP_ERR_INVALID;
  }
  dicp::tl_batch = new dicp::Recorder();
  return DICP_OK;
}

// ... and issue them grouped: stage by stage (every call's k-th launch), one batched launch
// per kernel instantiation and stage (in first-appearance order), on `stream`.
extern "C" int dicp_batch_end(dicp_stream_t stream) {
  std::unique_ptr<dicp::Recorder> rec(dicp::tl_batch);
  dicp::tl_batch = nullptr;
  if (!rec) {
    dicp::set_error("dicp_batch_end: no open batch on this thread");
    return DICP_ERR_INVALID;
  }
  if (rec->failed) return DICP_ERR_UNSUPPORTED;   // the message was set by the failing call
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  size_t nstage = 0;
  for (const auto& c : rec->calls) nstage = c.size() > nstage ? c.size() : nstage;
  for (size_t s = 0; s < nstage; ++s) {
    std::vector<std::pair<dicp::BatchFlush, std::vector<const void*>>> groups;
    for (const auto& c : rec->calls) {
      if (s >= c.size()) continue;
      const dicp::BatchItem& it = c[s];
      size_t g = 0;
      while (g < groups.size() && groups[g].first != it.flush) ++g;
      if (g == groups.size()) groups.emplace_back(it.flush, std::vector<const void*>());
      groups[g].second.push_back(it.entry.get());
    }
    for (const auto& g : groups) {
      const int rc = g.first(g.second, st);
      if (rc) return rc;
    }
  }
  return DICP_OK;
}

// Discard an open batch (nothing recorded runs); no-op without one.
extern "C" int dicp_batch_abort(void) {
  delete dicp::tl_batch;
  dicp::tl_batch = nullptr;
  return DICP_OK;
}
