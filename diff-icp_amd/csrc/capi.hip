// C-ABI glue: thread-local error message, workspace sizing, version.
#include <stdarg.h>
#include <stdio.h>

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
