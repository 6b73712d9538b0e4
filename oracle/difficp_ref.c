/*
 * ORACLE -- test / CPU-baseline infrastructure only (never linked into the product).
 *
 * Plain-C (OpenMP over rows, double accumulation) restatement of the reference's hot-path
 * arithmetic (AdrienWohrer/diff-icp, torch path), written directly from the formulas:
 *   - LDDMM ODE right-hand side on the support points, eta = 0 (LDDMM.py:176-227):
 *       v = KRed(q,q,p) (kernel.py:186), Gq = GenDKRed(q,q,p,p) (kernel.py:202),
 *       g_i = p_i . GradKRed(q,q)_i (mdivsum terms, LDDMM.py:138)
 *   - its vector-Jacobian product (what autograd computes through the torch path at
 *     optim.py:46), hand-derived; pinned by tests against torch autograd of oracle/torch_ref.py
 *   - the GMM E-step log-normaliser T_n = LSE_c t_nc (GMM.py:263-270) and sum_c gamma D2.
 * Used for (1) large-size spot checks where the dense torch oracle is too slow and
 * (2) bench.py's cpu_baseline leg ("kind": "port").
 */
#include <math.h>
#include <stdint.h>

void oracle_ode_self_fwd(const float* q, const float* p, int64_t M, int D, double sigma,
                         float* v, float* mG, float* g) {
  const double s = 1.0 / (sigma * sigma);
#pragma omp parallel for schedule(dynamic, 64)
  for (int64_t i = 0; i < M; ++i) {
    double V[8] = {0}, Z[8] = {0}, G[8] = {0};
    for (int64_t j = 0; j < M; ++j) {
      double z[8], r2 = 0, pp = 0;
      for (int d = 0; d < D; ++d) {
        z[d] = (double)q[i * D + d] - q[j * D + d];
        r2 += z[d] * z[d];
        pp += (double)p[i * D + d] * p[j * D + d];
      }
      const double K = exp(-0.5 * s * r2);
      for (int d = 0; d < D; ++d) {
        V[d] += K * p[j * D + d];
        Z[d] += K * z[d];
        G[d] += K * pp * z[d];
      }
    }
    double gi = 0;
    for (int d = 0; d < D; ++d) {
      v[i * D + d] = (float)V[d];
      mG[i * D + d] = (float)(s * G[d]);
      gi += -s * p[i * D + d] * Z[d];
    }
    if (g) g[i] = (float)gi;
  }
}

void oracle_ode_self_bwd(const float* q, const float* p, const float* a, const float* b,
                         double gam, int64_t M, int D, double sigma, float* gq, float* gp) {
  const double s = 1.0 / (sigma * sigma);
#pragma omp parallel for schedule(dynamic, 64)
  for (int64_t m = 0; m < M; ++m) {
    double GP[8] = {0}, GQ[8] = {0};
    for (int64_t j = 0; j < M; ++j) {
      double z[8], db[8], dp[8], r2 = 0, pp = 0, ap = 0, zb = 0, zp = 0;
      for (int d = 0; d < D; ++d) {
        z[d] = (double)q[m * D + d] - q[j * D + d];
        db[d] = (double)b[m * D + d] - b[j * D + d];
        dp[d] = (double)p[m * D + d] - p[j * D + d];
        r2 += z[d] * z[d];
        pp += (double)p[m * D + d] * p[j * D + d];
        ap += (double)a[m * D + d] * p[j * D + d] + (double)a[j * D + d] * p[m * D + d];
      }
      for (int d = 0; d < D; ++d) {
        zb += z[d] * db[d];
        zp += z[d] * dp[d];
      }
      const double K = exp(-0.5 * s * r2);
      const double w = s * (gam * zp - pp * zb) - ap;
      for (int d = 0; d < D; ++d) {
        GP[d] += K * (a[j * D + d] + s * zb * p[j * D + d] - s * gam * z[d]);
        GQ[d] += K * (pp * db[d] - gam * dp[d] + w * z[d]);
      }
    }
    for (int d = 0; d < D; ++d) {
      gp[m * D + d] = (float)GP[d];
      gq[m * D + d] = (float)(s * GQ[d]);
    }
  }
}

void oracle_gmm_estep(const float* X, int64_t N, const float* mu, const float* w, int64_t C,
                      int D, double sigma, float* T, float* gD2) {
  double Zw = -INFINITY;
  for (int64_t c = 0; c < C; ++c) Zw = Zw > w[c] ? Zw + log1p(exp(w[c] - Zw)) : w[c] + log1p(exp(Zw - w[c]));
  const double lgn = D * (log(sigma) + 0.5 * log(2 * M_PI));
#pragma omp parallel for schedule(dynamic, 256)
  for (int64_t n = 0; n < N; ++n) {
    double mx = -INFINITY;
    for (int64_t c = 0; c < C; ++c) {
      double d2 = 0;
      for (int d = 0; d < D; ++d) {
        const double z = (double)X[n * D + d] - mu[c * D + d];
        d2 += z * z;
      }
      const double t = w[c] - Zw - d2 / (2 * sigma * sigma) - lgn;
      if (t > mx) mx = t;
    }
    double l = 0, acc = 0;
    for (int64_t c = 0; c < C; ++c) {
      double d2 = 0;
      for (int d = 0; d < D; ++d) {
        const double z = (double)X[n * D + d] - mu[c * D + d];
        d2 += z * z;
      }
      const double e = exp(w[c] - Zw - d2 / (2 * sigma * sigma) - lgn - mx);
      l += e;
      acc += e * d2;
    }
    T[n] = (float)(mx + log(l));
    if (gD2) gD2[n] = (float)(acc / l);
  }
}
