/*
 * difficp_hip.h -- C-ABI of the MI355X (gfx950) hot path of diff-ICP.
 *
 * This library replaces the KeOps-generated (JIT CUDA) reductions that the reference
 * binds at two seams:
 *   - GenKernel.set_computversion (diffICP/tools/kernel.py:91-110) which binds the ten
 *     Gaussian-kernel reductions KBase ... GradKRed_rev (kernel.py:127-168 KeOps formulas,
 *     :177-215 torch restatement);
 *   - GaussianMixtureUnif.set_computversion (diffICP/core/GMM.py:126-144) which binds
 *     EM_step (torch: GMM.py:236-325, KeOps: GMM.py:402-529).
 * plus the LDDMM ODE right-hand side that the reference builds from those reductions
 * (LDDMMModel.ODE, diffICP/core/LDDMM.py:176-227) and its autograd backward
 * (optim.py:46 `L.backward()`), which the reference gets from KeOps autodiff.
 *
 * Conventions (all entry points):
 *   - every pointer is a caller-owned DEVICE buffer, row-major float32, contiguous;
 *   - nothing is allocated inside; scratch space is passed in `ws` (size from
 *     dicp_workspace_bytes) -- the call is hipGraph-capturable;
 *   - every call is stream-ordered on `stream` and never synchronises the host;
 *   - return 0 on success, else a nonzero code; dicp_last_error() gives a message
 *     (thread-local).  Unsupported D or op -> DICP_ERR_UNSUPPORTED.
 *   - results are deterministic: no float atomics; split-column partial sums are
 *     reduced in a fixed order.
 *
 * Notation: i = row ("target", KeOps Vi), j = column ("source", KeOps Vj);
 *   z = x_i - y_j,  K = exp(-|z|^2 / (2 sigma^2)),  s = 1/sigma^2.
 */
#ifndef DIFFICP_HIP_H
#define DIFFICP_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* dicp_stream_t; /* a hipStream_t (NULL = legacy default stream) */

enum dicp_status {
  DICP_OK = 0,
  DICP_ERR_INVALID = 1,     /* bad sizes / null pointers */
  DICP_ERR_UNSUPPORTED = 2, /* D or op not compiled in */
  DICP_ERR_WORKSPACE = 3,   /* ws too small */
  DICP_ERR_HIP = 4          /* a HIP launch error (message has hipGetErrorString) */
};

/* ------------------------------------------------------------------------------------
 * Gaussian-kernel reductions (GenKernel aliases, kernel.py:100-107).
 * ---------------------------------------------------------------------------------- */
enum dicp_red_op {
  DICP_KBASE = 0,      /* out_i   = sum_j K                          (M,)  kernel.py:131,178 */
  DICP_KREDSCAL = 1,   /* out_i   = sum_j K d_j        b=d (N,)      (M,)  kernel.py:135,182 */
  DICP_KRED = 2,       /* out_i   = sum_j K b_j        b (N,D)       (M,D) kernel.py:138,186 */
  DICP_GRADK = 3,      /* out_i   = sum_j -s z K                     (M,D) kernel.py:142,190 */
  DICP_GRADK_REV = 4,  /* out_j   = sum_i grad K(x_i-y_j).d_i; call with (x=y_rows, y=x_cols,
                          b=d (N,D)); computes out_i = sum_j s (z.b_j) K  (M,) kernel.py:147,194 */
  DICP_DDK = 5,        /* out_i^d = sum_j -s z^d K b_j^d             (M,D) kernel.py:151,198 */
  DICP_GENDK = 6,      /* out_i   = sum_j -s z K (c_i.b_j)  c (M,D)  (M,D) kernel.py:155,202 */
  DICP_HESSK = 7,      /* out_i   = sum_j [s^2 (z.u) z - s u] K, u=c_i-b_j (M,D) kernel.py:160,284 */
  DICP_LAPK = 8,       /* out_i   = sum_j (s^2|z|^2 - D s) K         (M,)  kernel.py:164,206 */
  DICP_GRADLAPK = 9,   /* out_i   = sum_j -z (s^3|z|^2-(D+2)s^2) K   (M,D) kernel.py:168,289 */
  DICP_GRADKSCAL = 10, /* out_i   = sum_j -s z K d_j    b=d (N,)     (M,D) (autograd of KBase/KRedScal) */
  DICP_GRADLAPKSCAL = 11, /* out_i = sum_j -z (s^3|z|^2-(D+2)s^2) K d_j (M,D) (autograd of LapKRed) */
  DICP_MIN_SQDIST = 12, /* out_i  = min_j |z|^2                      (M,)  check_coverage kernel.py:324-329 */
  DICP_MIN_SQDIST_OTHER = 13 /* out_i = min_{j != i} |z|^2, x == y, M == N (M,)  intrinsic_scale
                          point_sets.py:13-26 (Kmin(2)[:,1]); sigma unused */
};
/* MIN_SQDIST, MIN_SQDIST_OTHER and dicp_radius_count_f32 compute |z|^2 with the torch CPU
 * arithmetic of ((x_i - y_j)**2).sum(-1) (no FMA contraction), so threshold decisions are
 * bit-identical to the reference's. */

/* One reduction.  x (M,D) rows, y (N,D) columns, b column weights ((N,D) or (N,) or NULL),
 * c row weights ((M,D) or NULL), out (M,D) or (M,) as listed above.
 * Replaces the bound aliases GK.KBase ... GK.GradKRed_rev (kernel.py:100-107). */
int dicp_gauss_red_f32(int op, const float* x, int64_t M, const float* y, int64_t N, int D,
                       const float* b, const float* c, double sigma, float* out, void* ws,
                       size_t ws_bytes, dicp_stream_t stream);

/* counts_i = #{j < N : |x_i - y_j|^2 <= (float)(R*R)}, x (M,D), y (N,D), counts (M,) float
 * (exact integers below 2^24).  The O(N^2) part of the greedy support decimation
 * decimate(x, R) (point_sets.py:102-133); workspace kind DICP_WS_RED. */
int dicp_radius_count_f32(const float* x, int64_t M, const float* y, int64_t N, int D, double R,
                          float* counts, void* ws, size_t ws_bytes, dicp_stream_t stream);

/* ------------------------------------------------------------------------------------
 * LDDMM geodesic-shooting ODE (LDDMMModel.ODE, LDDMM.py:176-227), fused: one pass over
 * the M x M support pairs produces every self-interaction term with one exp per pair.
 *   v_i   = sum_j K p_j - eta grad K                                  (LDDMM.py:100-116)
 *   mG_i  = -(GenDKRed(q,q,p,p) - eta HessKRed - eta^2 GradLapKRed)   (LDDMM.py:198-203)
 *           (the ODE returns -Gq, so mG is exactly dp/dt)
 *   g_i   = p_i . GradKRed(q,q)_i + eta LapKRed(q,q)_i  (per-row terms of mdivsum, LDDMM.py:133-138;
 *           sum_i g_i = mdivsum(q,q,p))
 *   h_i   = per-row terms of the Hamiltonian (LDDMM.py:150-155); sum_i h_i = H(q,p)
 * g and h may be NULL (not computed).  eta = 0 (classic/hybrid) or 1/lambda (logdet).
 * ---------------------------------------------------------------------------------- */
int dicp_lddmm_ode_self_fwd_f32(const float* q, const float* p, int64_t M, int D, double sigma,
                                double eta, float* v, float* mG, float* g, float* h, void* ws,
                                size_t ws_bytes, dicp_stream_t stream);

/* Vector-Jacobian product of the fused self ODE (what KeOps autodiff provides at
 * optim.py:46).  Cotangents: gv (M,D) on v, gmG (M,D) on mG, and gdiv = cotangent of
 * sum_i g_i, a DEVICE scalar (may be NULL = 0).  Outputs gq, gp (M,D), overwritten; gq may be
 * NULL (gp only: with the default symmetric packed kernels -- both models -- the gq half of the
 * pair algebra, about half of it, is then skipped).  gmG may be NULL = a zero cotangent (with
 * the default symmetric packed kernels; eta != 0 with another "bwd_eta_alg": DICP_ERR_INVALID). */
int dicp_lddmm_ode_self_bwd_f32(const float* q, const float* p, const float* gv,
                                const float* gmG, const float* gdiv, int64_t M, int D,
                                double sigma, double eta, float* gq, float* gp, void* ws,
                                size_t ws_bytes, dicp_stream_t stream);

/* One explicit-Euler step with the state update fused into the pass's epilogue
 * (integrators.py:20-33 EulerIntegrator over LDDMMModel.ODE, LDDMM.py:176-227):
 *   q_next = q + dt v(q,p),  p_next = p + dt mG(q,p),  g (M,) as above or NULL.
 * Outputs must not alias inputs.  Workspace kind DICP_WS_ODE_SELF_FWD. */
int dicp_lddmm_euler_step_f32(const float* q, const float* p, int64_t M, int D, double sigma,
                              double eta, double dt, float* q_next, float* p_next, float* g,
                              void* ws, size_t ws_bytes, dicp_stream_t stream);

/* Its exact discrete adjoint (the reverse sweep of optim.py:46's backward through the Euler
 * loop): with (gq, gp) the VJP of dicp_lddmm_ode_self_bwd_f32 for cotangents (lq, lp, gdiv),
 *   lq_next = lq + dt gq + addq,  lp_next = lp + dt gp + addp   (addq/addp (M,D) or NULL).
 * lq_next may be NULL (the last step of a sweep whose start points q0 need no gradient:
 * only lp_next, with the gq half skipped as above).  lp may be NULL = a zero cotangent on the
 * momenta (the first step of a sweep whose loss does not depend on the final momenta; as gmG
 * above): the terms of the VJP in it are then skipped.
 * Outputs must not alias inputs.  Workspace kind DICP_WS_ODE_SELF_BWD. */
int dicp_lddmm_euler_adjoint_step_f32(const float* q, const float* p, const float* lq,
                                      const float* lp, const float* gdiv, int64_t M, int D,
                                      double sigma, double eta, double dt, const float* addq,
                                      const float* addp, float* lq_next, float* lp_next,
                                      void* ws, size_t ws_bytes, dicp_stream_t stream);

/* External data points x (N,D) carried by the flow (LDDMM.py:219-227):
 *   vx_i = v(x_i) (LDDMM.py:226), gx_i = per-row terms of mdivsum(x,q,p) (LDDMM.py:223),
 *   summed in row (x) order; gx may be NULL. */
int dicp_lddmm_ode_ext_fwd_f32(const float* x, int64_t N, const float* q, const float* p,
                               int64_t M, int D, double sigma, double eta, float* vx, float* gx,
                               void* ws, size_t ws_bytes, dicp_stream_t stream);

/* VJP of the external-point terms.  Cotangents gvx (N,D) on vx and device scalar gdiv on
 * sum_i gx_i.  Writes gxo (N,D) (gradient w.r.t. x) and ACCUMULATES into gq, gp (M,D)
 * (gradient w.r.t. the support points / momenta), so it can follow the self backward. */
int dicp_lddmm_ode_ext_bwd_f32(const float* x, int64_t N, const float* q, const float* p,
                               int64_t M, int D, double sigma, double eta, const float* gvx,
                               const float* gdiv, float* gxo, float* gq, float* gp, void* ws,
                               size_t ws_bytes, dicp_stream_t stream);

/* ------------------------------------------------------------------------------------
 * Row-split of ONE frame over ranks (C2/C3 two-set matches across GPUs).
 * The reference has no multi-device path; these split LDDMMModel.ODE (LDDMM.py:176-227) and
 * its VJP (optim.py:46) so that every rank holds the full (q, p) (M x 2D floats), computes a
 * slice, and the host exchanges O(M) floats per ODE evaluation (all-gather of the forward
 * slices, all-reduce of the VJP parts).
 * ---------------------------------------------------------------------------------- */

/* Rows [row0, row0 + nrows) of dicp_lddmm_ode_self_fwd_f32 against all M columns; v, mG
 * (nrows, D), g, h (nrows,) address the slice.  Workspace kind DICP_WS_ODE_SELF_FWD_ROWS
 * (M = nrows, N = M). */
int dicp_lddmm_ode_self_fwd_rows_f32(const float* q, const float* p, int64_t M, int64_t row0,
                                     int64_t nrows, int D, double sigma, double eta, float* v,
                                     float* mG, float* g, float* h, void* ws, size_t ws_bytes,
                                     dicp_stream_t stream);

/* Rows [row0, row0 + nrows) of dicp_lddmm_euler_step_f32: q_next = q[rows] + dt v(rows),
 * p_next = p[rows] + dt mG(rows), g (nrows,) or NULL.  Same workspace kind as above. */
int dicp_lddmm_euler_step_rows_f32(const float* q, const float* p, int64_t M, int64_t row0,
                                   int64_t nrows, int D, double sigma, double eta, double dt,
                                   float* q_next, float* p_next, float* g, void* ws,
                                   size_t ws_bytes, dicp_stream_t stream);

/* General forms of the four forward entry points above: rows [row0, row0 + nrows) against
 * all M columns, the rows visited in `row_order` (nrows int32 indices into the slice, a
 * permutation of 0..nrows-1; NULL = natural order).  Outputs are indexed like the plain
 * forms (by row, not by visit order), so the order never changes WHAT is computed, only which
 * rows share a workgroup: the matrix-core forward (fwd_alg 3) centres the column channels on
 * its workgroup's rows, and its fp32 error grows with their spread, so a spatial order (e.g.
 * Morton, _lib.spatial_order) keeps it at the ordered-pair kernels' level for any cloud extent.
 * No reference counterpart (KeOps has no row grouping to choose).  In the Euler form p_next
 * may be NULL: the momentum update is then not formed (the packed pass skips the sums that feed
 * mG only: Gs', and for eta != 0 Hs and GL') -- the last step of a shooting whose final
 * momenta are not used. */
int dicp_lddmm_ode_self_fwd_ord_f32(const float* q, const float* p, int64_t M, int64_t row0,
                                    int64_t nrows, int D, double sigma, double eta,
                                    const int32_t* row_order, float* v, float* mG, float* g,
                                    float* h, void* ws, size_t ws_bytes, dicp_stream_t stream);
int dicp_lddmm_euler_step_ord_f32(const float* q, const float* p, int64_t M, int64_t row0,
                                  int64_t nrows, int D, double sigma, double eta, double dt,
                                  const int32_t* row_order, float* q_next, float* p_next,
                                  float* g, void* ws, size_t ws_bytes, dicp_stream_t stream);

/* Part `part` of `nparts` of dicp_lddmm_ode_self_bwd_f32: gq, gp (M, D) over a subset of
 * the pairs such that the SUM over the parts is the full VJP (eta = 0: the symmetric
 * kernel's quads Q = part mod nparts, every row touched; eta != 0: a row slice, other rows 0).
 * Workspace kind DICP_WS_ODE_SELF_BWD_PART (M, N = nparts). */
int dicp_lddmm_ode_self_bwd_part_f32(const float* q, const float* p, const float* gv,
                                     const float* gmG, const float* gdiv, int64_t M, int D,
                                     double sigma, double eta, int part, int nparts, float* gq,
                                     float* gp, void* ws, size_t ws_bytes, dicp_stream_t stream);

/* ------------------------------------------------------------------------------------
 * Divergence-row reuse (eta = 0, the hybrid / withlogdet model).  The divergence cotangent
 * gdiv enters the VJP's dL/dp only through the per-row sums
 *   zs_i = sum_j K(q_i - q_j) (q_i - q_j)     (= -sigma^2 GradKRed(q,q)_i, kernel.py:142;
 *                                              g_i = -p_i.zs_i / sigma^2, LDDMM.py:133-138)
 * (gp_i gets -gdiv zs_i / sigma^2), which the forward pass already forms.  The _zs forms let
 * the forward write them (original units) and the VJP take them: its pair loop then drops
 * those terms (the packed symmetric kernel: 90 instead of 120 packed instructions per 4
 * unordered pairs) and its merge adds -gdiv zs_i / sigma^2 once per row.  Same results as the
 * plain forms up to fp32 summation order.  No reference counterpart (KeOps autodiff
 * re-differentiates GradKRed pair by pair).
 * ---------------------------------------------------------------------------------- */

/* dicp_lddmm_euler_step_ord_f32 that also writes zs (nrows, D) of the slice's rows (NULL: not
 * formed, = the plain form).  zs needs eta = 0 and the packed ordered forward (fwd_alg 2;
 * DICP_ERR_INVALID otherwise). */
int dicp_lddmm_euler_step_zs_f32(const float* q, const float* p, int64_t M, int64_t row0,
                                 int64_t nrows, int D, double sigma, double eta, double dt,
                                 const int32_t* row_order, float* q_next, float* p_next,
                                 float* g, float* zs, void* ws, size_t ws_bytes,
                                 dicp_stream_t stream);

/* A row-split Euler step in two COLUMN PHASES (no reference counterpart: the reference has no
 * multi-device path; the step itself is LDDMM.py:194-227 + integrators.py:20-51).  Rows
 * [row0, row0 + nrows) of (q, p) (M points), 0 < nrows < M:
 *   phase 0: the rows against their own slice, given as (q_loc, p_loc) (nrows, D) -- the values
 *            a rank of a row split holds before the all-gather of the step's input (q, p) has
 *            landed; partial sums into the first slots of `ws` (outputs not written; q, p may
 *            be NULL);
 *   phase 1: the rows of (q, p) against the other M - nrows points (from row0 + nrows on,
 *            wrapping), into the remaining slots, then one merge of all slots with the Euler
 *            epilogue: q_next = q_row + dt v, p_next = p_row + dt mG, g, zs as
 *            dicp_lddmm_euler_step_zs_f32 of the slice (fp32 summation order and each phase's
 *            coordinate origin aside).
 * Both calls take the same sizes, the same output pointers (their NULL pattern selects the
 * pass: p_next NULL = no momentum update, g / zs NULL = not formed; zs needs eta = 0) and the
 * same `ws`, untouched in between, on one stream.  Outputs must not overlap (q, p) (they may
 * be the local slice's buffers: only phase 0 reads those).  Workspace kind DICP_WS_ODE_SELF_FWD_PHASED (M = nrows, N = M).  Ordered packed
 * forward only (fwd_alg 2, 5, 6; DICP_ERR_UNSUPPORTED otherwise).  Not batchable. */
int dicp_lddmm_euler_step_phase_f32(int phase, const float* q_loc, const float* p_loc, const float* q,
                                    const float* p, int64_t M, int64_t row0, int64_t nrows, int D,
                                    double sigma, double eta, double dt, float* q_next, float* p_next,
                                    float* g, float* zs, void* ws, size_t ws_bytes, dicp_stream_t stream);

/* dicp_lddmm_ode_self_fwd_ord_f32 with zs (nrows, D) in place of h (the first ODE evaluation of
 * a shooting: v, mG, g as the plain form, bitwise; H = sum_i p_i.v_i / 2 is then formed by the
 * caller).  Same requirements as above. */
int dicp_lddmm_ode_self_fwd_zs_f32(const float* q, const float* p, int64_t M, int64_t row0,
                                   int64_t nrows, int D, double sigma, double eta,
                                   const int32_t* row_order, float* v, float* mG, float* g,
                                   float* zs, void* ws, size_t ws_bytes, dicp_stream_t stream);

/* dicp_lddmm_euler_adjoint_step_f32 given zs (M, D) of the same q (NULL = the plain form).
 * zs needs eta = 0 and the packed symmetric VJP (bwd_alg 3, or lp = NULL). */
int dicp_lddmm_euler_adjoint_step_zs_f32(const float* q, const float* p, const float* lq,
                                         const float* lp, const float* gdiv, int64_t M, int D,
                                         double sigma, double eta, double dt, const float* addq,
                                         const float* addp, const float* zs, float* lq_next,
                                         float* lp_next, void* ws, size_t ws_bytes,
                                         dicp_stream_t stream);

/* dicp_lddmm_ode_self_bwd_part_f32 given the zs rows [zrow0, zrow0 + znrows) (a rank's forward
 * slice; NULL = the plain form): part `part` adds their -gdiv zs_i / sigma^2 term, so every
 * row's term is added once over the parts when the ranks' slices tile 0..M-1. */
int dicp_lddmm_ode_self_bwd_part_zs_f32(const float* q, const float* p, const float* gv,
                                        const float* gmG, const float* gdiv, int64_t M, int D,
                                        double sigma, double eta, int part, int nparts,
                                        const float* zs, int64_t zrow0, int64_t znrows, float* gq,
                                        float* gp, void* ws, size_t ws_bytes,
                                        dicp_stream_t stream);

/* ------------------------------------------------------------------------------------
 * GMM EM step reductions (GaussianMixtureUnif.EM_step_torch, GMM.py:236-325).
 * log2-domain internally; outputs in natural log.
 * ---------------------------------------------------------------------------------- */

/* The C-sized column vectors are precomputed by the caller on the device (they are
 * O(C) torch ops): w2_c = (w_c - LSE(w)) * log2(e), mu2_c = |mu_c|^2, lpi_c = w_c - LSE(w).
 * Internally logits are kept in the log2 domain: t2_nc = w2_c - |x_n-mu_c|^2 log2(e)/(2 sigma^2).
 *
 * E-step row pass over points n (rows X (N,D)) against components (mu (C,D)):
 *   T[n]  = LSE_c t_nc = ln2 * T2[n] - lgn,  lgn = D (log sigma + 0.5 log 2 pi)   (GMM.py:263-270)
 *   T2[n] = log2 sum_c 2^t2_nc  (consumed by the M-step and targets passes; may be NULL)
 * if stats != NULL also the responsibility-weighted row sums (gamma = exp(t - T)):
 *   stats[n*(D+4) + ...] = { sum_c gamma mu_c (D), sum_c gamma |mu_c|^2,
 *                            sum_c gamma lgamma, sum_c gamma lpi_c, sum_c gamma D2_nc }
 *   (Y with the current mu GMM.py:303; Cfe terms :312-314; NDsigma2 with the old mu :296). */
int dicp_gmm_estep_f32(const float* X, int64_t N, const float* mu, const float* w2,
                       const float* mu2, int64_t C, int D, double sigma, double lgn, float* T,
                       float* T2, float* stats, void* ws, size_t ws_bytes, dicp_stream_t stream);

/* The same E-step with an optional per-row shift hint (extension; NULL = dicp_gmm_estep_f32):
 * shift_hint[n] ~ the row's log2-domain LSE, e.g. the T2 of the previous EM step over the same
 * rows.  The single exp sweep shifts each row's terms by
 *     m = clamp(shift_hint[n] - 8, m64, m64 + 100),  m64 = max of the chunk's first 64 logits
 * instead of m64 alone, so a small sigma (nearest component far closer than any of a random
 * 64-column sample) no longer forces a re-referenced tile per record; any hint is safe (the
 * clamp), a good one makes re-referencing rare.  Results agree with the hint-less call to
 * float32 rounding (the shift is a change of reference, not an approximation). */
int dicp_gmm_estep_hint_f32(const float* X, int64_t N, const float* mu, const float* w2,
                            const float* mu2, int64_t C, int D, double sigma, double lgn,
                            const float* shift_hint, float* T, float* T2, float* stats, void* ws,
                            size_t ws_bytes, dicp_stream_t stream);

/* M-step column pass over components c (evaluated as a row pass, log domain, robust for
 * empty components like softmax(lgamma, dim=0)):
 *   colstats[c*(D+1) + ...] = { log sum_n gamma_nc          (= new w_c,  GMM.py:293),
 *                               sum_n gamma_nc x_n / sum_n gamma_nc (D)  (= new mu_c, GMM.py:287) } */
int dicp_gmm_mstep_f32(const float* X, const float* T2, int64_t N, const float* mu,
                       const float* w2, int64_t C, int D, double sigma, float* colstats,
                       void* ws, size_t ws_bytes, dicp_stream_t stream);

/* Targets / free-energy row pass with OLD responsibilities and NEW parameters
 * (GMM.py:303-314): gamma from (mu_old, w2_old, sigma_old, T2) against mu_new, lpi_new:
 *   rows[n*(D+4) + ...] = { Y_n = sum_c gamma mu_new_c (D), sum_c gamma |mu_new_c|^2,
 *                           sum_c gamma lpi_new_c, sum_c gamma, sum_c gamma |x_n - mu_new_c|^2 } */
int dicp_gmm_targets_f32(const float* X, const float* T2, int64_t N, const float* mu_old,
                         const float* w2_old, double sigma_old, const float* mu_new,
                         const float* lpi_new, int64_t C, int D, float* rows, void* ws,
                         size_t ws_bytes, dicp_stream_t stream);

/* ------------------------------------------------------------------------------------
 * Momenta from speeds (LDDMMModel.v2p, LDDMM.py:235-253): ridge solve
 *   (K(x,x) + alpha I) b = v,   x (M,D), v, b (M,D)
 * by conjugate gradients with the KRed reduction as mat-vec.  Replaces KridgeSolve_keops
 * (kernel.py:239-241: KeOps LazyTensor.solve, i.e. CG on the flattened (M,D) system with the
 * stopping rule |r|^2 < M*D*eps^2) and KridgeSolve_torch (kernel.py:234-237, dense solve).
 * start = 1 initialises (b = 0, r = v); each call then launches `iters` CG iterations,
 * stream-ordered, without synchronising the host; iterations after convergence are no-ops
 * (device flag).  Call again with start = 0 to continue.  The first 16 bytes of `ws` hold the
 * solver status { int32 done (0 running, 1 converged, 2 breakdown), int32 iterations,
 * float |r|^2, float threshold }, which the caller reads between chunks.
 * Workspace kind DICP_WS_RIDGE_CG (the state must persist across calls: same ws). */
int dicp_kernel_ridge_cg_f32(const float* x, int64_t M, int D, double sigma, double alpha,
                             double eps, const float* v, float* b, int start, int iters,
                             void* ws, size_t ws_bytes, dicp_stream_t stream);

/* ------------------------------------------------------------------------------------ */
/* Gradient reductions: the backward passes of GenDKRed, HessKRed, GradLapKRed, DDKRed and
 * GradKRed_rev, which the reference takes from KeOps / torch autodiff (kernel.py:147-168,
 * :194-207, :284-292).  Rows x (M, D) with optional row D-vectors r1, r2; columns y (N, D)
 * with optional column D-vectors c1, c2 and optional column scalar cw (N,).  NULL reads as
 * zeros (r2 and c2 both NULL: the weight r2.c2 reads as 1; cw NULL reads as 1).
 * z = x_i - y_j, K = exp(-|z|^2 / (2 sigma^2)), s = 1/sigma^2; out (M, D):
 *   HESSW    sum_j cw_j (r2_i.c2_j) [s^2 (z.u) z - s u] K,    u = r1_i - c1_j
 *   HESSWP   sum_j [s^2 (z.u) z - s u] K,                     u = r1_i * c1_j (elementwise)
 *   ZDOTV    sum_j -s (z.a) K c2_j,                           a = r1_i + c1_j
 *   HESS3    sum_j K (s^2 [(z.g) u + (z.u) g] - s z [s^2 (z.u)(z.g) - s (u.g)]),
 *                                                             u = r1_i - c1_j, g = r2_i + c2_j
 *   GRADLAP3 sum_j -K [(s^3 |z|^2 - (D+2) s^2) g + s^3 (D + 4 - s |z|^2)(g.z) z],  g = r1_i + c1_j
 * Workspace kind DICP_WS_GRAD. */
enum dicp_grad_kind {
  DICP_GRAD_HESSW = 0, DICP_GRAD_HESSWP = 1, DICP_GRAD_ZDOTV = 2, DICP_GRAD_HESS3 = 3,
  DICP_GRAD_GRADLAP3 = 4
};
int dicp_gauss_red_grad_f32(int kind, const float* x, int64_t M, const float* y, int64_t N, int D,
                            const float* r1, const float* r2, const float* c1, const float* c2,
                            const float* cw, double sigma, float* out, void* ws, size_t ws_bytes,
                            dicp_stream_t stream);

/* Scratch bytes needed by entry `kind` (one of the DICP_WS_* below) at these sizes.
 * LDDMM kinds: M = support points, N = columns (RED) or external points (EXT).
 * GMM kinds: M = data points N, N = components C. */
enum dicp_ws_kind {
  DICP_WS_RED = 0, DICP_WS_ODE_SELF_FWD = 1, DICP_WS_ODE_SELF_BWD = 2, DICP_WS_ODE_EXT_FWD = 3,
  DICP_WS_ODE_EXT_BWD = 4, DICP_WS_GMM_ESTEP = 5, DICP_WS_GMM_MSTEP = 6, DICP_WS_GMM_TARGETS = 7,
  DICP_WS_RIDGE_CG = 8,          /* M = points, N unused */
  DICP_WS_ODE_SELF_FWD_ROWS = 9, /* M = rows of the slice, N = all points (columns) */
  DICP_WS_ODE_SELF_BWD_PART = 10, /* M = points, N = nparts */
  DICP_WS_GRAD = 11,             /* dicp_gauss_red_grad_f32: M rows, N columns */
  DICP_WS_ODE_SELF_FWD_PHASED = 12 /* dicp_lddmm_euler_step_phase_f32: M = rows, N = points */
};
size_t dicp_workspace_bytes(int kind, int64_t M, int64_t N, int D);

const char* dicp_last_error(void);
const char* dicp_version(void);
/* 1 if D is compiled in. */
int dicp_supports_dim(int D);
/* Tuning / A-B knobs (process-wide unless stated; results of every setting agree to fp32
 * summation order):
 *   "fwd_alg"      eta = 0 ODE forward: 0 ordered rows, 1 symmetric pair-once, 2 packed-FP32
 *                  (default: ordered packed rows, and for whole passes from 20k points -- or,
 *                  under a "batch_share" hint, >= 1e9 pairs over the sharing calls -- the
 *                  symmetric pass of 5; its mG-less form stays ordered), 3 channel
 *                  contraction on the matrix cores (opt-in; fp32 error bounded by the rows'
 *                  spread: pass a spatial row_order), 4 symmetric pair-once with packed-FP32
 *                  rows, 5 symmetric pair-once with 4 packed rows per lane and packed column
 *                  sums wherever it applies (whole passes in scaled coordinates; row slices and
 *                  raw coordinates run the ordered rows), 6 ordered packed rows always;
 *                  eta != 0: >= 2 packed-FP32 rows, otherwise ordered scalar rows
 *   "bwd_alg"      eta = 0 VJP: 0 / 1 ordered pair algebras, 2 symmetric pair-once, 3 symmetric
 *                  with packed-FP32 rows (default)
 *   "bwd_eta_alg"  eta != 0 VJP: 0 ordered, 1 symmetric, 2 symmetric packed-FP32 (default)
 *   "r_fwd" / "r_bwd"  rows per thread {1,2,4} of the ordered passes (env DICP_R_FWD / DICP_R_BWD)
 *   "split_rounds", "force_splits", "sym_L"  column-split / symmetric-chunk geometry (0 = auto)
 *   "min_chunk"    smallest column chunk of a split, 16..65536; 0 (default) = 256
 *   "pk_rp"        packed row passes: row pairs per thread, 0 automatic (2 for the eta = 0 fused
 *                  forward and the packed external-point / KRed passes from 32k rows and 8k
 *                  columns, else 1), 1 or 2 forced
 *   "sym_rp"       packed symmetric eta = 0 VJP: row pairs per lane, 0 automatic (2, i.e. 4 rows
 *                  in 256-point groups, for whole passes from 40k points, for row-split parts
 *                  from 64k points with >= 2e9 pairs per part, under a "batch_share" hint from
 *                  1e9 pairs over the sharing calls; else 1), 1 or 2 forced
 *   "red_alg"      KBase / KRedScal / KRed / GradKRed and the external-point forward: 0 never
 *                  the centred expansion, 1 automatic by size (default), 2 always
 *   "sym_red"      KBase / KRedScal / KRed with the rows equal to the columns (x == y): 0 never
 *                  the pair-once symmetric centred sum, 1 automatic (default: wherever the
 *                  centred expansion applies -- "red_alg" -- i.e. from 50k x 50k), 2 always
 *                  (x == y only)
 *   "sym_red_rows" rows per lane of the pair-once sums: 0 automatic (4), 4 or 8 forced
 *   "sym_fwd_rows" rows per lane of the symmetric eta = 0 forward: 0 automatic (6 from 40k, 8 from 180k
 *                  points alone on the chip, else 4), 4, 6 or 8 forced
 *   "lse_pk"       GMM E / M passes: 1 rows packed in float2 pairs (v_pk_fma_f32, default),
 *                  0 scalar rows (bitwise equal)
 *   "lse_adapt"    GMM E / M passes: tiles with a tile-end re-reference (anywhere in the
 *                  workgroup) before the rest of the chunk tests per pair; 0 per pair from the
 *                  start (default 1; env DICP_LSE_ADAPT)
 *   "lse_bound"    hinted GMM E-step against >= 8192 components: 1 (default; env
 *                  DICP_LSE_BOUND) the shift min(hint - 8, max_c w2_c - 8), which no logit can
 *                  overflow, and rows whose LSE ends > 80 below it summed again exactly; 0 the
 *                  sampled shift (unhinted calls always take the sampled shift)
 *   "cx_rho_x100"  centred expansion: largest compact sub-tile radius (scaled units x 100)
 *   "mfma_rmax_x100"  matrix-core forward (fwd_alg 3): largest workgroup row spread (scaled
 *                  units x 100) that takes the MFMA branch; >= 100000 always, 0 never (default 300)
 *   "ext_alg"      KRed and the external-point passes below the centred sizes: 0 generic
 *                  scalar rows, 1 packed-FP32 rows (default)
 *   "batch_share"  PER HOST THREAD geometry hint, default 1: the number of equal calls a launch
 *                  shares the device with (the frames of a launch batch); split counts, column
 *                  groups per workgroup and the 4-row rules are then sized for 1/share of the
 *                  chip.  Changes only the fp32 summation order; a call made alone with the same
 *                  share computes the same bits.  Workspace sizes do not depend on it.
 *   "coord_raw"    PER HOST THREAD: 1 runs the default packed shooting kernels (fwd_alg 2,
 *                  bwd_alg 3) in original-unit coordinates -- exact pair differences at any
 *                  cloud extent, one packed multiply more per two pairs; 0 (default) scaled
 *                  coordinates alpha (q - q_0), float32-exact up to ~200 sigma of extent
 * Returns DICP_ERR_INVALID for an unknown name or an out-of-range value. */
int dicp_set_option(const char* name, int value);
/* Current value of a knob of dicp_set_option (same names; the compile-time defaults until
 * set), written to *value.  Returns DICP_ERR_INVALID for an unknown name or a NULL value.
 * No reference counterpart: lets the host binding ask which kernel variant an entry point
 * will run instead of mirroring the library's defaults. */
int dicp_get_option(const char* name, int* value);
/* Number of column splits the library will use for an M x N pass (diagnostics/bench). */
int dicp_num_splits(int kind, int64_t M, int64_t N);

/* ----------------------------------------------------------------------------------
 * Launch batching (no reference counterpart; replaces the per-frame launches of the atlas'
 * independent frames, PSR.py:528-569, by one grid over all of them).
 * dicp_batch_begin: from now on, the calling host thread's calls of the dicp_lddmm_ode_self_*
 * / dicp_lddmm_euler_* entry points validate their arguments and RECORD their kernel launches
 * (each call with its own arguments, outputs and workspace) instead of issuing them; they return
 * DICP_OK without touching the device.  The calls of one batch must be independent (no call
 * reads another's outputs) and their buffers must stay allocated until the batch has run.
 * dicp_batch_end(stream): issue everything recorded on `stream`, stage by stage (every call's
 * first launch, then every call's second launch, ...), one batched launch per kernel
 * instantiation and stage (blockIdx.z = the call, up to 12 calls per launch).  Each call
 * computes bitwise what it computes alone (same geometry, same order of summation).  Returns
 * DICP_ERR_UNSUPPORTED, and issues nothing, if a recorded call took a path whose kernels have
 * no batched form (checked before the first launch); returns DICP_ERR_HIP if a batched launch
 * fails, in which case earlier stages may already have been issued and the outputs and
 * workspaces of every call of the batch are undefined -- the batchable paths are the packed eta = 0 forward passes (fwd_alg 2,
 * with or without the divergence rows) and the packed symmetric eta = 0 VJPs (bwd_alg 3: full,
 * zero mG cotangent, gp only, 2 or 4 rows per lane, scaled or raw coordinates) with their
 * merges.  dicp_batch_abort: discard an open batch.  One open batch per host thread. */
int dicp_batch_begin(void);
int dicp_batch_end(dicp_stream_t stream);
int dicp_batch_abort(void);

#ifdef __cplusplus
}
#endif
#endif /* DIFFICP_HIP_H */
