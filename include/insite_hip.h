/*
 * insite_hip.h — C ABI of libinsite_hip.so, the MI355X (gfx950) implementation of the
 * INSITE ODE-discovery hot path.
 *
 * Reference interfaces replaced (paths relative to the reference repo root):
 *   - pysindy  PolynomialLibrary(degree=2, interaction_only=True)
 *       called at libs_m/ct/src/models/sindy.py:186-188          -> insite_poly_library
 *   - pysindy  SINDy(STLSQ(threshold, alpha, max_iter=100),
 *                    SmoothedFiniteDifference(savgol 5/3, order=4),
 *                    PolynomialLibrary).fit(X_a, u=U_a, t=dt, multiple_trajectories=True)
 *       called at libs_m/ct/src/models/sindy.py:190-192           -> insite_gram_f64
 *                                                                   + insite_stlsq_f64
 *   - STLSQ._reduce / LSQIntialMask (per-patient initial-mask refit)
 *       libs_m/ct/src/data/pkpd/utils.py:183-327;
 *       pkpd_simulation.py:791-800                  -> insite_sindy_fit_per_patient_f64,
 *                                                      insite_stlsq_f64 (n_sys = N)
 *   - jit(vmap(simulate_cancer_volume))(y0, treatments, dt, statics) with the Euler-5
 *       odeint (libs_m/ct/src/models/sindy.py:413-431; pkpd/utils.py:68-94)
 *                                                                -> insite_rollout_f64
 *   - predict_with_reduced_coefs (per-patient coefficients)
 *       libs_m/ct/src/models/sindy.py:767-778                     -> insite_rollout_f64
 *                                                                   (coef_row_stride != 0)
 *   - masked squared-error sums of get_normalised_masked_rmse /
 *       get_normalised_n_step_rmses (time_varying_model.py:236-313) -> insite_masked_sse_f64
 *
 * The reference has no FFI (it is Python/JAX); these entry points are what a ctypes /
 * cffi binding of the two call sites above binds to (INTEGRATION.md shows the stub).
 *
 * Conventions
 *   - Every array argument is a DEVICE pointer to caller-owned memory unless documented
 *     as host; row-major; leading dimensions in elements.  The library never allocates
 *     device memory: callers size workspaces with the *_workspace_bytes queries.
 *   - Every compute entry point is asynchronous on the caller's HIP stream (`stream` is a
 *     hipStream_t passed as void*; NULL = the default stream) and uses the caller's current
 *     device.  No entry point synchronises the device.
 *   - Return value: 0 = success, negative = error (insite_strerror).  No exceptions cross
 *     the ABI.  Entry points are reentrant; the library holds no mutable global state apart from
 *     the mutex-guarded hipRTC kernel cache of insite_rollout_ms_sparse_f32.
 *   - Polynomial libraries are over the inputs [x, u_0, .., u_{U-1}] (one state x, U static
 *     covariates) and are described by an exponent table exps[F][1+U] (int8, HOST memory)
 *     in pysindy column order (insite_poly_library produces it).
 */
#ifndef INSITE_HIP_H_
#define INSITE_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define INSITE_ABI_VERSION 9

/* status codes */
#define INSITE_OK 0
#define INSITE_E_INVALID_ARG (-1)
#define INSITE_E_UNSUPPORTED (-2)
#define INSITE_E_WORKSPACE (-3)
#define INSITE_E_HIP (-4)

/* derivative estimators (pysindy differentiation methods used at sindy.py:190-203) */
#define INSITE_FD_SMOOTHED4 0 /* SmoothedFiniteDifference(savgol 5/3, order=4); x_dot from the smoothed
                                 series, library on the RAW x (pinned: tests/test_reference_cohort.py) */
#define INSITE_FD_ORDER4 1    /* FiniteDifference(order=4) */
#define INSITE_FD_ORDER1 2    /* FiniteDifference(order=1): forward, backward at the last sample */
#define INSITE_FD_SMOOTHED1 3 /* SmoothedFiniteDifference(savgol window 2, polyorder 1) + order 1 */

/* integrators (odeint, pkpd/utils.py:68-94) */
#define INSITE_METHOD_EULER 0 /* `substeps` forward-Euler steps per interval; 5 = reference Euler-5 */
#define INSITE_METHOD_RK4 1   /* `substeps` classical RK4 steps per interval */

/* storage layouts of per-step matrices (arm, y): element (patient r, step k) at
 *   PATIENT_MAJOR: a[r * ld + k]   (the reference's [N, T] arrays; ld >= T)
 *   TIME_MAJOR:    a[k * ld + r]   (ld >= n_rows; every step of a wavefront is one contiguous run)
 *   TIME_MAJOR_BITS (rollout only, n_arms <= 2): y as TIME_MAJOR; the arms are a bitmask,
 *                  arm of (r, k) = bit (r & 31) of ((const uint32_t*)arm)[k * ld_arm + (r >> 5)],
 *                  ld_arm in 32-bit words >= ceil(n_rows / 32), arm 4-byte aligned;
 *                  or, with ld_arm < 0 (round 6, INSITE_ARM_BITS_TILE_MAJOR; insite_rollout_f64, the fused /
 *                  deferred / lagged steps and insite_refit_rollout_moments_f64), TILE-major: with S = -ld_arm >= T
 *                  steps per tile, arm of (r, k) = bit (r & 31) of
 *                  ((const uint32_t*)arm)[((r >> 6) * S + k) * 2 + ((r >> 5) & 1)] -- a 64-patient tile's
 *                  32-step arm group is 256 contiguous bytes (the time-major rows put 16 tiles on one 128-B line,
 *                  which a 1M-patient rollout re-fetches once per tile) */
#define INSITE_ARM_BITS_TILE_MAJOR(steps_per_tile) (-(int64_t)(steps_per_tile)) /* the ld_arm value */
#define INSITE_LAYOUT_PATIENT_MAJOR 0
#define INSITE_LAYOUT_TIME_MAJOR 1
#define INSITE_LAYOUT_TIME_MAJOR_BITS 2
#define INSITE_LAYOUT_PATIENT_MAJOR_BITS 3 /* insite_rollout_rk45_f64 only: t_obs / y_out [n_rows, ld],
                                            arm bits [n_rows, ld_arm] words, bit k & 31 of word k >> 5 */

/* limits of this ABI version */
#define INSITE_MAX_TERMS 9  /* F of the fused affine path (one Gram/moment entry per lane, F(F+1)/2 + F <= 64);
                               insite_gen_gram_f64 / STLSQ take F <= 64 */
#define INSITE_MAX_STATICS 3
#define INSITE_MAX_ARMS 4
#define INSITE_MAX_STATE_DEGREE 1 /* max exponent of x of the fused affine kernels; the general path
                                     (insite_gen_gram_f64, insite_rollout_f64's polynomial dispatch) takes 4 */

int32_t insite_abi_version(void);
const char* insite_strerror(int32_t code);

/* pysindy PolynomialLibrary column order over (1 + n_statics) inputs: bias, linear, then
 * products by degree in itertools.combinations(_with_replacement) order.
 * exps_out: HOST int8 [max_terms][1 + n_statics]; *n_terms receives F. */
int32_t insite_poly_library(int32_t n_statics, int32_t degree, int32_t interaction_only,
                            int8_t* exps_out, int32_t max_terms, int32_t* n_terms);

/* Fused discovery pass (smoothing + finite differences + library + Gram), replacing the
 * row materialisation and Theta^T Theta of SINDy.fit.  For every patient p with
 * L = min(rows[p], n_steps) >= 5 observation rows x[p, 0..L-1] and training arm a = arm[p]:
 *     G_out[a] += Theta_p^T Theta_p,   b_out[a] += Theta_p^T xdot_p
 * where Theta_p[k, j] = column j evaluated at (x[k], u[p, :]) — the raw samples; only x_dot
 * comes from the savgol 5/3-smoothed series for INSITE_FD_SMOOTHED4.  Patients with L < 5 contribute nothing
 * (pysindy raises; the caller validates).  Deterministic: fixed-order reductions.
 *   x     f64, `layout` (INSITE_LAYOUT_*) with n_steps stored steps:
 *           PATIENT_MAJOR x[p * ldx + k], ldx >= n_steps  (the reference's [N, T] array)
 *           TIME_MAJOR    x[k * ldx + p], ldx >= n_patients (coalesced streaming)
 *   u     [n_patients, n_statics] f64
 *   arm   [n_patients] int8 in [0, n_arms)
 *   rows  [n_patients] int32
 *   G_out [n_arms, F, F] f64 (overwritten), b_out [n_arms, F] f64 (overwritten)
 * Workspace: insite_gram_workspace_bytes; its first 512 bytes (the in-launch reduction's arrival
 * counters) must be zero before the workspace's first use -- every call leaves them zero (ABI 3).
 * The same holds for the workspaces of insite_sindy_fit_f64 and the *_segments_* calls.          */
size_t insite_gram_workspace_bytes(int64_t n_patients, int32_t n_arms, int32_t n_terms);
int32_t insite_gram_f64(const double* x, int64_t ldx, int32_t layout, int32_t n_steps, const double* u,
                        const int8_t* arm, const int32_t* rows, int64_t n_patients, int32_t n_statics,
                        int32_t n_arms, const int8_t* exps, int32_t n_terms, int32_t fd_kind, double dt,
                        double* G_out, double* b_out, void* workspace, size_t workspace_bytes,
                        void* stream);

/* SINDy.fit replacement (reference sindy.py:190-192): insite_gram_f64 followed, in the same
 * finalisation launch, by one STLSQ fit per arm (insite_stlsq_f64 semantics).
 *   coef_out [n_arms, F] f64, mask_out [n_arms, F] int8 (may be NULL),
 *   iters_out [n_arms] int32 (may be NULL; -1 flags a non-positive-definite solve).
 *   G_out / b_out receive the Gram/moment sums as in insite_gram_f64.                     */
int32_t insite_sindy_fit_f64(const double* x, int64_t ldx, int32_t layout, int32_t n_steps, const double* u,
                             const int8_t* arm, const int32_t* rows, int64_t n_patients, int32_t n_statics,
                             int32_t n_arms, const int8_t* exps, int32_t n_terms, int32_t fd_kind, double dt,
                             double threshold, double alpha, int32_t max_iter, int32_t unbias,
                             double* G_out, double* b_out, double* coef_out, int8_t* mask_out,
                             int32_t* iters_out, void* workspace, size_t workspace_bytes, void* stream);

/* Fused step for a stream of cohorts (the C2 pipeline; a serving loop): ONE launch that runs the
 * discovery of one cohort (insite_sindy_fit_f64 semantics, TIME_MAJOR x) and, concurrently, the
 * rollout of another cohort with already-known coefficients coef_in (insite_rollout_f64 semantics,
 * TIME_MAJOR_BITS arms, coef_row_stride 0).  The reference runs these as SINDy.fit (sindy.py:190-192)
 * then the counterfactual scan (sindy.py:413-431, 767-778) per dataset; here cohort k's discovery
 * overlaps cohort k-1's rollout inside one kernel (two independent HBM streams: x read, y written),
 * replacing a two-stream pipeline and its events.  Typical use: coef_out of call k is coef_in of call
 * k + 1 (double-buffered by the caller).  Shape restrictions of this entry point (others return
 * INSITE_E_UNSUPPORTED; use the two separate calls): n_arms = 2, n_terms = 7 (the degree-2 library
 * over [x, u0, u1]), state degree <= 1.  The library (exps, n_statics) is shared by both halves; ru
 * [n_rows, n_statics] are the rollout cohort's statics.  n_rows = 0 or T = 0 skips the rollout (then
 * its pointers may be NULL).  gram_blocks: blocks given to the discovery (0 = the library's default
 * split).  Outputs are those of the separate calls: y_out bitwise; G/b/coef as insite_sindy_fit_f64
 * with the same block count (fixed-order sums).  Workspace: insite_gram_workspace_bytes(n_patients, 2,
 * 7), header zero as for insite_sindy_fit_f64. */
int32_t insite_fit_rollout_f64(const double* x, int64_t ldx, int32_t n_steps, const double* u, const int8_t* arm,
                               const int32_t* rows, int64_t n_patients, int32_t n_statics, int32_t n_arms,
                               const int8_t* exps, int32_t n_terms, int32_t fd_kind, double dt, double threshold,
                               double alpha, int32_t max_iter, int32_t unbias, double* G_out, double* b_out,
                               double* coef_out, int8_t* mask_out, int32_t* iters_out, const double* y0,
                               const double* ru, const uint32_t* arm_bits, int64_t ld_arm, const double* coef_in,
                               int64_t n_rows, int32_t T, double rdt, int32_t method, int32_t substeps,
                               double drop_below, double* y_out, int64_t ld_y, int32_t gram_blocks, void* workspace,
                               size_t workspace_bytes, void* stream);

/* The fused step with the discovery's finalisation deferred by one call (ABI 6; the C2 bench's N = 1 schedule).
 * In insite_fit_rollout_f64 the discovery's last block reduces every block's partial and solves the STLSQ after
 * all other blocks have streamed -- a serial tail the launch cannot end before.  Here call k streams cohort k's
 * Gram into workspace partial slot `slot` (0 or 1) only; with finalize_prev = 1 one block of the same launch
 * reduces the partials the previous call left in slot 1 - slot and writes THAT cohort's G_out, b_out, coef_out,
 * mask_out, iters_out (insite_sindy_fit_f64 semantics, the same fixed-order sums as insite_fit_rollout_f64 with
 * the same gram_blocks); the rollout half is that of insite_fit_rollout_f64 (y_out bitwise).  A stream: call k
 * uses slot k % 2, finalize_prev = (k > 0), and rolls out with the coefficients call k - 1 produced (cohort
 * k - 2); a last call with n_patients = 0, n_rows = 0 and finalize_prev = 1 finalises the stream's last
 * cohort.  Each slot's header records the block count and system size its partials were streamed with (ABI 8),
 * and the finalisation sums exactly those: consecutive calls may change gram_blocks, method or fd_kind.  A
 * finalisation of a slot no call has streamed (or streamed for another system: the record holds a fingerprint of
 * the library's columns, statics count and arm count) writes NaN G|b and coefficients,
 * mask 0 and iters -3.  Same shape restrictions as insite_fit_rollout_f64.  Workspace:
 * insite_fit_rollout_deferred_workspace_bytes: 4 KiB of claim areas at offset 0 that must be zero before the first call
 * (a zero-filled buffer; every call leaves them zero, and their place does not depend on the cohort size), then the
 * two slots (their headers need not be zero). */
size_t insite_fit_rollout_deferred_workspace_bytes(int64_t n_patients, int32_t n_arms, int32_t n_terms);
int32_t insite_fit_rollout_deferred_f64(const double* x, int64_t ldx, int32_t n_steps, const double* u,
                                        const int8_t* arm, const int32_t* rows, int64_t n_patients, int32_t n_statics,
                                        int32_t n_arms, const int8_t* exps, int32_t n_terms, int32_t fd_kind, double dt,
                                        double threshold, double alpha, int32_t max_iter, int32_t unbias,
                                        double* G_out, double* b_out, double* coef_out, int8_t* mask_out,
                                        int32_t* iters_out, const double* y0, const double* ru,
                                        const uint32_t* arm_bits, int64_t ld_arm, const double* coef_in,
                                        int64_t n_rows, int32_t T, double rdt, int32_t method, int32_t substeps,
                                        double drop_below, double* y_out, int64_t ld_y, int32_t gram_blocks,
                                        int32_t slot, int32_t finalize_prev, void* workspace, size_t workspace_bytes,
                                        void* stream);

/* The deferred step for N > 1 ranks (ABI 8; bench.py --gpus N): between the gram and the STLSQ the ranks
 * all-reduce G|b (one RCCL all-reduce of the Gram/moment matrices), so the finalisation splits in
 * two roles of the same launch.  Call k streams cohort k's Gram into slot `slot` (as the deferred call); with
 * reduce_prev = 1 one block reduces the other slot's partials to this RANK'S G_out, b_out (the same fixed-order
 * sums, no STLSQ); with G_fit/b_fit non-NULL another block solves the STLSQ of that (all-reduced, [A, F, F] and
 * [A, F], full symmetric G) system into coef_out, mask_out, iters_out (insite_stlsq_f64 semantics, bitwise equal
 * on every rank given equal G|b); the other blocks roll out (y0, ru, arm_bits) with coef_in.  A stream at N > 1
 * with K fits per all-reduce bucket: G_out of cohort c is written by call c + 1, the bucket of cohorts
 * [jK, jK + K) is all-reduced after call jK + K on the same stream, cohort c is solved by call c + K + 1 and
 * rolled out by call c + K + 2 (bench.py lagged_run).  G_fit and b_fit must not alias G_out/b_out of the same
 * call.  coef_out may be NULL when G_fit is.  Workspace as insite_fit_rollout_deferred_f64 (slot records too). */
int32_t insite_fit_rollout_lagged_f64(const double* x, int64_t ldx, int32_t n_steps, const double* u,
                                      const int8_t* arm, const int32_t* rows, int64_t n_patients, int32_t n_statics,
                                      int32_t n_arms, const int8_t* exps, int32_t n_terms, int32_t fd_kind, double dt,
                                      double threshold, double alpha, int32_t max_iter, int32_t unbias, double* G_out,
                                      double* b_out, const double* G_fit, const double* b_fit, double* coef_out,
                                      int8_t* mask_out, int32_t* iters_out, const double* y0, const double* ru,
                                      const uint32_t* arm_bits, int64_t ld_arm, const double* coef_in, int64_t n_rows,
                                      int32_t T, double rdt, int32_t method, int32_t substeps, double drop_below,
                                      double* y_out, int64_t ld_y, int32_t gram_blocks, int32_t slot,
                                      int32_t reduce_prev, void* workspace, size_t workspace_bytes, void* stream);

/* Treatment-segment discovery for the cancer_sim / EQ_5 datasets, replacing
 * process_sindy_training_data's segment split (libs_m/ct/src/data/pkpd/utils.py:433-462, 607-637)
 * and the four per-arm SINDy(FiniteDifference(order=1)).fit calls (libs_m/ct/src/models/sindy.py:
 * 193-216).  For patient p with L = min(seq_len[p], n_steps - 1) the samples x(p, 0..L) are cut at
 * every k in 1..L-1 where arm(p, k) != arm(p, k-1) into treatment-constant segments that share their
 * boundary sample (each >= 2 samples); every segment s of arm a adds
 *     G_out[a] += Theta_s^T Theta_s,   b_out[a] += Theta_s^T xdot_s
 * with xdot from pysindy FiniteDifference(order=1) on the segment (forward differences, backward at
 * its last sample; INSITE_FD_ORDER1) or SmoothedFiniteDifference(savgol window 2, polyorder 1)
 * (INSITE_FD_SMOOTHED1: the library then sees the smoothed samples).  G_out[a][0][0] (bias column)
 * is arm a's sample count; an arm with none has G = b = 0 (pysindy raises; the caller checks).
 *   x        f64 element (p, k) at x[p * ldx + k] (PATIENT_MAJOR, ldx >= n_steps) or x[k * ldx + p]
 *            (TIME_MAJOR, ldx >= n_patients), k < n_steps
 *   arm      int8 in [0, n_arms), element (p, k), k < n_steps - 1, same layout, leading dim ld_arm
 *   seq_len  [n_patients] int32;  u [n_patients, n_statics] f64 (statics, constant over time)
 *   G_out [n_arms, F, F], b_out [n_arms, F] f64 (overwritten); deterministic (fixed-order sums).
 * insite_sindy_fit_segments_f64 adds one STLSQ fit per arm in the finalisation launch
 * (insite_sindy_fit_f64 semantics for coef_out / mask_out / iters_out). */
size_t insite_gram_segments_workspace_bytes(int64_t n_patients, int32_t n_arms, int32_t n_terms);
int32_t insite_gram_segments_f64(const double* x, int64_t ldx, const int8_t* arm, int64_t ld_arm, int32_t layout,
                                 int32_t n_steps, const int32_t* seq_len, const double* u, int64_t n_patients,
                                 int32_t n_statics, int32_t n_arms, const int8_t* exps, int32_t n_terms,
                                 int32_t fd_kind, double dt, double* G_out, double* b_out, void* workspace,
                                 size_t workspace_bytes, void* stream);
int32_t insite_sindy_fit_segments_f64(const double* x, int64_t ldx, const int8_t* arm, int64_t ld_arm, int32_t layout,
                                      int32_t n_steps, const int32_t* seq_len, const double* u, int64_t n_patients,
                                      int32_t n_statics, int32_t n_arms, const int8_t* exps, int32_t n_terms,
                                      int32_t fd_kind, double dt, double threshold, double alpha, int32_t max_iter,
                                      int32_t unbias, double* G_out, double* b_out, double* coef_out, int8_t* mask_out,
                                      int32_t* iters_out, void* workspace, size_t workspace_bytes, void* stream);

/* Per-patient refit (reference LSQIntialMask, pkpd/utils.py:183-327,
 * as used by determine_individualized_equation_coefs, pkpd_simulation.py:791-800): for every patient
 * with >= 5 rows, STLSQ on its own rows (same derivative estimator and library as
 * insite_gram_f64) starting from the support of global_coef[arm[p]] (|c| > 1e-14); unbias = the
 * minimum-norm least-squares solution on the final support (lstsq semantics; with constant statics a
 * patient's Theta has rank <= 2); if sum |c| > 10 the last ridge iterate is kept (the reference's
 * unbias=False refit).  Other arms keep the global rows; patients with < 5 rows keep the global
 * model (iters 0).  Inputs as insite_gram_f64, plus
 *   global_coef [n_arms, F] f64 (device); coef_out [n_patients, n_arms, F] f64 (feeds
 *   insite_rollout_f64 with coef_row_stride = n_arms * F); mask_out [n_patients, F] int8 (may be
 *   NULL); iters_out [n_patients] int32 (may be NULL).                                          */
size_t insite_per_patient_workspace_bytes(int64_t n_patients);
int32_t insite_sindy_fit_per_patient_f64(const double* x, int64_t ldx, int32_t layout, int32_t n_steps,
                                         const double* u, const int8_t* arm, const int32_t* rows,
                                         int64_t n_patients, int32_t n_statics, int32_t n_arms, const int8_t* exps,
                                         int32_t n_terms, int32_t fd_kind, double dt, const double* global_coef,
                                         double threshold, double alpha, int32_t max_iter, int32_t unbias,
                                         double* coef_out, int8_t* mask_out, int32_t* iters_out, void* workspace,
                                         size_t workspace_bytes, void* stream);

/* Global and per-patient fits from ONE pass over x (config C4, ABI 4).  insite_gram_moments_f64 is
 * insite_gram_f64 (coef_out NULL) or insite_sindy_fit_f64 (coef_out set) that also writes every patient's
 * moments mom_out [n_patients, 5] f64 = {rows, sum x, sum x^2, sum xdot, sum xdot x} (the state the
 * per-patient refit needs); insite_fit_per_patient_moments_f64 is the per-patient STLSQ of
 * insite_sindy_fit_per_patient_f64 from those moments (global_coef on the device: the fused fit's
 * coef_out, or the all-reduced model at N > 1).  Together they replace insite_sindy_fit_f64 +
 * insite_sindy_fit_per_patient_f64, which read x twice.  Requires the library to fit the MFMA Gram plan
 * (n_arms * n_terms <= 16; else INSITE_E_UNSUPPORTED).  Workspace: insite_gram_workspace_bytes. */
int32_t insite_gram_moments_f64(const double* x, int64_t ldx, int32_t layout, int32_t n_steps, const double* u,
                                const int8_t* arm, const int32_t* rows, int64_t n_patients, int32_t n_statics,
                                int32_t n_arms, const int8_t* exps, int32_t n_terms, int32_t fd_kind, double dt,
                                double threshold, double alpha, int32_t max_iter, int32_t unbias, double* G_out,
                                double* b_out, double* coef_out, int8_t* mask_out, int32_t* iters_out, double* mom_out,
                                void* workspace, size_t workspace_bytes, void* stream);
int32_t insite_fit_per_patient_moments_f64(const double* mom, const double* u, const int8_t* arm, const int32_t* rows,
                                           int64_t n_patients, int32_t n_steps, int32_t n_statics, int32_t n_arms,
                                           const int8_t* exps, int32_t n_terms, const double* global_coef,
                                           double threshold, double alpha, int32_t max_iter, int32_t unbias,
                                           double* coef_out, int8_t* mask_out, int32_t* iters_out, void* stream);

/* The per-patient refit of insite_fit_per_patient_moments_f64 folded into the rollout that uses it (C4; ABI
 * 5): one launch, wave = 64 patients, whose prologue refits each lane's factual-arm row (arm[p]) from its
 * moments mom [n_patients, 5] -- the same STLSQ from the global support, the ridge iterations in closed form
 * (rank-2 Gram: a 2 x 2 solve per iteration) and the same unbias -- and whose time loop is insite_rollout_f64's
 * (TIME_MAJOR_BITS arms arm_bits [T, ld_bits], y_out [T, ld_y]; the other arm keeps global_coef).  Replaces
 * predict_with_reduced_coefs over the LSQIntialMask refits (pkpd_simulation.py:791-800, sindy.py:767-778)
 * without the per-patient coefficient rows' HBM round trip.  coef_out [n_patients, n_arms, F] / mask_out
 * [n_patients, F] / iters_out [n_patients] as insite_fit_per_patient_moments_f64, each may be NULL.
 * Restrictions (else INSITE_E_UNSUPPORTED; use the two calls): n_arms <= 2, alpha > 0, state degree <= 1. */
int32_t insite_refit_rollout_moments_f64(const double* mom, const int8_t* arm, const int32_t* rows, int64_t n_patients,
                                         int32_t n_steps, int32_t n_statics, int32_t n_arms, const int8_t* exps,
                                         int32_t n_terms, const double* global_coef, double threshold, double alpha,
                                         int32_t max_iter, int32_t unbias, const double* y0, const double* u,
                                         const uint32_t* arm_bits, int64_t ld_bits, int32_t T, double dt,
                                         int32_t method, int32_t substeps, double drop_below, double* y_out,
                                         int64_t ld_y, double* coef_out, int8_t* mask_out, int32_t* iters_out,
                                         void* stream);

/* Batched sequentially-thresholded least squares on Gram systems (one system per thread):
 * STLSQ._reduce semantics (all-ones initial support; ridge (G_SS + alpha I) c = b_S by
 * Cholesky; zero |c| < threshold; stop when nothing was removed in the first pass or the
 * support is unchanged; empty support -> 0) followed by the pysindy unbias (G_SS c = b_S)
 * on ind = |c| > 1e-14 when `unbias` != 0.
 *   G [n_sys, F, F], b [n_sys, F]; coef_out [n_sys, F] f64; mask_out [n_sys, F] int8 (may be
 *   NULL); iters_out [n_sys] int32 (may be NULL; -1 flags a non-positive-definite solve). */
int32_t insite_stlsq_f64(const double* G, const double* b, int64_t n_sys, int32_t n_terms,
                         double threshold, double alpha, int32_t max_iter, int32_t unbias,
                         double* coef_out, int8_t* mask_out, int32_t* iters_out, void* stream);

/* Batched open-loop counterfactual rollout (one patient per lane, state in registers).
 * For k = 0..T-1:  a = arm[r, k];  advance y over one interval dt with the RHS
 *     f_a(y) = sum_j c[a, j] * Theta_j(y, u[r, :])   over terms with |c[a, j]| > drop_below
 * and store y_out[r, k].  coef is [n_arms, F] (coef_row_stride = 0) or per row
 * [n_rows, n_arms, F] (coef_row_stride = n_arms * F).  `layout` (INSITE_LAYOUT_*) applies to
 * both arm and y_out.
 *   y0 [n_rows] f64, u [n_rows, n_statics] f64, arm int8 and y_out f64 per `layout`.       */
int32_t insite_rollout_f64(const double* y0, const double* u, const int8_t* arm, int64_t ld_arm,
                           const double* coef, int64_t coef_row_stride, const int8_t* exps,
                           int32_t n_terms, int64_t n_rows, int32_t T, int32_t n_statics,
                           int32_t n_arms, double dt, int32_t method, int32_t substeps,
                           double drop_below, double* y_out, int64_t ld_y, int32_t layout, void* stream);

/* Adaptive RK45 rollout on irregular observation grids (configuration C5): for patient r and
 * interval k < n_obs[r] - 1, y advances from t_obs(r, k) to t_obs(r, k + 1) under the arm of bit
 * (r, k) of arm_bits (n_arms <= 2) by scipy's
 * solve_ivp(method='RK45', rtol, atol) controller (Dormand-Prince 5(4), select_initial_step per
 * interval; the reference odeint's tolerances are rtol = atol = 1.4e-8, pkpd/utils.py:87).  This
 * replaces the fixed-grid odeint scan (sindy.py:413-424) when the observation times are irregular.
 *   layout INSITE_LAYOUT_TIME_MAJOR_BITS: t_obs [T_max, ld_t] f64 (ld_t >= n_rows), y_out [T_max, ld_y],
 *          arm_bits [T_max, ld_arm >= ceil(n_rows / 32)] (bit r & 31 of word r >> 5 in row k);
 *   layout INSITE_LAYOUT_PATIENT_MAJOR_BITS (ABI 3; the fast one): t_obs [n_rows, ld_t >= T_max],
 *          y_out [n_rows, ld_y >= T_max], arm_bits [n_rows, ld_arm >= ceil((T_max - 1) / 32)] (bit k & 31
 *          of word k >> 5 in row r).  A lane's window refills and stores stay within its own row, so
 *          binned row orders cost no coalescing.
 *   n_obs [n_rows] int32 in [1, T_max]
 *   coef  [n_arms, F] or per row [n_rows, n_arms, F] (coef_row_stride = n_arms * F)
 *   y_out element (r, k) = state at t_obs(r, k + 1) (elements k >= n_obs[r] - 1 untouched)
 *   steps_out [n_rows] int32 step attempts (accepted + rejected) per row, may be NULL
 *   row_order [n_rows] int32 lane -> row map, a permutation of [0, n_rows) (insite_rk45_order_i32), or
 *             NULL for lane r = row r.  Outputs do not depend on it; rows binned by n_obs keep the
 *             wavefronts' step counts uniform (a wave runs until its slowest lane has finished).  (ABI 3) */
int32_t insite_rollout_rk45_f64(const double* y0, const double* u, const uint32_t* arm_bits, int64_t ld_arm,
                                const double* t_obs, int64_t ld_t, const int32_t* n_obs, const double* coef,
                                int64_t coef_row_stride, const int8_t* exps, int32_t n_terms, int64_t n_rows,
                                int32_t T_max, int32_t n_statics, int32_t n_arms, double rtol, double atol,
                                double drop_below, double* y_out, int64_t ld_y, int32_t* steps_out,
                                const int32_t* row_order, int32_t layout, void* stream);

/* Lane order for insite_rollout_rk45_f64: rows sorted by n_obs, descending (counting sort on the
 * device; bins min(n_obs, 1023)).  No reference counterpart (scheduling only).  n_rows <= INT32_MAX.
 *   n_obs [n_rows] int32, order_out [n_rows] int32; workspace >= insite_rk45_order_workspace_bytes (zeroed by the
 *   call itself; a build with INSITE_RK45_ORDER_SELFRESET=1 instead needs it zero before its first use and leaves it
 *   zero). */
size_t insite_rk45_order_workspace_bytes(int32_t T_max);
int32_t insite_rk45_order_i32(const int32_t* n_obs, int64_t n_rows, int32_t T_max, int32_t* order_out, void* workspace,
                              size_t workspace_bytes, void* stream);

/* INSITE per-patient refinement (reference SINDY._get_fine_tuned_predictions /
 * f_to_min_func / predict_with_reduced_coefs, sindy.py:433-715, 767-794): for every row r with
 * seq_len[r] > tau, the active global coefficients (|coef0| > 1e-3) are refined by BFGS
 * (jax.scipy.optimize.minimize(method='BFGS') semantics) on
 *   f(c) = mse(c) / (2.5 mse(coef0)) + lam * mean((coef0 - c)^2),
 *   mse  = mean_{k < min(seq_len - tau, T - 1)} (V[k + 1] - pred_k)^2, pred = the Euler scan
 *          (`substeps` sub-steps per dt; 5 = odeint) from V[0] under the row's per-step arms;
 * revert_on_zoom_fail != 0: BFGS status 3 (zoom failed) keeps coef0, as the reference CODE reads
 * (sindy.py:628-631); 0: the row keeps its BFGS iterate, which is what the reference's PUBLISHED runs
 * show (all eight EQ_4 INSITE metrics of results/2_main_table/final_with_insite.txt:2387-2402 are
 * reproduced to 1e-10 only without the revert).  Every row then gets the Euler scan
 * of its (refined or global) model over all T steps.
 *   V        [T, ld_v] f64 unscaled observations, time-major (ld_v >= n_rows)
 *   arm_bits TIME_MAJOR_BITS [T, ld_arm] per-step arm (n_arms <= 2)
 *   coef0    HOST [n_arms, F] f64: the global model (any number of active coefficients: up to 16
 *            run register-resident, denser models up to n_arms * F run the scratch-resident kernel)
 *   preds    [T, ld_p] f64 (row k = state after step k); coef_out [n_rows, n_arms, F] (may be NULL);
 *   status_out [n_rows] int32 (-1 = not refined: seq_len <= tau; else the BFGS status: 0 converged,
 *   1 maxiter, 3 zoom failed, 5 line-search maxiter), iters_out [n_rows] int32 (may be NULL).
 *   row_order [n_rows] int32 (ABI 4; may be NULL = identity): lane i refines row row_order[i], a
 *   permutation of 0..n_rows-1 -- scheduling only (outputs are per row, bitwise independent of it); rows
 *   binned by seq_len (insite_rk45_order_i32 on seq_len) keep a wave's objective scans equally long. */
int32_t insite_refine_f64(const double* V, int64_t ld_v, int32_t T, const uint32_t* arm_bits, int64_t ld_arm,
                          const double* u, const int32_t* seq_len, int64_t n_rows, int32_t n_statics, const int8_t* exps,
                          int32_t n_terms, const double* coef0, int32_t n_arms, double dt, double lam, int32_t tau,
                          int32_t substeps, int32_t revert_on_zoom_fail, double* preds, int64_t ld_p,
                          double* coef_out, int32_t* status_out, int32_t* iters_out, const int32_t* row_order,
                          void* stream);

/* INSITE refinement with int8 per-step arms, n_arms <= 4: the cancer_sim / EQ_5 branches of
 * _get_fine_tuned_predictions (sindy.py:484-550: pred_dy_dt picks all_reduced_coefs[argmax(treatment)])
 * with the same objective, BFGS and outputs as insite_refine_f64.
 *   arm [T, ld_arm] int8 time-major per-step arm in [0, n_arms) (ld_arm >= n_rows); the rest as above. */
int32_t insite_refine_arms_f64(const double* V, int64_t ld_v, int32_t T, const int8_t* arm, int64_t ld_arm,
                               const double* u, const int32_t* seq_len, int64_t n_rows, int32_t n_statics,
                               const int8_t* exps, int32_t n_terms, const double* coef0, int32_t n_arms, double dt,
                               double lam, int32_t tau, int32_t substeps, int32_t revert_on_zoom_fail, double* preds,
                               int64_t ld_p, double* coef_out, int32_t* status_out, int32_t* iters_out,
                               const int32_t* row_order, void* stream);

/* Treatment-segment discovery with a GENERAL library (ABI 5, insite_gen.hip): the degree-4 ablation
 * (PolynomialLibrary(degree=4, interaction_only=False), sindy.py:185-186) on the cancer_sim / EQ_5 datasets
 * (run.py:96-104, 208; their DE format pkpd/utils.py:433-462, 607-637).  Same segment walk, derivative
 * (fd_kind INSITE_FD_ORDER1 / INSITE_FD_SMOOTHED1) and arrays as insite_gram_segments_f64, any library with
 * state exponents <= 4 over [x, statics] (exps [n_terms][1 + n_statics], n_terms <= 64): per arm a
 *   G_out[a] = sum over arm-a segment rows of Theta^T Theta,  b_out[a] = Theta^T x_dot  (overwritten),
 * from per-patient power moments (sum x^e, e <= 8; sum x_dot x^e, e <= 4) contracted in a fixed order. */
size_t insite_gen_gram_segments_workspace_bytes(int64_t n_patients, int32_t n_arms, int32_t n_terms);
int32_t insite_gen_gram_segments_f64(const double* x, int64_t ldx, const int8_t* arm, int64_t ld_arm, int32_t layout,
                                     int32_t n_steps, const int32_t* seq_len, const double* u, int32_t n_statics,
                                     int64_t n_patients, int32_t n_arms, const int8_t* exps, int32_t n_terms,
                                     int32_t fd_kind, double dt, double* G_out, double* b_out, void* workspace,
                                     size_t workspace_bytes, void* stream);

/*
 * INSITE layout preparation (ABI 7): the reference hands the refinement patient-major prev_outputs and
 * per-step arms (sindy.py:555-566); the refinement kernels read time-major.  One pass writes
 * Vt [T, ld_vt] from V [n_rows, ld_v] and, when arm [n_rows, ld_arm] is given, either the bit-packed
 * arms arm_bits [T, ld_bits >= ceil(n_rows / 32)] (bit r & 31 of word r >> 5: arm != 0; the per-arm
 * two-arm and joint two-input entries) or int8 arm_t [T, ld_armt] (exactly one of the two).  Replaces
 * three torch copies and an int64 bit-pack of the reference-side transposes.  row_order [n_rows] (may be NULL):
 * output column l takes row row_order[l] (rows binned by sequence length, so a wave's lanes scan similar
 * prefixes while every kernel load stays coalesced); the refinement then runs with the identity lane order
 * on the permuted inputs, and insite_refine_finish_f64 scatters its predictions back.  ABI 8: the same pass also
 * gathers the per-row statics u [n_rows, n_statics] -> u_out (row l = u[row_order[l]]) and the sequence lengths
 * seq_len -> seq_len_out when those pointers are non-NULL (one launch instead of two more gathers).
 */
int32_t insite_refine_prepare_f64(const double* V, int64_t ld_v, const int8_t* arm, int64_t ld_arm, int64_t n_rows,
                                  int32_t T, double* Vt, int64_t ld_vt, uint32_t* arm_bits, int64_t ld_bits,
                                  int8_t* arm_t, int64_t ld_armt, const int32_t* row_order, const double* u,
                                  int32_t n_statics, double* u_out, const int32_t* seq_len, int32_t* seq_len_out,
                                  void* stream);

/* The inverse of insite_refine_prepare_f64 for the refinement's predictions (ABI 7): time-major preds_tm
 * [T, ld_t] whose column l is row row_order[l] (identity when NULL) -> patient-major preds_pm [n_rows, ld_pm],
 * the layout the reference's predictions come in (sindy.py:658-665).  ABI 8: the same pass scatters the lane-order
 * per-row outputs back to row order when given: coef_lane [n_rows, n_coef] -> coef_out, status_lane -> status_out,
 * iters_lane -> iters_out (each pair NULL to skip). */
int32_t insite_refine_finish_f64(const double* preds_tm, int64_t ld_t, const int32_t* row_order, int64_t n_rows,
                                 int32_t T, double* preds_pm, int64_t ld_pm, const double* coef_lane, int32_t n_coef,
                                 double* coef_out, const int32_t* status_lane, int32_t* status_out,
                                 const int32_t* iters_lane, int32_t* iters_out, void* stream);

/* INSITE refinement of ANY global model of the reference (ABI 5, csrc/insite_refine.hip): the joint
 * "one ODE" model (sindy.py:469-483, 503-517, 537-551: one coefficient row over a library whose inputs
 * include the per-step binary treatments) and the degree-4 library (ABLATION_MORE_COMPLEX_BASIS_FUNCTIONS,
 * sindy.py:185-186), besides the per-arm models of the two calls above (which it generalises).  Coefficient
 * q of coef0 [n_coef] contributes c_q * x^coef_exps[q][0] * prod_t u_t^coef_exps[q][1 + t] to the RHS on
 * every step whose arm a has bit a set in coef_arm_mask[q]; per-arm models: q = a * F + j, mask 1 << a;
 * the joint model: arm = the step's treatment bit code, mask = the codes that switch on column j's
 * treatment inputs (their exponents dropped, binary inputs).  State exponents <= 4 (a model with a
 * non-zero coefficient of exponent >= 2 runs the state-polynomial kernels).  Objective, BFGS, status and
 * outputs as insite_refine_f64; coef_out [n_rows, n_coef].
 *   arm_bits TIME_MAJOR_BITS [T, ld_arm] (n_arms <= 2)  XOR  arm [T, ld_arm] int8 (n_arms <= 4)
 *   coef0 / coef_arm_mask [n_coef] / coef_exps [n_coef][1 + n_statics]: HOST arrays, n_coef <= 72   * nfev_out [n_rows] int32 (may be NULL): evaluations of the objective and its gradient per row (each one
 * Euler scan of the row's K-step window with its sensitivities) -- the refinement's work count (bench.py's
 * INSITE roofline: flops = sum_r nfev_r K_r x flops per sensitivity step). */
int32_t insite_refine_general_f64(const double* V, int64_t ld_v, int32_t T, const uint32_t* arm_bits,
                                  const int8_t* arm, int64_t ld_arm, const double* u, const int32_t* seq_len,
                                  int64_t n_rows, int32_t n_statics, int32_t n_coef, const double* coef0,
                                  const int32_t* coef_arm_mask, const int8_t* coef_exps, int32_t n_arms, double dt,
                                  double lam, int32_t tau, int32_t substeps, int32_t revert_on_zoom_fail,
                                  double* preds, int64_t ld_p, double* coef_out, int32_t* status_out,
                                  int32_t* iters_out, int32_t* nfev_out, const int32_t* row_order, void* stream);

/* The refinement on the reference's OWN row layout (ABI 9): _get_fine_tuned_predictions hands over the patient-major
 * prev_outputs [N, T], per-step treatments, statics and sequence lengths (sindy.py:555-566) and takes back the
 * patient-major predictions (sindy.py:658-665).  insite_refine_general_f64 semantics (model description, objective,
 * BFGS, status, outputs bitwise equal), without the prepare / finish passes: the windowed kernel gathers the rows of
 * its lanes (row_order: lane l refines row row_order[l], NULL = identity) straight from V through its LDS ring and
 * stores the predictions through the same ring as 64-B row segments.
 *   V [n_rows, ld_v] f64, ld_v even and V 16-B aligned; arm [n_rows, ld_arm] int8 with values 0 / 1 (n_arms <= 2)
 *   or in [0, n_arms) (n_arms 3-4: the dense 4-arm and joint models, 9-16 active coefficients, on the cooperative
 *   kernel -- 8 lanes a row, the wave's 8 rows staged whole from V and arm, predictions stored into the rows; round 6);
 *   u [n_rows, n_statics], seq_len [n_rows]; preds [n_rows, ld_p], coef_out [n_rows, n_coef], status_out / iters_out
 *   / nfev_out [n_rows] -- every per-row array in ROW order.  ld_v, ld_arm, ld_p >= T.
 * Returns INSITE_E_UNSUPPORTED outside these kernels' shapes (n_arms <= 2: T not in [2, 64], more than 3 active
 * coefficients, odd ld_v / unaligned V; n_arms 3-4: T > 64, not 9-16 active coefficients, INSITE_REFINE_COOP=0; either:
 * a state exponent >= 2 in the model): the caller then takes the prepare / insite_refine_general_f64 / finish route,
 * which covers every model.
 * Concurrency: the opt-in dynamic row assignment (INSITE_REFINE_DYN=1 in the environment; off by default) takes its
 * queue heads from 64 device words handed out round-robin per call, so at most 64 such calls may be in flight at
 * once across independent streams -- a 65th shares a head with a running call (rows skipped or refined twice).  The
 * default static kernel has no such limit. */
int32_t insite_refine_rows_f64(const double* V, int64_t ld_v, int32_t T, const int8_t* arm, int64_t ld_arm,
                               const double* u, const int32_t* seq_len, int64_t n_rows, int32_t n_statics,
                               int32_t n_coef, const double* coef0, const int32_t* coef_arm_mask,
                               const int8_t* coef_exps, int32_t n_arms, double dt, double lam, int32_t tau,
                               int32_t substeps, int32_t revert_on_zoom_fail, double* preds, int64_t ld_p,
                               double* coef_out, int32_t* status_out, int32_t* iters_out, int32_t* nfev_out,
                               const int32_t* row_order, void* stream);

/* General one-state discovery (insite_gen.hip): libraries with state exponents up to 4 and/or per-step
 * binary treatment INPUTS — the reference's degree-4 ablation (PolynomialLibrary(degree=4,
 * interaction_only=False), sindy.py:185-186, run.py:208) and joint "one ODE" model (joint_model with
 * multilabel treatments, pkpd/utils.py:486-497, 639-672; run.py:198-201).  For every patient p with
 * L = min(rows[p], n_steps) >= 5 rows (>= 2 for the order-1 methods) and group g = group[p] (0 when
 * group is NULL):   G_out[g] += Theta_p^T Theta_p,  b_out[g] += Theta_p^T xdot_p,  where row k of
 * Theta_p evaluates column j = x^exps[j][0] * prod_i in_i(k)^exps[j][1+i] * prod_t u_t^exps[j][1+n_in+t]
 * on the RAW x[k] (x_dot by fd_kind over the whole row), in_i(k) = bit i of step_in(p, k) (binary).
 *   x, step_in: `layout` PATIENT_MAJOR ([p * ld + k]) or TIME_MAJOR ([k * ld + p]); n_inputs <= 2
 *   exps [n_terms][1 + n_inputs + n_statics] int8 (HOST), n_terms <= 64
 *   G_out [n_groups, F, F], b_out [n_groups, F] (overwritten); deterministic fixed-order sums.   */
size_t insite_gen_gram_workspace_bytes(int64_t n_patients, int32_t n_steps, int32_t n_groups, int32_t n_terms);
int32_t insite_gen_gram_f64(const double* x, int64_t ldx, int32_t layout, int32_t n_steps, const double* u,
                            int32_t n_statics, const int8_t* step_in, int64_t ld_in, int32_t n_inputs,
                            const int8_t* group, int32_t n_groups, const int32_t* rows, int64_t n_patients,
                            const int8_t* exps, int32_t n_terms, int32_t fd_kind, double dt, double* G_out,
                            double* b_out, void* workspace, size_t workspace_bytes, void* stream);

/* Batched STLSQ for INSITE_MAX_TERMS < F <= 64 (one wavefront per system); insite_stlsq_f64 dispatches
 * here on its own, same arguments and semantics. */
int32_t insite_stlsq_wave64_f64(const double* G, const double* b, int64_t n_sys, int32_t n_terms, double threshold,
                                double alpha, int32_t max_iter, int32_t unbias, double* coef_out, int8_t* mask_out,
                                int32_t* iters_out, void* stream);

/* Stage-evaluated rollout of a library with state degree 2..4 (Euler / RK4 on f_a(y) = sum_e P_a[e] y^e,
 * P_a folded per patient from the columns with |coef| > drop_below), PATIENT_MAJOR or TIME_MAJOR layouts;
 * insite_rollout_f64 dispatches here on its own when exps has a state exponent > 1.  Arguments as
 * insite_rollout_f64. */
int32_t insite_rollout_poly_f64(const double* y0, const double* u, const int8_t* arm, int64_t ld_arm,
                                const double* coef, int64_t coef_row_stride, const int8_t* exps, int32_t n_terms,
                                int64_t n_rows, int32_t T, int32_t n_statics, int32_t n_arms, double dt, int32_t method,
                                int32_t substeps, double drop_below, double* y_out, int64_t ld_y, int32_t layout,
                                void* stream);

/* Masked squared-error sums for the RMSE metrics (time_varying_model.py:236-313):
 *   err[r,k]  = (pred[r, k] * scale + shift - target[r, k])^2 * active[r, k]
 *   per_step_out[k] = sum_r err[r, k]        per_step_cnt_out[k] = sum_r active[r, k]
 *   last_out[0] = sum_r err[r, last_r], last_out[1] = count, where last_r is the final
 *   active entry of row r (active[r,k]=1 and active[r,k+1]=0, or k = T-1).
 * Deterministic fixed-order reduction.  pred [n_rows, ld_pred], target/active [n_rows, T].
 * Outputs f64 device arrays (overwritten). */
size_t insite_masked_sse_workspace_bytes(int64_t n_rows, int32_t T);
int32_t insite_masked_sse_f64(const double* pred, int64_t ld_pred, double scale, double shift,
                              const double* target, const double* active, int64_t n_rows,
                              int32_t T, double* per_step_out, double* per_step_cnt_out,
                              double* last_out, void* workspace, size_t workspace_bytes,
                              void* stream);

/* ---------------------------------------------------------------------------------------------
 * Multi-state path (configuration C3 of BASELINE.json: S = 5 coupled states + one binary per-step
 * treatment input, fp32 storage, fp64 Gram).  Build-defined extension of the same discovery
 * semantics to S states (no reference counterpart; oracle/multistate_ref.py is the restatement):
 * the library is pysindy PolynomialLibrary(degree 2) over the inputs (x_1..x_S, a) — states first,
 * then the input —, the derivative estimator savgol(5,3) + FD4 per state (SmoothedFiniteDifference,
 * reference sindy.py:190), one STLSQ per target state on the shared Gram.
 * Layouts (time-major structure of arrays):
 *   states   x[(k * S + s) * ldx + p]  f32, ldx >= N          (step k, state s, patient p)
 *   input    TIME_MAJOR_BITS bitmask [T, ld_bits] u32, bit p & 31 of word k * ld_bits + p / 32
 *   y0       y0[s * ld_y0 + p] f32;   trajectories y[(k * S + s) * ld_y + p] f32
 * This ABI version instantiates S = 5.
 * --------------------------------------------------------------------------------------------- */

/* Gram of the multi-state regression, replacing the per-target SINDy.fit rows / X^T X:
 *   G_out [F, F] = sum_p Theta_p^T Theta_p,  B_out [F, S] = sum_p Theta_p^T xdot_p  (f64)
 * over patients with >= 5 rows (rows may be NULL: every patient has n_steps rows).  inp_bits may be
 * NULL (library over the states only).  exps: HOST int8 [F][S + (inp_bits != NULL)], the pysindy
 * degree-2 library over those inputs (interaction_only, or full degree 2 without an input);
 * other tables return INSITE_E_UNSUPPORTED.  fd_kind: INSITE_FD_SMOOTHED4. */
size_t insite_gram_ms_workspace_bytes(int64_t n_patients);
int32_t insite_gram_ms_f32(const float* x, int64_t ldx, int32_t n_steps, int32_t n_states, const uint32_t* inp_bits,
                           int64_t ld_bits, const int32_t* rows, int64_t n_patients, const int8_t* exps,
                           int32_t n_terms, int32_t fd_kind, double dt, double* G_out, double* B_out, void* workspace,
                           size_t workspace_bytes, void* stream);

/* One STLSQ (insite_stlsq_f64 semantics) per target on a shared Gram, F <= 32 (one wavefront per
 * target, lane-per-row Cholesky):  G [F, F], B [F, n_targets] (column t = target t);
 * coef_out [n_targets, F], mask_out [n_targets, F] (may be NULL), iters_out [n_targets] (may be NULL,
 * -1 flags a non-positive-definite solve). */
int32_t insite_stlsq_wave_f64(const double* G, const double* B, int32_t n_terms, int32_t n_targets, double threshold,
                              double alpha, int32_t max_iter, int32_t unbias, double* coef_out, int8_t* mask_out,
                              int32_t* iters_out, void* stream);

/* Multi-state open-loop rollout (odeint/RK4 of pkpd/utils.py:68-94 with an S-dimensional state):
 * for k = 0..T-1 the input a = bit (p, k) of inp_bits (0 when NULL) is held over interval k and
 * y advances by `substeps` Euler / RK4 steps of f(y, a) = coef Theta(y, a), coef [S, F] f64 with
 * |c| <= drop_below dropped (utils.py:388); y_out row k = the state after interval k.
 * Arithmetic in fp32 (the C3 configuration's dtype).  exps as insite_gram_ms_f32 (interaction_only). */
int32_t insite_rollout_ms_f32(const float* y0, int64_t ld_y0, const uint32_t* inp_bits, int64_t ld_bits,
                              const double* coef, const int8_t* exps, int32_t n_terms, int32_t n_states,
                              int64_t n_rows, int32_t T, double dt, int32_t method, int32_t substeps,
                              double drop_below, float* y_out, int64_t ld_y, void* stream);

/* Support-specialised variant of insite_rollout_ms_f32 (a sparse discovered model keeps
 * the S-state rollout off the VALU roof).  support: HOST int8 [S][F], nonzero = the term is in the model
 * (e.g. the STLSQ mask).  On first use per (support, method, input count, device) the kernel is generated
 * and compiled with hipRTC (cached for the process; the first call pays ~1-2 s), and evaluates only the
 * supported terms, in the library's column order — the same fp32 sums as the dense kernel, whose dropped
 * terms add fmaf(0, th, f) = f.  Coefficient values are read from `coef` (device) at every launch; if
 * any coefficient outside the support is above drop_below, the launch runs the dense RHS instead (a
 * stale support costs speed, not correctness).  Other arguments and results as insite_rollout_ms_f32.
 * The kernel is compiled for the current device's ISA (hipDeviceProp_t.gcnArchName); if hipRTC or the
 * module load fails, or 64 supports are already cached, the launch runs insite_rollout_ms_f32 (dense
 * RHS, bitwise the same result). */
int32_t insite_rollout_ms_sparse_f32(const float* y0, int64_t ld_y0, const uint32_t* inp_bits, int64_t ld_bits,
                                     const double* coef, const int8_t* support, const int8_t* exps, int32_t n_terms,
                                     int32_t n_states, int64_t n_rows, int32_t T, double dt, int32_t method,
                                     int32_t substeps, double drop_below, float* y_out, int64_t ld_y, void* stream);

/* Counter-based random words of the on-device PK/PD cohort generator (csrc/insite_rng.hip; SURVEY.md §8
 * F3).  Replaces the words under every jax.random draw the reference makes for a cohort
 * (libs_m/ct/src/data/pkpd/dataset.py:52-54 PRNGKey(seed) per subset; pkpd_simulation.py:117-197,
 * 233-236, 290-291 split / normal / uniform / permutation): out[0 .. n_words) = jax.prng.threefry_2x32
 * ((key0, key1), iota(n_words)) -- Threefry-2x32-20 over the pairs (j, j + ceil(n/2)), the odd count
 * padded with one zero, output halves concatenated.  The uniform / normal / permutation transforms run
 * on these words in insite_amd/threefry.py.  out: device uint32 [n_words], 0 <= n_words < 2^32 - 1. */
int32_t insite_threefry2x32_iota_u32(uint32_t key0, uint32_t key1, int64_t n_words, uint32_t* out, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* INSITE_HIP_H_ */
