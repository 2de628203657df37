// insite_refine.hip — INSITE per-patient refinement on MI355X (gfx950): one lane per row, the BFGS
// optimiser state in VGPRs (sparse models) or per-lane scratch (dense ones).
//
// Reference: SINDY._get_fine_tuned_predictions / f_to_min_func / predict_with_reduced_coefs
// (libs_m/ct/src/models/sindy.py:433-715, 767-794); restatement oracle/insite_refine_ref.py.  Per row
//   f(c) = mse(c * mask) / (2.5 mse(c0)) + lam * mean((c0 - c)^2),  mask = |c0| > 1e-3,
//   mse  = mean over k < min(sl - tau, T - 1) of (V[k+1] - pred_k)^2, pred = Euler-5 scan from V[0],
// minimised by jax.scipy.optimize.minimize(method='BFGS') restated: BFGS with the inverse-Hessian update,
// strong-Wolfe line search, cubic / quadratic / bisection zoom (oracle docstring).
//
// Every model of the reference is described per global coefficient q by (arm mask, state exponent e_q,
// static monomial m_q(u)): on a step whose arm is a the RHS is the state polynomial
//   f_a(y) = sum_e gamma_{a,e} y^e,   gamma_{a,e} = sum_{q : a in mask_q, e_q = e} c_q m_q(u).
//   * separate per-arm models (sindy.py:457-467, 489-499, 523-533): q = (a, j), mask 1 << a;
//   * the joint "one ODE" model (sindy.py:469-483, 503-517, 537-551): one coefficient row whose library
//     takes the per-step binary treatments as inputs; "arm" = the step's treatment bit code, and column j
//     (x^e in^tau m(u)) acts on every code covering tau's inputs (the fold of insite_amd SINDY._fold_joint);
//   * the degree-4 library (ABLATION_MORE_COMPLEX_BASIS_FUNCTIONS, sindy.py:185-186): e_q up to 4.
// The objective depends on c only through gamma, so one forward pass with NA (D + 1) tangents
// d y / d gamma_{a,e} gives f and its exact gradient (what jax's autodiff computes):
//   d <- d (1 + h f_a'(y)) + [arm == a] h y^e,  then y <- y + h f_a(y)   (D = 1: f' = gamma_{a,1}).
// Only the m active coefficients move (inactive ones have zero data gradient and start at c0, so BFGS
// with H0 = I keeps their block fixed): the search runs in the m-dimensional active subspace.
// M <= 8: the optimiser state lives in VGPRs, every loop unrolled, inverse-Hessian update w @ H @ w.T as in
// the oracle.  M = 16 / 72 (dense global models): rolled loops (RU = 1), per-lane scratch, the O(M^2)
// update.  Measured at 200k 4-arm rows (tools/refine_arms_bench.py): M = 16 unrolled 80 ms (512 VGPRs +
// spills) vs rolled 62 ms; M = 36 rolled O(M^3) 1437 ms vs O(M^2) 108 ms; M = 8 5.5 ms.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "insite_hip.h"
#include "insite_common.h"

namespace {

constexpr int kRefineMaxCoef = 72;  // n_arms * F of a global model: the degree-4 library, 2 arms x 35 terms
#ifndef INSITE_REFINE_REG
#define INSITE_REFINE_REG 8  // largest M whose loops are fully unrolled (register-resident state)
#endif
constexpr int kRefineRegActive = INSITE_REFINE_REG;

struct RefineArgs {
  const double* V;      // [T, ldv] unscaled observations (time-major)
  const uint32_t* arm;  // TIME_MAJOR_BITS [T, lda] per-step arm (NA = 2)
  const int8_t* arm8;   // [T, lda] int8 per-step arm (NA = 4)
  const double* u;      // [N, U]
  const int32_t* sl;    // [N] sequence lengths
  double* preds;        // [T, ldp]
  double* coef_out;     // [N, n_coef] or NULL
  int32_t* status;      // [N] or NULL (-1 skipped, else the BFGS status)
  int32_t* iters;       // [N] or NULL
  int32_t* nfev;        // [N] or NULL: objective + gradient evaluations (the roofline's flop count)
  const int32_t* order; // [N] lane -> row (rows binned by seq_len), NULL = identity
  int64_t ldv, lda, ldp, N;
  int32_t T, tau, sub, U, A, m, n_coef;
  int32_t revert3;      // 1: BFGS status 3 reverts to the global model (sindy.py:628-631); 0: keep the iterate
  int32_t pm;           // 1: the row layout below (WIN kernels only)
  // row layout (insite_refine_rows_f64): V [N, ldv], arm8 [N, lda] and preds [N, ldp] patient-major, every per-row
  // array indexed by the row order[lane] selects; st16 = 16-B prediction stores (preds 16-B aligned, ldp even)
  int32_t st16;
  double dt, lam;
  // active coefficients i < m: flat index, arm mask, state exponent, static-monomial code
  int32_t t_flat[kRefineMaxCoef], t_mask[kRefineMaxCoef], t_ex[kRefineMaxCoef], t_ucode[kRefineMaxCoef];
  // every coefficient q < n_coef: arm mask, static-monomial code | state exponent << 24
  int32_t q_mask[kRefineMaxCoef], q_code[kRefineMaxCoef];
  double c0[kRefineMaxCoef];
  // the active terms' (arm, exponent) routing as ONE scalar when it fits 32 bits: bit i * 8 + a * 2 + e set when
  // active coefficient i feeds gamma_{a,e} (D = 1, NA <= 4, m <= 4) -- the objective's gamma sums and gradient
  // gathers test one SGPR instead of keeping 2m kernel-argument words live in SGPRs (which spilled into VGPR lanes)
  int32_t gmap;
};

// The kernels read RefineArgs (a by-value kernel argument, ~2.9 KB of tables) through a pointer into the kernarg
// segment (constant address space): binding a reference to the by-value parameter itself made the compiler copy
// the whole struct into per-lane scratch at kernel entry and index the copy with vector loads -- 6.3 KB of scratch
// per lane in the rolled M = 16 kernel, whose counters showed ~374 GB of HBM traffic per 1M-row launch.
typedef const __attribute__((address_space(4))) RefineArgs KArgs;
__device__ __forceinline__ KArgs& kernel_args() {
  return *(KArgs*)(__builtin_amdgcn_kernarg_segment_ptr());
}

__device__ __forceinline__ double monomial_code(int code, const double* u) {
  double m = 1.0;
#pragma unroll
  for (int i = 0; i < INSITE_MAX_STATICS; ++i) {
    const int e = (code >> (8 * i)) & 0xff;
    for (int k = 0; k < e; ++k) m *= u[i];
  }
  return m;
}

// sum_e g[e] y^e and its derivative by Horner (the oracle's _poly / _dpoly)
template <int D>
__device__ __forceinline__ double poly(const double (&g)[D + 1], double y) {
  double f = g[D];
#pragma unroll
  for (int e = D - 1; e >= 0; --e) f = g[e] + f * y;
  return f;
}
template <int D>
__device__ __forceinline__ double dpoly(const double (&g)[D + 1], double y) {
  double f = (double)D * g[D];
#pragma unroll
  for (int e = D - 1; e >= 1; --e) f = (double)e * g[e] + f * y;
  return f;
}

#ifndef INSITE_REFINE_SU4
#define INSITE_REFINE_SU4 5  // sub-step unroll of the M <= 4 kernel: 7.23 -> 7.03 ms INSITE step (profiles/r03/v30); 1 = rolled
#endif
// Windowed scans (INSITE_REFINE_WIN, T <= 64, two bit arms, M <= 4, affine RHS): the objective's targets V[k + 1]
// reach the wave through an LDS ring of kWin-step slots filled by LDS-DMA (global_load_lds_dwordx4: one instruction
// moves 2 steps x 64 rows, 1 KiB, no VGPR destination) one slot AHEAD, and each lane's arms sit in one 64-bit mask
// (no per-step loads at all).  With a one-step register prefetch every step of every scan waited on an L2 / MALL
// round trip (the kernel ran ~3x its VALU time at 3 waves per SIMD).  The ring needs the wave's lanes to run the
// scan together, so the flat loop below becomes wave-uniform in this mode (a lane with nothing pending scans 0 steps).
constexpr int kWin = 8;
#ifndef INSITE_REFINE_WIN
#define INSITE_REFINE_WIN 1
#endif

// Row layout (PM, insite_refine_rows_f64): the same ring over the reference's patient-major V gathered through the
// lane order.  A slot holds COLUMNS [8c, 8c + 8) of the wave's 64 rows (the target of step k is column k + 1); one
// LDS-DMA instruction moves 16 rows x 64 B (4 lanes x 16 B per row), and lane 4m + j of instruction q writes the
// 16-B piece ((j + m / 4) & 3) of row 16 q + m: the swizzle spreads a step's 64 reads (row r reads its own column)
// over all 64 banks, 2 passes per ds_read_b64 as in the time-major ring.
// Element (row r, column col): slot (col / 8) & 1, instruction r / 16, row r % 16 = m, and within the row's 64 B the
// piece ((col % 8) / 2 - m / 4) & 3, element col & 1 -- i.e. (col - 2 (m / 4)) & 7 (an even shift keeps the low
// bit), so a lane adds its constant pm_lane_rot to the column and masks: 3 integer ops per read.
__device__ __forceinline__ int pm_lane_base(int r) { return (r >> 4) * 128 + (r & 15) * 8; }
__device__ __forceinline__ int pm_lane_rot(int r) { return (-2 * ((r & 15) >> 2)) & 7; }
__device__ __forceinline__ int pm_slot_index(int r, int col) {
  return ((col >> 3) & 1) * (kWin * kWave) + pm_lane_base(r) + ((col + pm_lane_rot(r)) & 7);
}

// NC (`#pragma clang fp contract(off)` in a block): the per-evaluation and per-iteration sums over coefficients (gamma,
// the gradient and penalty, dot products, H g, the inverse-Hessian update, the final model's gamma) are computed
// without fused multiply-adds, so every kernel that computes them -- the one-lane-per-row kernels with their loops
// rolled or unrolled, the cooperative kernel with its values shuffled in -- rounds them identically (the compiler's
// contraction choices differed between those code shapes: ~1e-13 apart, and on ill-conditioned joint-model rows a
// different BFGS path).  The scan's per-step arithmetic stays contracted (the same code in every kernel).
// The ring's wait: the hardware wait for the LDS-DMA loads (inline asm: the compiler does not track them) AND the
// same wait as a builtin the compiler's waitcnt pass sees, so it knows its own earlier loads (the scan's y0) have
// completed too.  With the asm alone the pass kept a vmcnt(0) for y0 inside the sub-step loop -- which, executed
// with a ring prefetch in flight, waited for the prefetch every step that issued one.
// CF (INSITE_REFINE_CF, the objective scans of the affine models, D = 1): the n = ra.sub Euler sub-steps of a step
// on arm a are the affine map y <- P_a y + B_a with q = 1 + h gamma_{a,1}, P_a = q^n, B_a = h gamma_{a,0} S,
// S = sum_{j<n} q^j, and the tangents follow in closed form from the step's start y:
//   d/dgamma_{b,e} <- P_a d                         (b != a: the other arms' tangents only scale)
//   d/dgamma_{a,0} <- P_a d + h S,   d/dgamma_{a,1} <- P_a d + n h q^(n-1) y + h^2 gamma_{a,0} sum_{j<=n-2} (j+1) q^j
// (the sums of the recurrences d <- q d + h, d <- q d + h y_s over the sub-steps): one FMA per value and step instead
// of n.  The objective's rounding is the restatement's own (the oracle and the reference differentiate the sub-step
// form; jax in reverse mode): the GPU matches the oracle per row to the tests' tolerances, and the final predictions
// (sindy.py:668) keep the sub-step form.  Every kernel computing an objective uses it (the single-lane, dynamic and
// cooperative kernels stay bitwise equal to each other).
#ifndef INSITE_REFINE_CF
#define INSITE_REFINE_CF 1
#endif
#ifndef INSITE_REFINE_SCAN_UNROLL
#define INSITE_REFINE_SCAN_UNROLL 1
#endif
#ifndef INSITE_REFINE_HOIST
#define INSITE_REFINE_HOIST 1  // 1 / K and dt / sub once per row (RefineLane::setK); measured neutral (profiles/r05/scan/run_hoist)
#endif
// INSITE_REFINE_SCAN_LROT 1: the ring offset formed per step (round 5: at 3 waves per SIMD the 8 hoisted offsets cost
// ~8 VGPRs of spills); at 2 waves (round 6, no spills) the hoisted form is back: 1.642-1.656 vs 1.654-1.661 ms/step,
// interleaved on one box (profiles/r06/refine_ab2/i3_lrot0_*)
#ifndef INSITE_REFINE_SCAN_LROT
#define INSITE_REFINE_SCAN_LROT 0
#endif
// the per-arm constants of CF for one evaluation
struct CfArm {
  double P, B, hS, C1, C2;
};
__device__ __forceinline__ CfArm cf_arm(double g0, double g1, double h, int n) {
  const double q = 1.0 + h * g1;
  double pw = 1.0, S = 0.0, Cs = 0.0, qn1 = 1.0;
  for (int j = 0; j < n; ++j) {  // pw = q^j
    if (j + 1 < n) Cs = fma((double)(j + 1), pw, Cs);
    S += pw;
    qn1 = pw;
    pw *= q;
  }
  CfArm c;
  c.P = pw;
  c.B = h * g0 * S;
  c.hS = h * S;
  c.C1 = (double)n * h * qn1;
  c.C2 = h * h * g0 * Cs;
  return c;
}

// fma as the three-address VOP3 form (INSITE_REFINE_FMA3): the compiler's two-address v_fmac ties the result to the
// addend -- in the unrolled scan a fresh select -- and then moves it back to the tangent's register (5 moves a step)
#ifndef INSITE_REFINE_FMA3
#define INSITE_REFINE_FMA3 1
#endif
__device__ __forceinline__ double fma3(double a, double b, double c) {
#if INSITE_REFINE_FMA3
  double r;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
#else
  return fma(a, b, c);
#endif
}

__device__ __forceinline__ void ring_wait() {
  __builtin_amdgcn_s_waitcnt(0x0F70);  // gfx9 encoding: vmcnt(0) expcnt(7) lgkmcnt(15)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Sums over the M coordinates of the BFGS vectors (dot products, the penalty, y^T H y, |g|^2).  M = 16 (the dense
// models; INSITE_REFINE_TREE): in the association of the cooperative kernel's 8-lane group reduction -- lane j holds
// coordinates j and j + 8, then butterfly pairs (j, j^1), (j, j^2), (j, j^4) -- so the cooperative kernel takes its
// dot products with three in-group exchanges instead of 16 gathers and 16 dependent adds, and stays bitwise equal to
// this kernel; the leading 0.0 + keeps the sequential sum's +0 for an all-zero sum.  Other M: coordinate order.
#ifndef INSITE_REFINE_TREE
#define INSITE_REFINE_TREE 1
#endif
// INSITE_REFINE_FUSEDUPD (M = 16): H g and H y as FMA chains, and the inverse-Hessian update in the rank-2 form
// H + s u^T + w s^T, w = -rho H y, u = cs s + w (2 FMAs an element instead of 5 multiplies and 3 adds); the single-
// lane and cooperative kernels run the same operations (bitwise equal), the oracle's association differs as before.
#ifndef INSITE_REFINE_FUSEDUPD
#define INSITE_REFINE_FUSEDUPD 1
#endif
template <int M>
__device__ __forceinline__ double coord_sum(const double (&v)[M]) {
#pragma clang fp contract(off)  // NC
  if constexpr (M == 16 && INSITE_REFINE_TREE) {
    double l[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) l[j] = v[j] + v[j + 8];
    const double m0 = l[0] + l[1], m1 = l[2] + l[3], m2 = l[4] + l[5], m3 = l[6] + l[7];
    return 0.0 + ((m0 + m1) + (m2 + m3));
  } else {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < M; ++i) s += v[i];
    return s;
  }
}

template <int M, int NA, int D, bool WIN = false, bool PM = false>
struct RefineLane {
  static constexpr int RU = M <= kRefineRegActive ? M : 1;
  // sub-step loop unrolled by odeint's 5 (the default): measured 12 active 62 -> 43 ms, 6 active 5.5 -> 5.2 ms;
  // for M = 4 rolled was faster while the sub-step held per-lane selects (9.6 vs 10.1 ms); without them unrolled
  // wins (INSITE_REFINE_SU4); dense models stay rolled
  static constexpr int SU = (M > 4 && M <= 16) ? 5 : (M <= 4 ? INSITE_REFINE_SU4 : 1);
  static constexpr bool kGmap = M <= 4 && D == 1 && NA <= 4;  // RefineArgs::gmap holds the routing
  KArgs& ra;
  int64_t p;
  int K;
  double norm;
  double mono[M];
  double c0a[M];
  double iKv = 0.0, hv = 0.0;  // 1 / K and the sub-step dt / sub, once per row (were two divisions per evaluation)
  __device__ void setK(int k) {
    K = k;
    iKv = 1.0 / (double)k;
    hv = ra.dt / (double)ra.sub;
  }
  uint64_t am = 0;         // WIN: arm of step k in bit k
  double* win = nullptr;   // WIN: this wave's ring, 2 slots x kWin steps x 64 rows (step j of a slot at j * 64)
  int64_t p0 = 0;          // WIN: the wave's first column
  __device__ int armbit_mem(int k) const {
    if constexpr (PM) return ra.arm8[p * ra.lda + k] != 0 ? 1 : 0;
    else if constexpr (NA == 2) return (int)((ra.arm[(int64_t)k * ra.lda + (p >> 5)] >> (p & 31)) & 1u);
    else return (int)ra.arm8[(int64_t)k * ra.lda + p];
  }
  __device__ int armbit(int k) const {
    if constexpr (WIN) return (int)((am >> k) & 1ull);
    else return armbit_mem(k);
  }
  // WIN: LDS-DMA of target rows V[1 + c kWin .. c kWin + kWin] (clamped to T - 1) of the wave's 64 columns into ring
  // slot `slot`; lanes 0-31 move rows 2q + 1, lanes 32-63 rows 2q + 2, 16 B (two columns) each.  Every lane of the
  // wave must execute it (the destination is the wave-uniform slot base + lane x 16 B).
  __device__ void fill(int c, int slot) const {
    const int lane = threadIdx.x & (kWave - 1);
    if constexpr (PM) {
      const int m = lane >> 2, pk = ((lane & 3) + (m >> 2)) & 3;
      int col = c * kWin + 2 * pk;
      if (col + 2 > ra.ldv) col = 0;  // past the row's end: any in-row pair (never read: targets stop at T - 1)
      const uint32_t base = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(win + slot * (kWin * kWave)));
      const int prow = (int)p;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = __shfl(prow, 16 * q + m);
        const double* src = ra.V + (int64_t)row * ra.ldv + col;
        unsigned keep;
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(src), "s"(base + q * 1024u)
                     : "memory");
      }
      return;
    }
    int64_t col = p0 + 2 * (lane & 31);
    if (col + 1 >= ra.ldv) col = ra.ldv - 2;  // past the last column: any in-bounds pair (ldv even, never read)
    const uint32_t base = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(win + slot * (kWin * kWave)));
#pragma unroll
    for (int q = 0; q < kWin / 2; ++q) {
      int row = c * kWin + 2 * q + (lane >> 5) + 1;
      row = row < ra.T - 1 ? row : ra.T - 1;
      const double* src = ra.V + (int64_t)row * ra.ldv + col;
      unsigned keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep)
                   : "v"(src), "s"(base + q * 1024u)
                   : "memory");
    }
  }
  // f and gradient at c (active coordinates)
  mutable int nev = 0;  // evaluations of f and its gradient (each one scan of the K-step window)
  // WIN: `live` = this lane's evaluation counts (its scan runs K steps); a lane with nothing pending passes false,
  // scans 0 steps and only keeps the wave's ring loads company
  __device__ double fg(const double (&c)[M], double (&g)[M], bool live = true) const {
    nev += live ? 1 : 0;
    const auto tmk = ra.t_mask, tex = ra.t_ex;  // (the single-lane kernels call fg in divergent code: no RELOAD)
    double gam[NA][D + 1];
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int e = 0; e <= D; ++e) gam[a][e] = 0.0;
#pragma unroll RU
    for (int i = 0; i < M; ++i) {
#pragma clang fp contract(off)  // NC
      if (i >= ra.m) break;
      const double t = c[i] * mono[i];
      if constexpr (kGmap) {
#pragma unroll
        for (int a = 0; a < NA; ++a)
#pragma unroll
          for (int e = 0; e <= D; ++e)
            if ((ra.gmap >> (i * 8 + a * 2 + e)) & 1) gam[a][e] += t;
      } else {
        const int mk = tmk[i], ex = tex[i];
#pragma unroll
        for (int a = 0; a < NA; ++a)
          if ((mk >> a) & 1)
#pragma unroll
            for (int e = 0; e <= D; ++e)
              if (ex == e) gam[a][e] += t;
      }
    }
    const double h = INSITE_REFINE_HOIST ? hv : ra.dt / (double)ra.sub;
    double y = PM ? ra.V[p * ra.ldv] : ra.V[p];
    double d[NA][D + 1], gG[NA][D + 1];
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int e = 0; e <= D; ++e) d[a][e] = gG[a][e] = 0.0;
    double L = 0.0;
    const int Kl = live ? K : 0;
    int Kw = Kl;      // WIN: the wave's longest scan (rows binned by seq_len: ~every lane's)
    int nch = 0;
    if constexpr (WIN) {
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) Kw = max(Kw, __shfl_xor(Kw, off));
      nch = PM ? (Kw > 0 ? Kw / kWin + 1 : 0) : (Kw + kWin - 1) / kWin;  // PM: column chunks 0 .. Kw / kWin
      // chunk 0 waited for here, unconditionally (with y0: the compiler then knows no load of its own is pending
      // inside the loop), chunk 1 prefetched; the loop waits at each later chunk boundary
      if (nch > 0) fill(0, 0);
      ring_wait();
      if (nch > 1) fill(1, 1);
    }
    // (non-WIN) step k's arm and target are requested one step ahead (issued before step k - 1's sub-steps) so the
    // dependent Euler chain does not wait on a load per step
    int ak_nx = WIN ? 0 : armbit(0);
    double v_nx = WIN ? 0.0 : ra.V[ra.ldv + p];
    const int kend = WIN ? (PM ? Kw : nch * kWin) : Kl;
    const int lbase = PM ? pm_lane_base(threadIdx.x & (kWave - 1)) : 0, lrot = PM ? pm_lane_rot(threadIdx.x & (kWave - 1)) : 0;
    constexpr bool kCf = INSITE_REFINE_CF && D == 1;
    CfArm cfa[kCf ? NA : 1];
    if constexpr (kCf) {
#pragma unroll
      for (int a = 0; a < NA; ++a) cfa[a] = cf_arm(gam[a][0], gam[a][1], h, ra.sub);
    }
    // INSITE_REFINE_SCAN_UNROLL (the row kernel's closed-form scan, WIN + PM, two arms): the loop runs over the ring's
    // column chunks and unrolls a chunk's 8 columns, so a step's column, ring offset and arm bit are compile-time
    // pieces (no loop-carried register rotation, the chunk check once per chunk) and the arm's constants are chosen
    // by selects instead of a divergent branch -- the same operations in the same order as the loop below
    constexpr bool kUnr = INSITE_REFINE_SCAN_UNROLL && WIN && PM && kCf && NA == 2;
    if constexpr (kUnr) {
      for (int c = 0; c < nch; ++c) {
        if (c > 0) {  // column chunk c landed; start the next one
          ring_wait();
          if (c + 1 < nch) fill(c + 1, (c + 1) & 1);
        }
        const double* ws = win + (c & 1) * (kWin * kWave) + lbase;
        const uint32_t amc = (uint32_t)(c == 0 ? (am << 1) : (am >> (kWin * c - 1)));  // bit j: arm of step 8c + j - 1
#pragma unroll
        for (int j = 0; j < kWin; ++j) {
          const int k = kWin * c + j - 1;
          if (k < 0 || k >= Kw) continue;  // wave-uniform
          if (k < Kl) {
            const bool a1 = ((amc >> j) & 1u) != 0u;
            int lr = lrot;
#if INSITE_REFINE_SCAN_LROT
            asm("" : "+v"(lr));  // the ring offset formed per step: 8 hoisted offsets held ~8 more VGPRs (spills)
#endif
            const double vk1 = ws[(j + lr) & (kWin - 1)];
            // only P and B are selected: each arm's own source terms come from its own constants (the inactive
            // arm's C1 y + C2 is formed and dropped), the active arm's values are the loop's
            const double P = a1 ? cfa[1].P : cfa[0].P, B = a1 ? cfa[1].B : cfa[0].B;
            const double a1v0 = fma(cfa[0].C1, y, cfa[0].C2), a1v1 = fma(cfa[1].C1, y, cfa[1].C2);
            d[0][0] = fma3(P, d[0][0], a1 ? 0.0 : cfa[0].hS);
            d[0][1] = fma3(P, d[0][1], a1 ? 0.0 : a1v0);
            d[1][0] = fma3(P, d[1][0], a1 ? cfa[1].hS : 0.0);
            d[1][1] = fma3(P, d[1][1], a1 ? a1v1 : 0.0);
            y = fma3(P, y, B);
            const double r = vk1 - y;
            L = fma(r, r, L);
            const double r2 = -2.0 * r;
#pragma unroll
            for (int a = 0; a < NA; ++a)
#pragma unroll
              for (int e = 0; e <= D; ++e) gG[a][e] = fma(r2, d[a][e], gG[a][e]);
          }
        }
      }
    }
    for (int k = 0; k < (kUnr ? 0 : kend); ++k) {
      int ak;
      double vk1;
      if constexpr (WIN && PM) {
        const int col = k + 1;
        if ((col & (kWin - 1)) == 0) {  // column chunk col / kWin landed; start the next one
          ring_wait();
          const int nx = col / kWin + 1;
          if (nx < nch) fill(nx, nx & 1);
        }
        if (k >= Kl) continue;
        ak = armbit(k);
        vk1 = win[((col >> 3) & 1) * (kWin * kWave) + lbase + ((col + lrot) & 7)];
      } else if constexpr (WIN) {
        if (k > 0 && (k & (kWin - 1)) == 0) {  // slot k / kWin landed; start the next one into the other slot
          ring_wait();
          if (k / kWin + 1 < nch) fill(k / kWin + 1, (k / kWin + 1) & 1);
        }
        if (k >= Kl) continue;
        ak = armbit(k);
        vk1 = win[((k / kWin) & 1) * (kWin * kWave) + (k & (kWin - 1)) * kWave + (threadIdx.x & (kWave - 1))];
      } else {
        ak = ak_nx;
        vk1 = v_nx;
        if (k + 1 < Kl) {
          ak_nx = armbit(k + 1);
          v_nx = ra.V[(int64_t)(k + 2) * ra.ldv + p];
        }
      }
      double gk[D + 1];
#pragma unroll
      for (int e = 0; e <= D; ++e) gk[e] = gam[0][e];
#pragma unroll
      for (int a = 1; a < NA; ++a)
        if (ak == a)
#pragma unroll
          for (int e = 0; e <= D; ++e) gk[e] = gam[a][e];
      if constexpr (kCf) {
        CfArm c = cfa[0];
#pragma unroll
        for (int a = 1; a < NA; ++a)
          if (ak == a) c = cfa[a];
        const double a1 = fma(c.C1, y, c.C2);
#pragma unroll
        for (int a = 0; a < NA; ++a) {
          d[a][0] = fma(c.P, d[a][0], ak == a ? c.hS : 0.0);
          d[a][1] = fma(c.P, d[a][1], ak == a ? a1 : 0.0);
        }
        y = fma(c.P, y, c.B);
      } else if constexpr (D == 1) {
        const double hb = h * gk[1];
        // the step's arm selects its tangent's source term once per step, not per sub-step: an inactive arm
        // adds +0.0 and 0 * y (bitwise the untouched value for finite y), so the sub-step loop has no
        // per-lane selects (8 v_cndmask of 18 VALU per sub-step before)
        double ha[NA];
#pragma unroll
        for (int a = 0; a < NA; ++a) ha[a] = (ak == a) ? h : 0.0;
#pragma unroll SU
        for (int s = 0; s < ra.sub; ++s) {
#pragma unroll
          for (int a = 0; a < NA; ++a) {
            // explicit fused forms (the cooperative kernel computes the same chain: see NC)
            d[a][0] = fma(hb, d[a][0], d[a][0]) + ha[a];
            d[a][1] = fma(ha[a], y, fma(hb, d[a][1], d[a][1]));
          }
          y = fma(h, fma(gk[1], y, gk[0]), y);
        }
      } else {
        for (int s = 0; s < ra.sub; ++s) {
          const double hf = h * dpoly<D>(gk, y);
#pragma unroll
          for (int a = 0; a < NA; ++a) {
            double ye = 1.0;
#pragma unroll
            for (int e = 0; e <= D; ++e) {
              d[a][e] = d[a][e] + hf * d[a][e];
              if (ak == a) d[a][e] += h * ye;
              ye *= y;
            }
          }
          y = y + h * poly<D>(gk, y);
        }
      }
      const double r = vk1 - y;
      L = fma(r, r, L);
      const double r2 = -2.0 * r;
#pragma unroll
      for (int a = 0; a < NA; ++a)
#pragma unroll
        for (int e = 0; e <= D; ++e) gG[a][e] = fma(r2, d[a][e], gG[a][e]);
    }
    const double iK = INSITE_REFINE_HOIST ? iKv : 1.0 / (double)K;   // (a non-live WIN lane: its own K; values unused)
    L *= iK;
    double pen = 0.0, sq[M];
#pragma unroll RU
    for (int i = 0; i < M; ++i) {
#pragma clang fp contract(off)  // NC
      sq[i] = 0.0;
      if (i >= ra.m) {
        g[i] = 0.0;
        continue;
      }
      const double dd = c0a[i] - c[i];
      if constexpr (M == 16 && INSITE_REFINE_TREE) sq[i] = dd * dd;
      else pen += dd * dd;
      double gd = 0.0;
      if constexpr (kGmap) {
#pragma unroll
        for (int a = 0; a < NA; ++a)
#pragma unroll
          for (int e = 0; e <= D; ++e)
            if ((ra.gmap >> (i * 8 + a * 2 + e)) & 1) gd += gG[a][e];
      } else {
        const int mk = tmk[i], ex = tex[i];
#pragma unroll
        for (int a = 0; a < NA; ++a)
          if ((mk >> a) & 1)
#pragma unroll
            for (int e = 0; e <= D; ++e)
              if (ex == e) gd += gG[a][e];
      }
      g[i] = gd * iK * mono[i] / norm + 2.0 * ra.lam * (c[i] - c0a[i]) / (double)ra.n_coef;
    }
    if constexpr (M == 16 && INSITE_REFINE_TREE) pen = coord_sum(sq);
    return L / norm + ra.lam * pen / (double)ra.n_coef;
  }
  __device__ double dot(const double (&a)[M], const double (&b)[M]) const {
#pragma clang fp contract(off)  // NC
    double pr[M];
#pragma unroll RU
    for (int i = 0; i < M; ++i) pr[i] = a[i] * b[i];
    return coord_sum(pr);
  }
  // phi(t) = f(x + t pk), dphi = g . pk
  __device__ double phi(const double (&x)[M], const double (&pk)[M], double t, double& dphi, double (&g)[M],
                        bool live = true) const {
    double xt[M];
#pragma unroll RU
    for (int i = 0; i < M; ++i) xt[i] = fma(t, pk[i], x[i]);
    const double f = fg(xt, g, live);
    dphi = dot(g, pk);
    return f;
  }
};

__device__ __forceinline__ double cubicmin(double a, double fa, double fpa, double b, double fb, double c, double fc) {
  const double C = fpa, db = b - a, dc = c - a;
  const double denom = (db * dc) * (db * dc) * (db - dc);
  const double A = (dc * dc * (fb - fa - C * db) + (-db * db) * (fc - fa - C * dc)) / denom;
  const double B = ((-dc * dc * dc) * (fb - fa - C * db) + (db * db * db) * (fc - fa - C * dc)) / denom;
  const double radical = B * B - 3.0 * A * C;
  return a + (-B + sqrt(radical)) / (3.0 * A);
}
__device__ __forceinline__ double quadmin(double a, double fa, double fpa, double b, double fb) {
  const double db = b - a;
  const double B = (fb - fa - fpa * db) / (db * db);
  return a - fpa / (2.0 * B);
}

// waves per SIMD of the M <= 4 affine kernels.  r04: 3 waves (<= 168 VGPRs) beat 4 with spills (kernel 2.21 vs 2.30 ms,
// flat BFGS) and 2 (2.01 vs 1.89 ms/step after the closed-form scans); r06: after the round-5 scan
// unroll the 3-wave M = 3 row kernel held 30 spilled VGPRs (scratch writes ~0.65 GB a launch), and 2 waves without
// spills measured 1.667-1.674 vs 1.724-1.730 ms/step on one box, interleaved (profiles/r06/refine_ab/) -- so 2.  (The
// per-lane LDS table of the arm constants the verdict named does not fit at 3 waves: H columns 18 KB + the ring 32 KB
// per 256-thread block = 150 of the CU's 160 KB at 3 blocks; the 10 constants would add 20 KB a block.)
#ifndef INSITE_REFINE_WPE4
#define INSITE_REFINE_WPE4 2
#endif
#ifndef INSITE_REFINE_WPE8
#define INSITE_REFINE_WPE8 1
#endif
#ifndef INSITE_REFINE_FLAT
#define INSITE_REFINE_FLAT 1  // the BFGS as a flat per-lane state machine (one scan per loop iteration)
#endif
#ifndef INSITE_REFINE_QUAD
#define INSITE_REFINE_QUAD 0  // 1: the O(M^2) inverse-Hessian update for the unrolled kernels too
#endif
// The inverse Hessian of the M <= 4 kernels lives in LDS (INSITE_REFINE_HLDS, one [M*M] column of doubles per lane,
// kBlock-strided: conflict-free): it is read once per iteration (p = -H g) and written once (the update), while
// the line search -- ~12 objective scans per row, each a dependent fp64 chain -- needs every VGPR it can get.  In
// VGPRs the 4-coefficient kernel at INSITE_REFINE_WPE4 = 4 waves/SIMD (<= 128 VGPRs) spilled 156 VGPRs to scratch
// (316 B/lane): PMC 13.6 GB of traffic per launch against 1.1 GB algorithmic (profiles/traffic_r03.json).
#ifndef INSITE_REFINE_HLDS
#define INSITE_REFINE_HLDS 1
#endif
template <int M, bool LDS>
struct HMat {
  double v[M][M];
  __device__ __forceinline__ double& at(int i, int j) { return v[i][j]; }
};
template <int M>
struct HMat<M, true> {
  double* base;  // &sH[threadIdx.x]; element (i, j) at base[(i * M + j) * kBlock]
  __device__ __forceinline__ double& at(int i, int j) { return base[(i * M + j) * kBlock]; }
};

// jax minimize_bfgs + line_search + _zoom as a flat per-lane state machine (INSITE_REFINE_FLAT): its state in one
// struct, advanced once per objective evaluation (insite_refine_kernel; insite_refine_dyn_kernel restarts it per row)
template <int M, bool kHL, int RU, class Lane>
struct BfgsFlat {
  HMat<M, kHL> H;
  double x[M], g[M], pk[M], g_star[M];
  double f, old_old, phi0, dphi0, a_i1, phi_i1, dphi_i1, a_star, phi_star;
  double a_lo, phi_lo, dphi_lo, a_hi, phi_hi, dphi_hi, a_rec, phi_rec, za, zphi, t_trial;
  int li, zj, k, ls_status;
  bool ls_failed, in_zoom, z_failed, converged, failed;
  __device__ void begin_ls(const Lane& ln) {
#pragma clang fp contract(off)  // NC
#pragma unroll RU
    for (int i = 0; i < M; ++i) {
      double s_ = 0.0;
#pragma unroll RU
      for (int j = 0; j < M; ++j) {
        if constexpr (M == 16 && INSITE_REFINE_FUSEDUPD) s_ = fma(H.at(i, j), g[j], s_);
        else s_ += H.at(i, j) * g[j];
      }
      pk[i] = -s_;
    }
    phi0 = f;
    dphi0 = ln.dot(g, pk);
    const double cand = 1.01 * 2.0 * (phi0 - old_old) / dphi0;
    t_trial = cand > 1.0 ? 1.0 : cand;
    li = 1;
    a_i1 = 0.0;
    phi_i1 = phi0;
    dphi_i1 = dphi0;
    a_star = 0.0;
    phi_star = phi0;
#pragma unroll RU
    for (int i = 0; i < M; ++i) g_star[i] = g[i];
    ls_failed = false;
    in_zoom = false;
  }
  __device__ void zoom_top() {
#pragma clang fp contract(off)  // NC
    const double dalpha = a_hi - a_lo;
    const double lo = fmin(a_hi, a_lo), hi = fmax(a_hi, a_lo);
    const double cchk = 0.2 * dalpha, qchk = 0.1 * dalpha;
    z_failed = z_failed || (dalpha <= 1e-10);
    const double a_cub = cubicmin(a_lo, phi_lo, dphi_lo, a_hi, phi_hi, a_rec, phi_rec);
    const bool use_cubic = (zj > 0) && (a_cub > lo + cchk) && (a_cub < hi - cchk);
    const double a_quad = quadmin(a_lo, phi_lo, dphi_lo, a_hi, phi_hi);
    const bool use_quad = !use_cubic && (a_quad > lo + qchk) && (a_quad < hi - qchk);
    double a_j = a_rec;
    if (use_cubic) a_j = a_cub;
    if (use_quad) a_j = a_quad;
    if (!use_cubic && !use_quad) a_j = (a_lo + a_hi) / 2.0;
    t_trial = a_j;
  }
  // the first evaluation s, gs (at c0, norm 1) -> minimize_bfgs's initial state; returns whether a trial is pending
  __device__ bool start(double s, const double (&gs)[M], Lane& ln, int maxiter) {
#pragma clang fp contract(off)  // NC
    ln.norm = s * 2.5;
    f = s / ln.norm + 0.0;
#pragma unroll RU
    for (int i = 0; i < M; ++i) g[i] = gs[i] / ln.norm + 0.0;
#pragma unroll RU
    for (int i = 0; i < M; ++i)
#pragma unroll RU
      for (int j = 0; j < M; ++j) H.at(i, j) = i == j ? 1.0 : 0.0;
    double gmax = 0.0, g2 = 0.0, gsq[M];
#pragma unroll RU
    for (int i = 0; i < M; ++i) {
      gmax = fmax(gmax, fabs(g[i]));
      gsq[i] = g[i] * g[i];
    }
    g2 = coord_sum(gsq);
    converged = gmax < 1e-5;
    failed = false;
    old_old = f + sqrt(g2) / 2.0;
    ls_status = 0;
    k = 0;
    const bool pending = !converged && k < maxiter;
    if (pending) begin_ls(ln);
    return pending;
  }
  // one trial's value / slope / gradient -> the next state (insite_refine_kernel's FLAT loop body); returns pending
  __device__ bool advance(double phi_t, double dphi_t, const double (&g_t)[M], const Lane& ln, int maxiter) {
#pragma clang fp contract(off)  // NC
    bool ls_end = false, ls_done = false, next_zoom = false;
    if (!in_zoom) {
      const double a_i = t_trial;
      const bool s_z1 = (phi_t > phi0 + 1e-4 * a_i * dphi0) || ((phi_t >= phi_i1) && (li > 1));
      const bool s_i = (fabs(dphi_t) <= -0.9 * dphi0) && !s_z1;
      const bool s_z2 = (dphi_t >= 0.0) && !s_z1 && !s_i;
      if (s_i) {
        a_star = a_i;
        phi_star = phi_t;
#pragma unroll RU
        for (int i = 0; i < M; ++i) g_star[i] = g_t[i];
      }
      if (s_z1 || s_z2) {
        if (s_z1) {
          a_lo = a_i1; phi_lo = phi_i1; dphi_lo = dphi_i1;
          a_hi = a_i; phi_hi = phi_t; dphi_hi = dphi_t;
        } else {
          a_lo = a_i; phi_lo = phi_t; dphi_lo = dphi_t;
          a_hi = a_i1; phi_hi = phi_i1; dphi_hi = dphi_i1;
        }
        zj = 0;
        z_failed = false;
        a_rec = (a_lo + a_hi) / 2.0;
        phi_rec = (phi_lo + phi_hi) / 2.0;
        za = 1.0;
        zphi = phi_lo;
#pragma unroll RU
        for (int i = 0; i < M; ++i) g_star[i] = g[i];
        in_zoom = true;
      }
      ++li;
      a_i1 = a_i;
      phi_i1 = phi_t;
      dphi_i1 = dphi_t;
      if (in_zoom) {
        next_zoom = true;
      } else if (s_i) {
        ls_end = ls_done = true;
      } else if (li > 10) {
        ls_end = true;
      } else {
        t_trial = a_i1 * 2.0;
      }
    } else {
      const double a_j = t_trial;
      const bool hi_to_j = (phi_t > phi0 + 1e-4 * a_j * dphi0) || (phi_t >= phi_lo);
      const bool star_to_j = (fabs(dphi_t) <= -0.9 * dphi0) && !hi_to_j;
      const bool hi_to_lo = (dphi_t * (a_hi - a_lo) >= 0.0) && !hi_to_j && !star_to_j;
      const bool lo_to_j = !hi_to_j && !star_to_j;
      if (hi_to_j) {
        a_rec = a_hi;
        phi_rec = phi_hi;
        a_hi = a_j;
        phi_hi = phi_t;
        dphi_hi = dphi_t;
      }
      if (star_to_j) {
        za = a_j;
        zphi = phi_t;
#pragma unroll RU
        for (int i = 0; i < M; ++i) g_star[i] = g_t[i];
      }
      if (hi_to_lo) {
        a_rec = a_hi;
        phi_rec = phi_hi;
        a_hi = a_lo;
        phi_hi = phi_lo;
        dphi_hi = dphi_lo;
      }
      if (lo_to_j) {
        a_rec = a_lo;
        phi_rec = phi_lo;
        a_lo = a_j;
        phi_lo = phi_t;
        dphi_lo = dphi_t;
      }
      ++zj;
      z_failed = ((z_failed ? 1 : 0) | zj) >= 30;  // jax: `failed | j >= 30` (no parentheses)
      if (star_to_j || z_failed) {
        a_star = za;
        phi_star = zphi;
        ls_failed = ls_failed || z_failed;
        ls_end = ls_done = true;
      } else {
        next_zoom = true;
      }
    }
    // the next zoom trial, from either branch: ONE copy of zoom_top (its five divisions and a square root), so a wave
    // whose lanes are in both phases issues it once rather than twice
    if (next_zoom) zoom_top();
    if (!ls_end) return true;
    ls_status = ls_failed ? 1 : (li > 10 ? 3 : 0);
    failed = ls_failed || !ls_done;
    return update(ln, maxiter);
  }
  // the inverse-Hessian update and the next iterate (minimize_bfgs after its line search)
  __device__ bool update(const Lane& ln, int maxiter) {
#pragma clang fp contract(off)  // NC
    double sk[M], yk[M];
#pragma unroll RU
    for (int i = 0; i < M; ++i) {
      sk[i] = a_star * pk[i];
      yk[i] = g_star[i] - g[i];
    }
    const double rho = 1.0 / ln.dot(yk, sk);
    if constexpr (RU == 1 || INSITE_REFINE_QUAD) {  // (compile-time: the rolled kernels never hold the WH temporary)
     if (isfinite(rho)) {
      double hy[M], yh[M];
#pragma unroll RU
      for (int i = 0; i < M; ++i) {
        double t = 0.0;
#pragma unroll RU
        for (int j = 0; j < M; ++j) {
          if constexpr (M == 16 && INSITE_REFINE_FUSEDUPD) t = fma(H.at(i, j), yk[j], t);
          else t += H.at(i, j) * yk[j];
        }
        hy[i] = t;
        yh[i] = yk[i] * t;
      }
      const double yhy = coord_sum(yh);
      const double cs = rho * rho * yhy + rho;
      if constexpr (M == 16 && INSITE_REFINE_FUSEDUPD) {
        double w[M], u[M];
#pragma unroll RU
        for (int i = 0; i < M; ++i) {
          w[i] = -rho * hy[i];
          u[i] = fma(cs, sk[i], w[i]);
        }
#pragma unroll RU
        for (int i = 0; i < M; ++i)
#pragma unroll RU
          for (int j = 0; j < M; ++j) H.at(i, j) = fma(sk[i], u[j], fma(w[i], sk[j], H.at(i, j)));
      } else {
#pragma unroll RU
      for (int i = 0; i < M; ++i)
#pragma unroll RU
        for (int j = 0; j < M; ++j)
          H.at(i, j) = H.at(i, j) - rho * (sk[i] * hy[j] + hy[i] * sk[j]) + cs * (sk[i] * sk[j]);
      }
     }
    } else if (isfinite(rho)) {
      auto w = [&](int i, int q) { return (i == q ? 1.0 : 0.0) - rho * (sk[i] * yk[q]); };
      double WH[M][M];
#pragma unroll RU
      for (int i = 0; i < M; ++i)
#pragma unroll RU
        for (int j = 0; j < M; ++j) {
          double s_ = 0.0;
#pragma unroll RU
          for (int q = 0; q < M; ++q) s_ += w(i, q) * H.at(q, j);
          WH[i][j] = s_;
        }
#pragma unroll RU
      for (int i = 0; i < M; ++i)
#pragma unroll RU
        for (int j = 0; j < M; ++j) {
          double s_ = 0.0;
#pragma unroll RU
          for (int q = 0; q < M; ++q) s_ += WH[i][q] * w(j, q);
          H.at(i, j) = s_ + rho * (sk[i] * sk[j]);
        }
    }
    double gm = 0.0;
#pragma unroll RU
    for (int i = 0; i < M; ++i) {
      x[i] = x[i] + sk[i];
      g[i] = g_star[i];
      gm = fmax(gm, fabs(g[i]));
    }
    converged = gm < 1e-5;
    old_old = f;
    f = phi_star;
    ++k;
    const bool pending = !converged && !failed && k < maxiter;
    if (pending) begin_ls(ln);
    return pending;
  }
};

// M <= 4 with the affine RHS (the EQ_4 models: two terms per arm) is sized for INSITE_REFINE_WPE4 waves per
// SIMD (<= 128 VGPRs; unconstrained the compiler takes 202 and runs 2 waves): the objective scan is a
// dependent fp64 chain per lane, hidden only by other waves.
template <int M, int NA, int D, bool WIN = false, bool PM = false>
__global__ void __launch_bounds__(kBlock)
__attribute__((amdgpu_waves_per_eu(M <= 4 && D == 1 ? INSITE_REFINE_WPE4 : (M <= 8 ? INSITE_REFINE_WPE8 : 1))))
insite_refine_kernel(RefineArgs) {
  KArgs& ra = kernel_args();  // (the parameter itself is never named: see KArgs)
  constexpr int RU = RefineLane<M, NA, D, WIN, PM>::RU;
  constexpr bool kHL = INSITE_REFINE_HLDS && RU == M && M <= 4;
  __shared__ double sH[(kHL ? M * M : 1) * kBlock];
  __shared__ double sV[WIN ? kWavesPerBlock * 2 * kWin * kWave : 1];
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // WIN: every lane of a wave stays (the ring loads are wave-cooperative); lanes past the last row are inert
  const bool valid = gid < ra.N;
  if (!WIN && !valid) return;
  // lane -> row: with rows binned by seq_len the lanes of a wave scan similar prefixes; every row's
  // computation is independent of its lane, so outputs are bitwise the same in any order
  const int64_t gl = valid ? gid : ra.N - 1;
  const int64_t p = ra.order ? (int64_t)ra.order[gl] : gl;
  double uu[INSITE_MAX_STATICS];
#pragma unroll
  for (int t = 0; t < INSITE_MAX_STATICS; ++t) uu[t] = t < ra.U ? ra.u[p * ra.U + t] : 0.0;
  RefineLane<M, NA, D, WIN, PM> ln{ra, p, 0, 1.0, {}, {}};
  if constexpr (WIN) {
    for (int k = 0; k < ra.T; ++k) ln.am |= (uint64_t)ln.armbit_mem(k) << k;
    ln.win = sV + (threadIdx.x / kWave) * (2 * kWin * kWave);
    ln.p0 = gid - (threadIdx.x & (kWave - 1));
  }
#pragma unroll RU
  for (int i = 0; i < M; ++i) {
    ln.mono[i] = i < ra.m ? monomial_code(ra.t_ucode[i], uu) : 0.0;
    ln.c0a[i] = i < ra.m ? ra.c0[ra.t_flat[i]] : 0.0;
  }
  double x[M];
#pragma unroll RU
  for (int i = 0; i < M; ++i) x[i] = ln.c0a[i];
  const int sl = valid ? ra.sl[p] : 0;
  int status = -1, nit = 0;
#if INSITE_REFINE_FLAT
  // ---------------- BFGS as a flat per-lane state machine: ONE objective scan per loop iteration ----------------
  // The nested form (line search loop { scan; zoom loop { scan } }) makes a wave walk the nesting of ALL its lanes:
  // lanes zooming and lanes doubling their trial step, lanes in their 3rd BFGS iteration and lanes in their 7th,
  // run their scans one after the other while the others wait.  Here every iteration of the single loop evaluates
  // each pending lane's next trial point (a line-search step a_i or a zoom step a_j) in the same scan, then
  // advances that lane's state (jax line_search / _zoom / minimize_bfgs transitions, in their order), so a wave
  // costs max over its lanes of the evaluation count instead of the sum over the nesting.  Per lane the arithmetic
  // is the nested form's, operation for operation (A/B: INSITE_REFINE_FLAT=0).
  const bool refine = sl > ra.tau && ra.T >= 2;  // (WIN: every lane enters; the inert ones scan nothing)
  if (WIN || refine) {
    ln.setK(refine ? min(sl - ra.tau, ra.T - 1) : 0);
    BfgsFlat<M, kHL, RU, RefineLane<M, NA, D, WIN, PM>> B;
    if constexpr (kHL) B.H.base = sH + threadIdx.x;
#pragma unroll RU
    for (int i = 0; i < M; ++i) {
      B.x[i] = x[i];
      B.pk[i] = 0.0;
    }
    B.t_trial = 0.0;
    double g[M];
    // jax evaluates f_to_min at c0 twice (start_res with norm_const = 1, then minimize's first value_and_grad with
    // norm_const = 2.5 start_res, sindy.py:591-627).  At c0 the penalty and its gradient are exactly zero, so the
    // second evaluation is the first divided by norm -- bitwise (fg's last operations are that one division plus
    // +0.0) -- and its scan is not repeated (BfgsFlat::start).
    const double start = ln.fg(B.x, g, refine);  // norm 1, penalty 0 at c0
    const int maxiter = 200 * ra.n_coef;
    bool pending = B.start(start, g, ln, maxiter) && refine;
    // WIN: the loop runs while ANY lane of the wave has a trial pending (its scans fill the shared ring)
    while (WIN ? __builtin_amdgcn_ballot_w64(pending) != 0 : pending) {
      double dphi_t, g_t[M];
      const double phi_t = ln.phi(B.x, B.pk, B.t_trial, dphi_t, g_t, pending);
      if (WIN && !pending) continue;
      pending = B.advance(phi_t, dphi_t, g_t, ln, maxiter);
    }
    if (refine) {
      nit = B.k;
      status = B.converged ? 0 : (B.k == maxiter ? 1 : (B.failed ? 2 + B.ls_status : -1));
#pragma unroll RU
      for (int i = 0; i < M; ++i)  // zoom failed: the reference code keeps the global coefficients (sindy.py:628-631)
        x[i] = (status == 3 && ra.revert3) ? ln.c0a[i] : B.x[i];
    }
  }
#else
  if (sl > ra.tau && ra.T >= 2) {
    ln.setK(min(sl - ra.tau, ra.T - 1));
    double g[M];
    const double start = ln.fg(x, g);  // norm 1, penalty 0 at c0
    ln.norm = start * 2.5;
    // jax evaluates f_to_min at c0 twice (start_res with norm_const = 1, then minimize's first value_and_grad with
    // norm_const = 2.5 start_res, sindy.py:591-627).  At c0 the penalty and its gradient are exactly zero, so the
    // second evaluation is the first divided by norm -- bitwise (fg's last operations are that one division plus
    // +0.0) -- and its scan is not repeated.
    // ---------------- BFGS (jax minimize_bfgs, norm = inf, gtol 1e-5) ----------------
    HMat<M, kHL> H;
    if constexpr (kHL) H.base = sH + threadIdx.x;
#pragma unroll RU
    for (int i = 0; i < M; ++i)
#pragma unroll RU
      for (int j = 0; j < M; ++j) H.at(i, j) = i == j ? 1.0 : 0.0;
    double f = start / ln.norm + 0.0;
#pragma unroll RU
    for (int i = 0; i < M; ++i) g[i] = g[i] / ln.norm + 0.0;
    double gmax = 0.0, gsq[M];
#pragma unroll RU
    for (int i = 0; i < M; ++i) {
      gmax = fmax(gmax, fabs(g[i]));
      gsq[i] = g[i] * g[i];
    }
    const double g2 = coord_sum(gsq);
    bool converged = gmax < 1e-5, failed = false;
    double old_old = f + sqrt(g2) / 2.0;
    int ls_status = 0;
    const int maxiter = 200 * ra.n_coef;
    int k = 0;
    while (!converged && !failed && k < maxiter) {
      double pk[M];
#pragma unroll RU
      for (int i = 0; i < M; ++i) {
        double s = 0.0;
#pragma unroll RU
        for (int j = 0; j < M; ++j) s += H.at(i, j) * g[j];
        pk[i] = -s;
      }
      // ---- line search (jax line_search, c1 1e-4, c2 0.9, maxiter 10) ----
      const double phi0 = f, dphi0 = ln.dot(g, pk);
      const double cand = 1.01 * 2.0 * (phi0 - old_old) / dphi0;
      const double start_a = cand > 1.0 ? 1.0 : cand;
      bool ls_done = false, ls_failed = false;
      int li = 1;
      double a_i1 = 0.0, phi_i1 = phi0, dphi_i1 = dphi0;
      double a_star = 0.0, phi_star = phi0;
      double g_star[M];
#pragma unroll RU
      for (int i = 0; i < M; ++i) g_star[i] = g[i];
      auto wolfe_one = [&](double a_, double ph) { return ph > phi0 + 1e-4 * a_ * dphi0; };
      auto wolfe_two = [&](double dph) { return fabs(dph) <= -0.9 * dphi0; };
      // zoom between (lo, hi); returns failure, fills the star point on success
      auto zoom = [&](double a_lo, double phi_lo, double dphi_lo, double a_hi, double phi_hi, double dphi_hi,
                      bool& z_failed) {
        bool done = false;
        z_failed = false;
        int j = 0;
        double a_rec = (a_lo + a_hi) / 2.0, phi_rec = (phi_lo + phi_hi) / 2.0;
        double za = 1.0, zphi = phi_lo;
        // the zoom's star gradient starts as the line search's g_0 (jax _zoom: g_star = g_0) and is the line
        // search's result: kept in g_star itself (no third gradient array live across the objective scans)
#pragma unroll RU
        for (int i = 0; i < M; ++i) g_star[i] = g[i];
        while (!done && !z_failed) {
          const double dalpha = a_hi - a_lo;
          const double lo = fmin(a_hi, a_lo), hi = fmax(a_hi, a_lo);
          const double cchk = 0.2 * dalpha, qchk = 0.1 * dalpha;
          z_failed = z_failed || (dalpha <= 1e-10);
          const double a_cub = cubicmin(a_lo, phi_lo, dphi_lo, a_hi, phi_hi, a_rec, phi_rec);
          const bool use_cubic = (j > 0) && (a_cub > lo + cchk) && (a_cub < hi - cchk);
          const double a_quad = quadmin(a_lo, phi_lo, dphi_lo, a_hi, phi_hi);
          const bool use_quad = !use_cubic && (a_quad > lo + qchk) && (a_quad < hi - qchk);
          double a_j = a_rec;
          if (use_cubic) a_j = a_cub;
          if (use_quad) a_j = a_quad;
          if (!use_cubic && !use_quad) a_j = (a_lo + a_hi) / 2.0;
          double dphi_j, g_j[M];
          const double phi_j = ln.phi(x, pk, a_j, dphi_j, g_j);
          const bool hi_to_j = wolfe_one(a_j, phi_j) || (phi_j >= phi_lo);
          const bool star_to_j = wolfe_two(dphi_j) && !hi_to_j;
          const bool hi_to_lo = (dphi_j * (a_hi - a_lo) >= 0.0) && !hi_to_j && !star_to_j;
          const bool lo_to_j = !hi_to_j && !star_to_j;
          if (hi_to_j) {
            a_rec = a_hi;
            phi_rec = phi_hi;
            a_hi = a_j;
            phi_hi = phi_j;
            dphi_hi = dphi_j;
          }
          done = done || star_to_j;
          if (star_to_j) {
            za = a_j;
            zphi = phi_j;
#pragma unroll RU
            for (int i = 0; i < M; ++i) g_star[i] = g_j[i];
          }
          if (hi_to_lo) {
            a_rec = a_hi;
            phi_rec = phi_hi;
            a_hi = a_lo;
            phi_hi = phi_lo;
            dphi_hi = dphi_lo;
          }
          if (lo_to_j) {
            a_rec = a_lo;
            phi_rec = phi_lo;
            a_lo = a_j;
            phi_lo = phi_j;
            dphi_lo = dphi_j;
          }
          ++j;
          z_failed = ((z_failed ? 1 : 0) | j) >= 30;  // jax: `failed | j >= 30` (no parentheses)
        }
        a_star = za;
        phi_star = zphi;
      };
      while (!ls_done && li <= 10 && !ls_failed) {
        const double a_i = li == 1 ? start_a : a_i1 * 2.0;
        double dphi_i, g_i[M];
        const double phi_i = ln.phi(x, pk, a_i, dphi_i, g_i);
        const bool s_z1 = wolfe_one(a_i, phi_i) || ((phi_i >= phi_i1) && (li > 1));
        const bool s_i = wolfe_two(dphi_i) && !s_z1;
        const bool s_z2 = (dphi_i >= 0.0) && !s_z1 && !s_i;
        if (s_i) {
          a_star = a_i;
          phi_star = phi_i;
#pragma unroll RU
          for (int i = 0; i < M; ++i) g_star[i] = g_i[i];
        }
        if (s_z1 || s_z2) {  // at most one of the two (jax runs both zooms masked; one body here)
          bool zf;
          if (s_z1) zoom(a_i1, phi_i1, dphi_i1, a_i, phi_i, dphi_i, zf);
          else zoom(a_i, phi_i, dphi_i, a_i1, phi_i1, dphi_i1, zf);
          ls_failed = ls_failed || zf;
        }
        ls_done = s_z1 || ls_done || s_i || s_z2;
        ++li;
        a_i1 = a_i;
        phi_i1 = phi_i;
        dphi_i1 = dphi_i;
      }
      ls_status = ls_failed ? 1 : (li > 10 ? 3 : 0);
      failed = ls_failed || !ls_done;
      // ---- BFGS update ----
      double sk[M], yk[M];
#pragma unroll RU
      for (int i = 0; i < M; ++i) {
        sk[i] = a_star * pk[i];
        yk[i] = g_star[i] - g[i];
      }
      const double rho = 1.0 / ln.dot(yk, sk);
      if (isfinite(rho) && (RU == 1 || INSITE_REFINE_QUAD)) {
        // rolled (scratch-resident) kernels: the same update expanded to O(M^2) with one matrix-vector
        // product, (I - rho s y^T) H (I - rho y s^T) + rho s s^T
        //   = H - rho (s (H y)^T + (H y) s^T) + (rho^2 y^T H y + rho) s s^T   (H symmetric),
        // instead of two O(M^3) products through two more M x M scratch matrices; the association order
        // differs from the oracle's w @ H @ w.T (jax's three-operand einsum fixes none either)
        double hy[M], yh[M];
#pragma unroll RU
        for (int i = 0; i < M; ++i) {
          double t = 0.0;
#pragma unroll RU
          for (int j = 0; j < M; ++j) t += H.at(i, j) * yk[j];
          hy[i] = t;
          yh[i] = yk[i] * t;
        }
        const double yhy = coord_sum(yh);
        const double cs = rho * rho * yhy + rho;
#pragma unroll RU
        for (int i = 0; i < M; ++i)
#pragma unroll RU
          for (int j = 0; j < M; ++j)
            H.at(i, j) = H.at(i, j) - rho * (sk[i] * hy[j] + hy[i] * sk[j]) + cs * (sk[i] * sk[j]);
      } else if (isfinite(rho)) {
        // (w @ H) @ w.T with w = I - rho s y^T formed on the fly (the same products and summation order as the
        // explicit w: w[i][q] = [i == q] - rho (s_i y_q)); WH in VGPRs (the line search's state is dead here)
        auto w = [&](int i, int q) { return (i == q ? 1.0 : 0.0) - rho * (sk[i] * yk[q]); };
        double WH[M][M];
#pragma unroll RU
        for (int i = 0; i < M; ++i)
#pragma unroll RU
          for (int j = 0; j < M; ++j) {
            double s = 0.0;
#pragma unroll RU
            for (int q = 0; q < M; ++q) s += w(i, q) * H.at(q, j);
            WH[i][j] = s;
          }
#pragma unroll RU
        for (int i = 0; i < M; ++i)
#pragma unroll RU
          for (int j = 0; j < M; ++j) {
            double s = 0.0;
#pragma unroll RU
            for (int q = 0; q < M; ++q) s += WH[i][q] * w(j, q);
            H.at(i, j) = s + rho * (sk[i] * sk[j]);
          }
      }
      double gm = 0.0;
#pragma unroll RU
      for (int i = 0; i < M; ++i) {
        x[i] = x[i] + sk[i];
        g[i] = g_star[i];
        gm = fmax(gm, fabs(g[i]));
      }
      converged = gm < 1e-5;
      old_old = f;
      f = phi_star;
      ++k;
    }
    nit = k;
    status = converged ? 0 : (k == maxiter ? 1 : (failed ? 2 + ls_status : -1));
    if (status == 3 && ra.revert3) {  // zoom failed: the reference code keeps the global coefficients (sindy.py:628-631)
#pragma unroll RU
      for (int i = 0; i < M; ++i) x[i] = ln.c0a[i];
    }
  }
#endif  // INSITE_REFINE_FLAT
  if (WIN && !PM && !valid) return;  // inert lanes past the last row: the wave-cooperative part is over
  // (PM: they stay -- the predictions leave through the wave's staging slot, every lane storing 4 rows' pieces)
  // ---------------- final Euler scan with the (refined) model, every coefficient (sindy.py:668) ----------------
  // coefficient q: the refined value if active, else the global one; resolved by comparison against the
  // active list (no dynamically indexed per-lane array, which would live in scratch)
  auto coef_at = [&](int q) -> double {
    double c = ra.c0[q];
#pragma unroll RU
    for (int i = 0; i < M; ++i)
      if (i < ra.m && ra.t_flat[i] == q) c = x[i];
    return c;
  };
  double gam[NA][D + 1];
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int e = 0; e <= D; ++e) gam[a][e] = 0.0;
  for (int q = 0; q < ra.n_coef; ++q) {
#pragma clang fp contract(off)  // NC
    const int code = ra.q_code[q], mk = ra.q_mask[q], ex = code >> 24;
    const double t = coef_at(q) * monomial_code(code & 0xffffff, uu);
#pragma unroll
    for (int a = 0; a < NA; ++a)
      if ((mk >> a) & 1)
#pragma unroll
        for (int e = 0; e <= D; ++e)
          if (ex == e) gam[a][e] += t;
  }
  const double h = ra.dt / (double)ra.sub;
  double y = PM ? ra.V[p * ra.ldv] : ra.V[p];
  for (int k = 0; k < ra.T; ++k) {
    const int ak = ln.armbit(k);
    double gk[D + 1];
#pragma unroll
    for (int e = 0; e <= D; ++e) gk[e] = gam[0][e];
#pragma unroll
    for (int a = 1; a < NA; ++a)
      if (ak == a)
#pragma unroll
        for (int e = 0; e <= D; ++e) gk[e] = gam[a][e];
    for (int s = 0; s < ra.sub; ++s) {
      if constexpr (D == 1) y = y + h * (gk[0] + gk[1] * y);
      else y = y + h * poly<D>(gk, y);
    }
    if constexpr (PM) {
      // stage step k in slot 0 (the ring is idle now) at the column-k position of this lane's row; after 8 steps
      // (or the last) every lane stores 16 B (two steps) of 4 rows: 64-B row segments, the whole 128-B lines of a
      // row written by consecutive flushes of the same wave
      const int lane = threadIdx.x & (kWave - 1);
      ln.win[pm_slot_index(lane, k & (kWin - 1))] = y;
      if ((k & (kWin - 1)) == kWin - 1 || k == ra.T - 1) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const int m = lane >> 2, pk = ((lane & 3) + (m >> 2)) & 3;
        const int col = (k & ~(kWin - 1)) + 2 * pk;
        const int prow = (int)p;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int r = 16 * q + m;
          const int row = __shfl(prow, r);
          const double2 v = *reinterpret_cast<const double2*>(ln.win + q * 128 + m * 8 + (lane & 3) * 2);
          if (ln.p0 + r < ra.N && col < ra.T) {
            double* dst = ra.preds + (int64_t)row * ra.ldp + col;
            if (col + 1 < ra.T && ra.st16) {
              *reinterpret_cast<double2*>(dst) = v;
            } else {
              dst[0] = v.x;
              if (col + 1 < ra.T) dst[1] = v.y;
            }
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
    } else {
      ra.preds[(int64_t)k * ra.ldp + p] = y;
    }
  }
  if (PM && !valid) return;
  if (ra.coef_out)
    for (int q = 0; q < ra.n_coef; ++q) ra.coef_out[p * ra.n_coef + q] = coef_at(q);
  if (ra.status) ra.status[p] = status;
  if (ra.iters) ra.iters[p] = nit;
  if (ra.nfev) ra.nfev[p] = ln.nev;
}

// ------------------------------------------------------------------------------------------------------------------
// Dynamic lane -> row assignment (row layout; INSITE_REFINE_DYN, runtime switch INSITE_REFINE_DYN=0 in the environment)
// ------------------------------------------------------------------------------------------------------------------
// With one row per lane a wave runs as long as its slowest row: rows binned by seq_len scan similar windows, but the
// number of evaluations per row (BFGS iterations x line-search trials) still varies (mean 10, wave maximum 17.8 on the
// INSITE bench: lanes idle ~40 % of the scans).  Here a persistent grid (the resident block count) takes rows from ONE
// device-wide queue in lane order -- rows sorted by seq_len, longest first: waves claiming at the same time hold rows
// of the same window length, and the cheapest rows come last (a longest-first schedule; per-block row ranges were
// measured slower: with rows sorted by length the blocks' work differs by the window length, profiles/r04).  A lane
// whose row is done writes the row's coefficients / status / iterations / evaluation count; once refill lanes of its
// wave are idle (or none is busy) the wave claims that many rows with one atomic and the new lanes start with their
// first evaluation (at c0, norm 1) in the next scan.  The row layout's ring gathers whatever rows the lanes hold
// (fill() shuffles each lane's row), so lanes of a wave need not hold neighbouring rows.  Per row the arithmetic is the
// static kernel's operation for operation (BfgsFlat is its flat state machine), so every output is bitwise the same;
// the final Euler scan runs in insite_refine_final_kernel from the written coefficients.  The queue head is one of
// kRefineQueues device words, zeroed on the stream before each launch (independent streams rotate through them).
// Measured (profiles/r04/dyn_sweep.txt, 1M rows): 2.25 ms per INSITE step against 2.16 for the static one-row-per-lane
// kernel, refill thresholds 2-32 and 512-1536 blocks no better; per-block row ranges 2.13-10 ms.  The lanes' rows sit
// at different BFGS phases, so every loop iteration issues the union of the start / line-search / zoom / update /
// finish paths, which costs what the better lane occupancy saves.  Kept as a knob (INSITE_REFINE_DYN=1 in the
// environment, or -DINSITE_REFINE_DYN=1), bitwise-tested against the static kernel.
#ifndef INSITE_REFINE_DYN
#define INSITE_REFINE_DYN 0
#endif
#ifndef INSITE_REFINE_DYN_REFILL
#define INSITE_REFINE_DYN_REFILL 8
#endif

template <int M>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(INSITE_REFINE_WPE4)))
insite_refine_dyn_kernel(RefineArgs, unsigned* queue, int refill) {
  KArgs& ra = kernel_args();
  constexpr int NA = 2, D = 1;
  using Lane = RefineLane<M, NA, D, true, true>;
  constexpr int RU = Lane::RU;
  constexpr bool kHL = INSITE_REFINE_HLDS && RU == M && M <= 4;
  __shared__ double sH[(kHL ? M * M : 1) * kBlock];
  __shared__ double sV[kWavesPerBlock * 2 * kWin * kWave];
  const int lane = threadIdx.x & (kWave - 1);
  auto row_of = [&](int64_t q) -> int64_t { return ra.order ? (int64_t)ra.order[q] : q; };
  Lane ln{ra, row_of(0), 0, 1.0, {}, {}};  // an idle lane keeps a valid row for the ring's gathers
  ln.win = sV + (threadIdx.x / kWave) * (2 * kWin * kWave);
#pragma unroll RU
  for (int i = 0; i < M; ++i) {
    ln.c0a[i] = i < ra.m ? ra.c0[ra.t_flat[i]] : 0.0;
    ln.mono[i] = 0.0;
  }
  BfgsFlat<M, kHL, RU, Lane> B;
  if constexpr (kHL) B.H.base = sH + threadIdx.x;
  B.t_trial = 0.0;
#pragma unroll RU
  for (int i = 0; i < M; ++i) B.x[i] = B.pk[i] = 0.0;
  const int maxiter = 200 * ra.n_coef;
  bool has = false, exhausted = false, pending = false, fresh = false;
  // a finished row: coefficients (every q: the refined value if active, else the global one), status, iterations
  auto finish = [&](int status, int nit) {
    const int64_t p = ln.p;
    if (status == 3 && ra.revert3) {  // zoom failed: the reference code keeps the global coefficients (sindy.py:628-631)
#pragma unroll RU
      for (int i = 0; i < M; ++i) B.x[i] = ln.c0a[i];
    }
    for (int q = 0; q < ra.n_coef; ++q) {
      double c = ra.c0[q];
#pragma unroll RU
      for (int i = 0; i < M; ++i)
        if (i < ra.m && ra.t_flat[i] == q) c = B.x[i];
      ra.coef_out[p * ra.n_coef + q] = c;
    }
    if (ra.status) ra.status[p] = status;
    if (ra.iters) ra.iters[p] = nit;
    if (ra.nfev) ra.nfev[p] = ln.nev;
    has = pending = false;
  };
  // wave-uniform: the idle lanes take the block's next rows (one LDS atomic for the wave)
  auto claim = [&]() {
    const uint64_t want = __builtin_amdgcn_ballot_w64(!has && !exhausted);
    if (want == 0ull) return;
    const int leader = __ffsll((unsigned long long)want) - 1;
    unsigned base = 0u;
    if (lane == leader) base = atomicAdd(queue, (unsigned)__popcll(want));
    base = __shfl(base, leader);
    if (has || exhausted) return;
    const int64_t q = (int64_t)base + __popcll(want & ((1ull << lane) - 1ull));
    if (q >= ra.N) {
      exhausted = true;
      return;
    }
    const int64_t p = row_of(q);
    ln.p = p;
    ln.nev = 0;
    double uu[INSITE_MAX_STATICS];
#pragma unroll
    for (int t = 0; t < INSITE_MAX_STATICS; ++t) uu[t] = t < ra.U ? ra.u[p * ra.U + t] : 0.0;
#pragma unroll RU
    for (int i = 0; i < M; ++i) ln.mono[i] = i < ra.m ? monomial_code(ra.t_ucode[i], uu) : 0.0;
    uint64_t am = 0ull;
    if ((ra.lda & 3) == 0 && ((uintptr_t)ra.arm8 & 3u) == 0) {  // the row's arm bytes as words (lda >= T)
      const uint32_t* w = reinterpret_cast<const uint32_t*>(ra.arm8 + p * ra.lda);
      for (int j = 0; 4 * j < ra.T; ++j) {
        const uint32_t v = w[j];
#pragma unroll
        for (int b = 0; b < 4; ++b)
          if (4 * j + b < ra.T) am |= (uint64_t)(((v >> (8 * b)) & 0xffu) != 0u ? 1 : 0) << (4 * j + b);
      }
    } else {
      for (int k = 0; k < ra.T; ++k) am |= (uint64_t)(ra.arm8[p * ra.lda + k] != 0 ? 1 : 0) << k;
    }
    ln.am = am;
#pragma unroll RU
    for (int i = 0; i < M; ++i) {
      B.x[i] = ln.c0a[i];
      B.pk[i] = 0.0;
    }
    B.t_trial = 0.0;
    B.k = 0;
    has = true;
    const int sl = ra.sl[p];
    if (sl > ra.tau && ra.T >= 2) {
      ln.setK(min(sl - ra.tau, ra.T - 1));
      ln.norm = 1.0;
      pending = fresh = true;
    } else {
      ln.setK(0);
      finish(-1, 0);
    }
  };
  claim();
  while (__builtin_amdgcn_ballot_w64(has || !exhausted) != 0ull) {
    double dphi_t, g_t[M];
    // a fresh row evaluates at c0 itself (t 0, direction 0: x + 0 * 0 is x bit for bit), the others their trial
    const double phi_t = ln.phi(B.x, B.pk, B.t_trial, dphi_t, g_t, pending);
    if (pending) {
      bool more;
      if (fresh) {
        more = B.start(phi_t, g_t, ln, maxiter);
        fresh = false;
      } else {
        more = B.advance(phi_t, dphi_t, g_t, ln, maxiter);
      }
      if (!more)
        finish(B.converged ? 0 : (B.k == maxiter ? 1 : (B.failed ? 2 + B.ls_status : -1)), B.k);
    }
    const uint64_t idle = __builtin_amdgcn_ballot_w64(!has && !exhausted);
    if (idle != 0ull && (__popcll(idle) >= refill || __builtin_amdgcn_ballot_w64(pending) == 0ull))
      claim();
  }
}

// The final Euler scan of the row layout from the refined coefficients insite_refine_dyn_kernel wrote (sindy.py:668):
// insite_refine_kernel's final scan, operation for operation, on identity rows (a wave's 64 rows are contiguous).  A
// wave stages its rows' coefficients and arm bytes in LDS with coalesced loads first (64 rows x n_coef doubles and
// 64 x lda bytes are contiguous runs; lane-per-row loads of them touched 64 lines per instruction and fetched 2 GB
// per launch for ~0.2 GB of data), and the predictions leave through the same staging as 64-B row segments.
constexpr int kFinalMaxCoef = 16;  // coefficients staged per row (larger models read theirs per lane)
template <int M>
__global__ void __launch_bounds__(kBlock) insite_refine_final_kernel(RefineArgs, int staged_arm) {
  KArgs& ra = kernel_args();
  constexpr int NA = 2, D = 1;
  // per wave: [64 x kFinalMaxCoef doubles | 64 x 64 arm bytes], its first 4 KB reused as the prediction staging once
  // the coefficients and arms are in registers (48 KB per block: 3 blocks per CU)
  constexpr int kWaveLds = kWave * kFinalMaxCoef * 8 + kWave * 64;
  __shared__ __attribute__((aligned(16))) uint8_t sL[kWavesPerBlock * kWaveLds];
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
  const int64_t p0 = gid - lane;
  if (p0 >= ra.N) return;  // (wave-uniform)
  const bool valid = gid < ra.N;
  const int64_t p = valid ? gid : ra.N - 1;
  const int nrow = ra.N - p0 < kWave ? (int)(ra.N - p0) : kWave;
  double* st = reinterpret_cast<double*>(sL + wv * kWaveLds);
  const bool stage_c = ra.n_coef <= kFinalMaxCoef;
  double* sc = st;
  uint32_t* sa = reinterpret_cast<uint32_t*>(sL + wv * kWaveLds + kWave * kFinalMaxCoef * 8);
  if (stage_c) {
    const double* src = ra.coef_out + p0 * ra.n_coef;
    const int cnt = nrow * ra.n_coef;
    for (int i = lane; i < cnt; i += kWave) sc[i] = src[i];
  }
  if (staged_arm) {  // lda % 4 == 0, 4-byte aligned rows, T <= 64
    const uint32_t* src = reinterpret_cast<const uint32_t*>(ra.arm8 + p0 * ra.lda);
    const int cnt = nrow * (int)(ra.lda / 4);
    for (int i = lane; i < cnt; i += kWave) sa[i] = src[i];
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  double uu[INSITE_MAX_STATICS];
#pragma unroll
  for (int t = 0; t < INSITE_MAX_STATICS; ++t) uu[t] = t < ra.U ? ra.u[p * ra.U + t] : 0.0;
  double gam[NA][D + 1];
#pragma unroll
  for (int a = 0; a < NA; ++a)
#pragma unroll
    for (int e = 0; e <= D; ++e) gam[a][e] = 0.0;
  const int lr = valid ? lane : nrow - 1;
  for (int q = 0; q < ra.n_coef; ++q) {
    const int code = ra.q_code[q], mk = ra.q_mask[q], ex = code >> 24;
    const double c = stage_c ? sc[lr * ra.n_coef + q] : ra.coef_out[p * ra.n_coef + q];
    const double t = c * monomial_code(code & 0xffffff, uu);
#pragma unroll
    for (int a = 0; a < NA; ++a)
      if ((mk >> a) & 1)
#pragma unroll
        for (int e = 0; e <= D; ++e)
          if (ex == e) gam[a][e] += t;
  }
  uint64_t am = 0ull;
  if (staged_arm) {
    const uint8_t* row = reinterpret_cast<const uint8_t*>(sa) + lr * ra.lda;
    for (int k = 0; k < ra.T; ++k) am |= (uint64_t)(row[k] != 0 ? 1 : 0) << k;
  } else {
    for (int k = 0; k < ra.T; ++k) am |= (uint64_t)(ra.arm8[p * ra.lda + k] != 0 ? 1 : 0) << k;
  }
  const double h = ra.dt / (double)ra.sub;
  double y = ra.V[p * ra.ldv];
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every lane's staged reads done before the staging reuse
  __builtin_amdgcn_wave_barrier();
  for (int k = 0; k < ra.T; ++k) {
    const int ak = (int)((am >> k) & 1ull);
    double gk[D + 1];
#pragma unroll
    for (int e = 0; e <= D; ++e) gk[e] = gam[0][e];
#pragma unroll
    for (int a = 1; a < NA; ++a)
      if (ak == a)
#pragma unroll
        for (int e = 0; e <= D; ++e) gk[e] = gam[a][e];
    for (int s = 0; s < ra.sub; ++s) y = y + h * (gk[0] + gk[1] * y);
    st[pm_slot_index(lane, k & (kWin - 1))] = y;
    if ((k & (kWin - 1)) == kWin - 1 || k == ra.T - 1) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const int m = lane >> 2, pk = ((lane & 3) + (m >> 2)) & 3;
      const int col = (k & ~(kWin - 1)) + 2 * pk;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t r = p0 + 16 * q + m;
        const double2 v = *reinterpret_cast<const double2*>(st + q * 128 + m * 8 + (lane & 3) * 2);
        if (r < ra.N && col < ra.T) {
          double* dst = ra.preds + r * ra.ldp + col;
          if (col + 1 < ra.T && ra.st16) {
            *reinterpret_cast<double2*>(dst) = v;
          } else {
            dst[0] = v.x;
            if (col + 1 < ra.T) dst[1] = v.y;
          }
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
  }
}

// ------------------------------------------------------------------------------------------------------------------
// Cooperative refinement of the dense 4-arm models (INSITE_REFINE_COOP): 9-16 active coefficients, int8 arms
// ------------------------------------------------------------------------------------------------------------------
// The rolled one-row-per-lane M = 16 kernel keeps the 16 x 16 inverse Hessian and a dozen 16-vectors in per-lane
// scratch (3.9 KB a lane): on the cancer_sim-shaped dense model (4 arms x 4 terms, the reference's slowest published
// path) its PMC traffic was ~374 GB per 1M-row launch, 66-72 ms.  Here a row is refined by a group of 8 lanes:
// lane j of a group owns coordinates j and j + 8 (their x, g, p, g* and their two rows of H, in VGPRs) and the
// sensitivity of tangent (arm j / 2, exponent j % 2) -- the 8 tangents of a 4-arm affine model.  Every lane runs the
// row's state chain y (so the tangents need no broadcast), and the scalars of the line search / zoom, replicated.
// Everything the single-lane kernel sums over coordinates (gamma, the penalty, dot products, H y, y^T H y) is
// summed in ITS order from values shuffled within the group, without contraction in both kernels ("NC"), and the
// QUAD inverse-Hessian update is the one that kernel runs (RU = 1): the outputs are bitwise the M = 16 kernel's
// (tested).  Shuffles only read lanes of the
// reading lane's own group, whose lanes always branch together (their replicated scalars are equal).
// STG (T <= 64): the wave's 8 rows of V and of the arms are staged in LDS once (lane k loads step k of all 8 rows),
// and every scan reads them there.  Read from global memory per step, each step of an evaluation waited for its
// one-step-ahead loads: at 2 waves per SIMD the scan was latency-bound (~30 us per wave-evaluation).
#ifndef INSITE_REFINE_COOP
#define INSITE_REFINE_COOP 1
#endif
#ifndef INSITE_REFINE_SWZ
#define INSITE_REFINE_SWZ 1  // the group gathers as ds_swizzle (0: ds_bpermute through __shfl)
#endif
#ifndef INSITE_REFINE_M6
#define INSITE_REFINE_M6 1  // a kernel sized for 5-6 active terms (the M = 8 one held its state in AGPRs at 1 wave)
#endif
#ifndef INSITE_REFINE_COOP8
#define INSITE_REFINE_COOP8 0  // A/B: the cooperative kernel for 5-8 active terms on 4 arms
#endif
// (measured: the sparse 4-arm line's 5-term model 11.3 ms cooperative vs 6.5 ms one lane per row -- with one
// coordinate a lane the group's 8-fold replicated scan and line search cost more than the single-lane kernel's
// spills; profiles/r04/coop8/)
#ifndef INSITE_REFINE_COOP_WPE
#define INSITE_REFINE_COOP_WPE 2
#endif
#ifndef INSITE_COOP_LDSV
#define INSITE_COOP_LDSV 1  // the cooperative kernel's whole-vector exchanges through LDS (0: per-coordinate swizzles)
#endif
#ifndef INSITE_COOP_SCAN_PIPE
#define INSITE_COOP_SCAN_PIPE 1  // the cooperative kernel's software-pipelined closed-form scan (0: the step-wise one)
#endif
// INSITE_COOP_SCAN_SPLIT: the pipelined scan in two ranges -- steps below the wave's shortest
// live window without the per-lane `k < K` guard (its exec-mask save / branch / restore is 3 SALU + a compare a
// step), then the rest guarded.  Lanes with nothing pending run the unguarded range too; their values are never used
// (every consumer of fg's results is under `pending`, and a row's 8 lanes share its liveness).  Live lanes issue the
// same operations in the same order: bitwise the guarded scan.
template <bool B>
struct ScanGuard {
  static constexpr bool value = B;
};
// Measured slower (profiles/r06/refine_ab/: dense 11.26-11.31 vs 10.94-11.04 ms/step, joint 12.51-12.72 vs 12.27-12.41,
// interleaved on one box) although the unguarded range issues 104 instead of 125 instructions per 4 steps (14 SALU
// instead of 24): the second copy of the scan, inlined into both objective calls, costs more than it saves.  Kept as a
// knob, off.
#ifndef INSITE_COOP_SCAN_SPLIT
#define INSITE_COOP_SCAN_SPLIT 0
#endif
constexpr int kCoopG = 8;  // lanes per row

constexpr int kCoopStT = 64;  // staged steps (STG)
constexpr int kCoopStPad = 8;
// lane C of the reading lane's 8-lane group: ds_swizzle in bitmask mode (and 0x18, or C: the group's base within the
// 32-lane half, plus C) -- the value of __shfl(v, group base + C) without the per-lane address of ds_bpermute
template <int C>
__device__ __forceinline__ double grp_lane(double v) {
  static_assert(C >= 0 && C < 8, "lane of an 8-lane group");
  constexpr int kPat = 0x18 | (C << 5);
  const int lo = __builtin_amdgcn_ds_swizzle(__double2loint(v), kPat);
  const int hi = __builtin_amdgcn_ds_swizzle(__double2hiint(v), kPat);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double grp_lane(double v, int c) {  // c a constant after unrolling
  switch (c & 7) {
    case 0: return grp_lane<0>(v);
    case 1: return grp_lane<1>(v);
    case 2: return grp_lane<2>(v);
    case 3: return grp_lane<3>(v);
    case 4: return grp_lane<4>(v);
    case 5: return grp_lane<5>(v);
    case 6: return grp_lane<6>(v);
    default: return grp_lane<7>(v);
  }
}
// lane j ^ X of the reading lane's 8-lane group (ds_swizzle bitmask mode: and 0x1f, xor X)
template <int X>
__device__ __forceinline__ double grp_xor(double v) {
  constexpr int kPat = 0x1f | (X << 10);
  const int lo = __builtin_amdgcn_ds_swizzle(__double2loint(v), kPat);
  const int hi = __builtin_amdgcn_ds_swizzle(__double2hiint(v), kPat);
  return __hiloint2double(hi, lo);
}
// coord_sum<16> over the group: v = the lane's own pair (coordinates j and j + 8) summed; every lane gets the same
// bits (each butterfly level adds two equal-valued operands in either order)
__device__ __forceinline__ double grp_tree_sum(double v) {
#pragma clang fp contract(off)  // NC
  v = v + grp_xor<1>(v);
  v = v + grp_xor<2>(v);
  v = v + grp_xor<4>(v);
  return 0.0 + v;
}
// PM (the row layout, insite_refine_rows_f64): V [N, ldv] and arm8 [N, lda] patient-major, staged by whole rows (lane
// = step: one coalesced row read per staged row), predictions stored into the patient-major rows; every other output
// is indexed by the row already (p = row_order[lane-order row]), so no gather / scatter pass surrounds the kernel
template <int MC, int NA, bool STG, bool PM = false>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(INSITE_REFINE_COOP_WPE)))
insite_refine_coop_kernel(RefineArgs) {
  constexpr int S = MC / kCoopG;  // coordinates per lane: i = j + kCoopG s
  static_assert(MC % kCoopG == 0 && NA * 2 <= kCoopG, "one tangent per lane");
  static_assert(!PM || STG, "the row layout stages its rows (T <= kCoopStT)");
  KArgs& ra = kernel_args();
  const int lane = threadIdx.x & (kWave - 1);
  const int j = lane & (kCoopG - 1);
  const int gbase = lane & ~(kCoopG - 1);
  const int64_t gt = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if ((gt - lane) / kCoopG >= ra.N) return;  // (wave-uniform)
  const int64_t gr = gt / kCoopG;            // lane-order row of this group
  const bool valid = gr < ra.N;
  const int64_t grc = valid ? gr : ra.N - 1;
  const int64_t p = ra.order ? (int64_t)ra.order[grc] : grc;
  const int ta = j >> 1, te = j & 1;  // this lane's tangent (arm, exponent)
  // the wave's rows staged in LDS: [step][row slot] doubles / arm bytes (row slot = lane / 8)
  // (the pipelined scan reads up to 4 steps past its end unclamped: kCoopStPad steps of padding whose offsets are
  // staged as valid table entries and whose values are never used)
  constexpr int kPipe = STG && INSITE_REFINE_CF && INSITE_COOP_SCAN_PIPE;
  constexpr int kStT = kCoopStT + (kPipe ? kCoopStPad : 0);
  __shared__ double sV[STG ? kWavesPerBlock * kStT * kCoopG : 1];
  __shared__ int8_t sA[STG ? kWavesPerBlock * kCoopStT * kCoopG : 1];
  // kPipe: step k's arm as the byte offset of its constants in the row's table, (row slot * NA + arm) * 40
  __shared__ int sO[kPipe ? kWavesPerBlock * kStT * kCoopG : 1];
  // the per-arm closed-form constants of the current evaluation (CfArm: P, B, hS, C1, C2), [row slot][arm][5] per
  // wave: written once per evaluation by the (ta, te = 0) lane of each arm, read per step by every lane of the row
  // at its step's arm (the 8 lanes of a row read one address: an LDS broadcast) -- instead of every lane computing
  // all NA arms' constants and selecting one per step through NA - 1 branchy register copies (5 moves each)
  constexpr int kCf5 = 5;
  __shared__ double sCf[INSITE_REFINE_CF ? kWavesPerBlock * kCoopG * NA * kCf5 : 1];
  const int rs = lane / kCoopG, wv = threadIdx.x / kWave;
  double* const wCf = sCf + (INSITE_REFINE_CF ? wv * kCoopG * NA * kCf5 : 0);
  double* const wV = sV + (STG ? wv * kStT * kCoopG : 0);
  int8_t* const wA = sA + (STG ? wv * kCoopStT * kCoopG : 0);
  int* const wO = sO + (kPipe ? wv * kStT * kCoopG : 0);
  if constexpr (STG) {  // (ra.T <= kCoopStT, checked at the launch)
    long long pg[kCoopG];
#pragma unroll
    for (int g = 0; g < kCoopG; ++g) pg[g] = __shfl((long long)p, g * kCoopG);
    if (lane < ra.T) {
#pragma unroll
      for (int g = 0; g < kCoopG; ++g) {
        wV[lane * kCoopG + g] = PM ? ra.V[pg[g] * ra.ldv + lane] : ra.V[(int64_t)lane * ra.ldv + pg[g]];
        // the arm clamped to [0, NA) (the documented contract; an out-of-range byte must not index another row's
        // or another wave's constants -- ADVICE r05)
        const int8_t a8 = PM ? ra.arm8[pg[g] * ra.lda + lane] : ra.arm8[(int64_t)lane * ra.lda + pg[g]];
        const int8_t am = a8 < 0 ? (int8_t)0 : a8 >= NA ? (int8_t)(NA - 1) : a8;
        wA[lane * kCoopG + g] = am;
        if constexpr (kPipe) wO[lane * kCoopG + g] = (g * NA + am) * kCf5 * (int)sizeof(double);
      }
    }
    if constexpr (kPipe) {
      // the pipelined scan's look-ahead reads offsets up to ~6 steps past the row's last step: steps [T, kStT) hold
      // the row's own arm-0 offset (a valid table entry; the values read through it are never used)
      for (int k = lane; k < kStT; k += kWave)
        if (k >= ra.T) {
#pragma unroll
          for (int g = 0; g < kCoopG; ++g) wO[k * kCoopG + g] = g * NA * kCf5 * (int)sizeof(double);
        }
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
  }
  auto v_at = [&](int k) -> double { return STG ? wV[k * kCoopG + rs] : ra.V[(int64_t)k * ra.ldv + p]; };
  auto a_at = [&](int k) -> int {  // (staged arms are clamped at staging; unstaged ones here)
    if constexpr (STG) return (int)wA[k * kCoopG + rs];
    const int a = (int)ra.arm8[(int64_t)k * ra.lda + p];
    return a < 0 ? 0 : a >= NA ? NA - 1 : a;
  };
  // coordinate i of a distributed vector: lane i % 8 of the group, slot i / 8
  auto gat = [&](const double (&v)[S], int i) -> double {
    return INSITE_REFINE_SWZ ? grp_lane(v[i / kCoopG], i % kCoopG) : __shfl(v[i / kCoopG], gbase + (i % kCoopG));
  };
  // LDSV: a distributed vector reaches every lane of its group through LDS -- each lane stores its S coordinates
  // (2 ds_write_b64), then every lane reads the MC values in coordinate order two at a time (MC / 2 ds_read_b128,
  // one address per group: a broadcast) -- instead of one 2 x ds_swizzle gather per coordinate (32 LDS
  // instructions for 16 values, 10 here).  Two buffers per group (the inverse-Hessian update needs sk and H yk at
  // once).  The LDS keeps one wave's accesses in issue order; only the compiler's order is pinned (vx_sync).
  constexpr int kVx = INSITE_COOP_LDSV && MC == 2 * kCoopG ? MC : 2;
  __shared__ __attribute__((aligned(16))) double sVx[kWavesPerBlock * kCoopG * 2 * kVx];
  double* const wVx = sVx + (wv * kCoopG + rs) * 2 * kVx;
  auto vx_sync = [&]() {
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
  };
  auto vx_store = [&](const double (&v)[S], int buf) {
    vx_sync();
#pragma unroll
    for (int s = 0; s < S; ++s) wVx[buf * kVx + j + kCoopG * s] = v[s];
    vx_sync();
  };
  auto vx_load2 = [&](int buf, int q) -> double2 {  // coordinates 2 q and 2 q + 1
    return *reinterpret_cast<const double2*>(wVx + buf * kVx + 2 * q);
  };
  constexpr bool kLdsv = INSITE_COOP_LDSV && MC == 2 * kCoopG;
  static_assert(!(MC == 16 && INSITE_REFINE_FUSEDUPD && !kLdsv), "the fused update (M = 16) is written for LDSV");
  double uu[INSITE_MAX_STATICS];
#pragma unroll
  for (int t = 0; t < INSITE_MAX_STATICS; ++t) uu[t] = t < ra.U ? ra.u[p * ra.U + t] : 0.0;
  double mono[S], c0a[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int i = j + kCoopG * s;
    mono[s] = i < ra.m ? monomial_code(ra.t_ucode[i], uu) : 0.0;
    c0a[s] = i < ra.m ? ra.c0[ra.t_flat[i]] : 0.0;
  }
  const int sl = valid ? ra.sl[p] : 0;
  const bool refine = sl > ra.tau && ra.T >= 2;
  const int K = refine ? min(sl - ra.tau, ra.T - 1) : 0;
  double norm = 1.0;
  int nev = 0;
  // Per-lane routing, once (round 5): lane j's tangent (ta, te) receives active coefficient i when bit i of `rbits`
  // is set, and its own coordinates i = j + 8 s carry (omk[s], oex[s]).  Every sum of the objective is still taken
  // in the single-lane kernel's order; what changes is WHO computes it: before, every lane walked all MC coefficients
  // with the (uniform but compiler-opaque) routing as selects -- 8 conditional adds per coefficient for gamma, and
  // each coordinate's gradient (two divisions) computed under an owner-lane mask, so the wave issued all MC of them:
  // ~1,600 of the loop's ~2,900 VALU per evaluation (profiles/r05/coop/).
  unsigned rbits = 0u;
  int omk[S], oex[S];
  for (int i = 0; i < ra.m && i < MC; ++i) {
    const int mk = ra.t_mask[i], ex = ra.t_ex[i];
    if (((mk >> ta) & 1) && ex == te) rbits |= 1u << i;
  }
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int i = j + kCoopG * s;
    omk[s] = i < ra.m ? ra.t_mask[i] : 0;
    oex[s] = i < ra.m ? ra.t_ex[i] : 0;
  }
  // f and its gradient at c (RefineLane::fg, D = 1, the non-windowed scan); every lane of the wave calls it
  auto fg = [&](const double (&c)[S], double (&g)[S], bool live) -> double {
    nev += live ? 1 : 0;
    // per-coordinate values are formed on their owner lane and gathered once (the same roundings as forming them
    // from two gathered operands on the reading lane: one gather per coordinate instead of two)
    double tm[S], sq[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
#pragma clang fp contract(off)  // NC
      tm[s] = c[s] * mono[s];
      const double dd = c0a[s] - c[s];
      sq[s] = dd * dd;
    }
    // gamma_{ta,te} on lane j (the coefficients routed to it, in coefficient order: the single-lane kernel's sum),
    // then gathered: lane 2a + e holds gamma_{a,e}
    double gown = 0.0;
    if constexpr (kLdsv) {
      vx_store(tm, 0);
#pragma unroll
      for (int q = 0; q < MC / 2; ++q) {
#pragma clang fp contract(off)  // NC
        const double2 t = vx_load2(0, q);
        if ((rbits >> (2 * q)) & 1u) gown += t.x;
        if ((rbits >> (2 * q + 1)) & 1u) gown += t.y;
      }
    } else {
#pragma unroll
    for (int i = 0; i < MC; ++i) {
#pragma clang fp contract(off)  // NC
      if (i >= ra.m) break;
      const double t = gat(tm, i);  // c_i m_i, formed on coordinate i's lane
      if ((rbits >> i) & 1u) gown += t;
    }
    }
    const double h = ra.dt / (double)ra.sub;
    double gam[NA][2];
    if constexpr (INSITE_REFINE_CF) {
      // arm ta's constants from (gamma_{ta,0}, gamma_{ta,1}) -- this lane's and its pair partner's (lane j ^ 1) --
      // computed by both lanes of the pair and stored by the te = 0 one
      const double gp = __shfl_xor(gown, 1);
      const CfArm c = cf_arm(te ? gp : gown, te ? gown : gp, h, ra.sub);
      if (te == 0) {
        double* const q = wCf + (rs * NA + ta) * kCf5;
        q[0] = c.P;
        q[1] = c.B;
        q[2] = c.hS;
        q[3] = c.C1;
        q[4] = c.C2;
      }
      __builtin_amdgcn_wave_barrier();
    } else {
#pragma unroll
      for (int a = 0; a < NA; ++a)
#pragma unroll
        for (int e = 0; e <= 1; ++e) gam[a][e] = grp_lane(gown, 2 * a + e);
    }
    double y = v_at(0);
    double d = 0.0, gGo = 0.0, L = 0.0;
    const int Kl = live ? K : 0;
    int Kw = Kl;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) Kw = max(Kw, __shfl_xor(Kw, off));
#if INSITE_COOP_SCAN_PIPE
    if constexpr (STG && INSITE_REFINE_CF) {
      // software-pipelined scan: step k's arm constants (5 doubles from the LDS table) and target are read during
      // step k - 1, and its arm index during step k - 2, so no step waits on an LDS round trip of its own (the
      // per-step table lookup after the arm read exposed two dependent LDS latencies a step); the addition term
      // is formed branch-free.  The arithmetic is the CF branch below, op for op.
      // row slot rs's staged steps: target of step k at vr[8 (k + 1)], its arm's constants at wCf + or[8 k] bytes
      const double* const vr = wV + rs;
      const int* const orow = wO + rs;
      const char* const cfb = reinterpret_cast<const char*>(wCf);
      struct Step {
        double P, B, hS, C1, C2, v;
        int off;
      };
      auto load = [&](int off, int k) -> Step {  // constants at byte offset off and the target of step k
        const double* const q = reinterpret_cast<const double*>(cfb + off);
        return Step{q[0], q[1], q[2], q[3], q[4], vr[(k + 1) * kCoopG], off};
      };
      const int own = (rs * NA + ta) * kCf5 * (int)sizeof(double);  // this lane's tangent arm, as an offset
      auto step = [&](const Step& c, int k) {
        if (k < Kl) {
          const double tv = te ? fma(c.C1, y, c.C2) : c.hS;
          const double add = c.off == own ? tv : 0.0;
          d = fma(c.P, d, add);
          y = fma(c.P, y, c.B);
          const double r = c.v - y;
          L = fma(r, r, L);
          gGo = fma(-2.0 * r, d, gGo);
        }
      };
      auto step_all = [&](const Step& c) {  // step without the per-lane guard (SPLIT's first range)
        const double tv = te ? fma(c.C1, y, c.C2) : c.hS;
        const double add = c.off == own ? tv : 0.0;
        d = fma(c.P, d, add);
        y = fma(c.P, y, c.B);
        const double r = c.v - y;
        L = fma(r, r, L);
        gGo = fma(-2.0 * r, d, gGo);
      };
      // two register sets alternate (s0, s1): while step k computes, step k + 1's constants are in flight, their
      // offset read three steps earlier (step k + j's in am[(k + j) % 4]) -- the LDS counter is in order, so an
      // arm read one step ahead made the next lookup wait for everything issued in between.  Reads past the
      // scan's end land in the padding (offsets staged valid, values never used).
      auto scan_range = [&](const int kb, const int ke, auto guarded) {  // steps [kb, ke), ke wave-uniform
        constexpr bool G = decltype(guarded)::value;
        auto st = [&](const Step& c, int k) {
          if constexpr (G) step(c, k);
          else step_all(c);
        };
        int am[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) am[q] = orow[(kb + q) * kCoopG];
        Step s0 = load(am[0], kb), s1;
        for (int k = kb; k < ke; k += 4) {  // (the breaks are uniform)
          s1 = load(am[1], k + 1);
          am[0] = orow[(k + 4) * kCoopG];
          st(s0, k);
          if (k + 1 >= ke) break;
          s0 = load(am[2], k + 2);
          am[1] = orow[(k + 5) * kCoopG];
          st(s1, k + 1);
          if (k + 2 >= ke) break;
          s1 = load(am[3], k + 3);
          am[2] = orow[(k + 6) * kCoopG];
          st(s0, k + 2);
          if (k + 3 >= ke) break;
          s0 = load(am[0], k + 4);
          am[3] = orow[(k + 7) * kCoopG];
          st(s1, k + 3);
        }
      };
      if (Kw > 0) {
        int Km = 0;  // steps [0, Km) unguarded
        if constexpr (INSITE_COOP_SCAN_SPLIT) {  // the wave's shortest live window (lanes with nothing pending: Kw)
          Km = Kl > 0 ? Kl : Kw;
#pragma unroll
          for (int off = 32; off >= 1; off >>= 1) Km = min(Km, __shfl_xor(Km, off));
          Km = __builtin_amdgcn_readfirstlane(Km);
          scan_range(0, Km, ScanGuard<false>{});
        }
        if (Km < Kw) scan_range(Km, Kw, ScanGuard<true>{});
      }
    } else
#endif
    {
    int ak_nx = Kw > 0 ? a_at(0) : 0;
    double v_nx = Kw > 0 ? v_at(1) : 0.0;
    for (int k = 0; k < Kw; ++k) {
      const int ak = ak_nx;
      const double vk1 = v_nx;
      if (k + 1 < Kw) {
        ak_nx = a_at(k + 1);
        v_nx = v_at(k + 2);
      }
      if (INSITE_REFINE_CF && k < Kl) {
        const double* const q = wCf + (rs * NA + ak) * kCf5;
        CfArm c;
        c.P = q[0];
        c.B = q[1];
        c.hS = q[2];
        c.C1 = q[3];
        c.C2 = q[4];
        const double add = ak == ta ? (te ? fma(c.C1, y, c.C2) : c.hS) : 0.0;
        d = fma(c.P, d, add);
        y = fma(c.P, y, c.B);
        const double r = vk1 - y;
        L = fma(r, r, L);
        gGo = fma(-2.0 * r, d, gGo);
      } else if (k < Kl) {
        double gk0 = gam[0][0], gk1 = gam[0][1];
#pragma unroll
        for (int a = 1; a < NA; ++a)
          if (ak == a) {
            gk0 = gam[a][0];
            gk1 = gam[a][1];
          }
        const double hb = h * gk1;
        const double ha = (ak == ta) ? h : 0.0;
#pragma unroll 5
        for (int s = 0; s < ra.sub; ++s) {
          const double dh = fma(hb, d, d);
          d = te ? fma(ha, y, dh) : dh + ha;
          y = fma(h, fma(gk1, y, gk0), y);
        }
        const double r = vk1 - y;
        L = fma(r, r, L);
        gGo = fma(-2.0 * r, d, gGo);
      }
    }
    }
    const double iK = 1.0 / (double)K;
    L *= iK;
    double gG[NA][2];
    if constexpr (kLdsv) {  // tangent 2 a + e's gradient part sits on lane 2 a + e: one store, NA reads
      vx_sync();
      wVx[j] = gGo;
      vx_sync();
#pragma unroll
      for (int a = 0; a < NA; ++a) {
        const double2 t = vx_load2(0, a);
        gG[a][0] = t.x;
        gG[a][1] = t.y;
      }
    } else {
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int e = 0; e <= 1; ++e) gG[a][e] = INSITE_REFINE_SWZ ? grp_lane(gGo, 2 * a + e) : __shfl(gGo, gbase + 2 * a + e);
    }
    double pen = 0.0;
    if constexpr (MC == 16 && INSITE_REFINE_TREE) {
#pragma clang fp contract(off)  // NC
      pen = grp_tree_sum((j < ra.m ? sq[0] : 0.0) + (j + kCoopG < ra.m ? sq[1] : 0.0));
    } else {
#pragma unroll
    for (int i = 0; i < MC; ++i) {
#pragma clang fp contract(off)  // NC
      const double sqi = gat(sq, i);
      if (i >= ra.m) break;
      pen += sqi;
    }
    }
    // the gradient of this lane's own coordinates only (each lane its S, not the wave all MC under owner masks)
#pragma unroll
    for (int s = 0; s < S; ++s) {
#pragma clang fp contract(off)  // NC
      if (j + kCoopG * s >= ra.m) {
        g[s] = 0.0;
        continue;
      }
      double gd = 0.0;
#pragma unroll
      for (int a = 0; a < NA; ++a)
        if ((omk[s] >> a) & 1)
#pragma unroll
          for (int e = 0; e <= 1; ++e)
            if (oex[s] == e) gd += gG[a][e];
      g[s] = gd * iK * mono[s] / norm + 2.0 * ra.lam * (c[s] - c0a[s]) / (double)ra.n_coef;
    }
    return L / norm + ra.lam * pen / (double)ra.n_coef;
  };
  auto dot = [&](const double (&a)[S], const double (&b)[S]) -> double {
#pragma clang fp contract(off)  // NC
    double pr[S];
#pragma unroll
    for (int s = 0; s < S; ++s) pr[s] = a[s] * b[s];
    if constexpr (MC == 16 && INSITE_REFINE_TREE) {
      return grp_tree_sum(pr[0] + pr[1]);
    } else {
      double s_ = 0.0;
#pragma unroll
      for (int i = 0; i < MC; ++i) s_ += gat(pr, i);
      return s_;
    }
  };
  // ---- the flat BFGS state machine (BfgsFlat with the vectors distributed; the QUAD update of RU = 1) ----
  double x[S], g[S], pk[S], g_star[S], Hr[S][MC];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    x[s] = c0a[s];
    pk[s] = 0.0;
  }
  double f = 0.0, old_old = 0.0, phi0 = 0.0, dphi0 = 0.0, a_i1 = 0.0, phi_i1 = 0.0, dphi_i1 = 0.0, a_star = 0.0,
         phi_star = 0.0, a_lo = 0.0, phi_lo = 0.0, dphi_lo = 0.0, a_hi = 0.0, phi_hi = 0.0, dphi_hi = 0.0, a_rec = 0.0,
         phi_rec = 0.0, za = 0.0, zphi = 0.0, t_trial = 0.0;
  int li = 1, zj = 0, k = 0, ls_status = 0;
  bool ls_failed = false, in_zoom = false, z_failed = false, converged = false, failed = false;
  const int maxiter = 200 * ra.n_coef;
  auto begin_ls = [&]() {
#pragma clang fp contract(off)  // NC
#pragma unroll
    for (int s = 0; s < S; ++s) pk[s] = 0.0;
    double acc[S];
#pragma unroll
    for (int s = 0; s < S; ++s) acc[s] = 0.0;
    if constexpr (kLdsv) {
      vx_store(g, 0);
#pragma unroll
      for (int q = 0; q < MC / 2; ++q) {
        const double2 gq = vx_load2(0, q);
#pragma unroll
        for (int s = 0; s < S; ++s) {
          if constexpr (INSITE_REFINE_FUSEDUPD) {
            acc[s] = fma(Hr[s][2 * q], gq.x, acc[s]);
            acc[s] = fma(Hr[s][2 * q + 1], gq.y, acc[s]);
          } else {
            acc[s] += Hr[s][2 * q] * gq.x;
            acc[s] += Hr[s][2 * q + 1] * gq.y;
          }
        }
      }
    } else {
#pragma unroll
    for (int q = 0; q < MC; ++q) {
      const double gq = gat(g, q);
#pragma unroll
      for (int s = 0; s < S; ++s) acc[s] += Hr[s][q] * gq;
    }
    }
#pragma unroll
    for (int s = 0; s < S; ++s) pk[s] = -acc[s];
    phi0 = f;
    dphi0 = dot(g, pk);
    const double cand = 1.01 * 2.0 * (phi0 - old_old) / dphi0;
    t_trial = cand > 1.0 ? 1.0 : cand;
    li = 1;
    a_i1 = 0.0;
    phi_i1 = phi0;
    dphi_i1 = dphi0;
    a_star = 0.0;
    phi_star = phi0;
#pragma unroll
    for (int s = 0; s < S; ++s) g_star[s] = g[s];
    ls_failed = false;
    in_zoom = false;
  };
  auto zoom_top = [&]() {
#pragma clang fp contract(off)  // NC
    const double dalpha = a_hi - a_lo;
    const double lo = fmin(a_hi, a_lo), hi = fmax(a_hi, a_lo);
    const double cchk = 0.2 * dalpha, qchk = 0.1 * dalpha;
    z_failed = z_failed || (dalpha <= 1e-10);
    const double a_cub = cubicmin(a_lo, phi_lo, dphi_lo, a_hi, phi_hi, a_rec, phi_rec);
    const bool use_cubic = (zj > 0) && (a_cub > lo + cchk) && (a_cub < hi - cchk);
    const double a_quad = quadmin(a_lo, phi_lo, dphi_lo, a_hi, phi_hi);
    const bool use_quad = !use_cubic && (a_quad > lo + qchk) && (a_quad < hi - qchk);
    double a_j = a_rec;
    if (use_cubic) a_j = a_cub;
    if (use_quad) a_j = a_quad;
    if (!use_cubic && !use_quad) a_j = (a_lo + a_hi) / 2.0;
    t_trial = a_j;
  };
  // the start: one scan at c0 (norm 1, penalty 0), minimize_bfgs's initial state
  bool pending = false;
  {
#pragma clang fp contract(off)  // NC
    double g0[S];
    const double start = fg(x, g0, refine);
    norm = start * 2.5;
    f = start / norm + 0.0;
#pragma unroll
    for (int s = 0; s < S; ++s) g[s] = g0[s] / norm + 0.0;
#pragma unroll
    for (int s = 0; s < S; ++s)
#pragma unroll
      for (int q = 0; q < MC; ++q) Hr[s][q] = (j + kCoopG * s) == q ? 1.0 : 0.0;
    double gmax = 0.0, g2 = 0.0;
    if constexpr (MC == 16 && INSITE_REFINE_TREE) {
      gmax = fmax(fabs(g[0]), fabs(g[1]));
#pragma unroll
      for (int off = 1; off < kCoopG; off <<= 1) gmax = fmax(gmax, __shfl_xor(gmax, off));  // (max: any order)
      g2 = dot(g, g);
    } else {
#pragma unroll
    for (int i = 0; i < MC; ++i) {
      const double gi = gat(g, i);
      gmax = fmax(gmax, fabs(gi));
      g2 += gi * gi;
    }
    }
    converged = gmax < 1e-5;
    old_old = f + sqrt(g2) / 2.0;
    pending = refine && !converged && k < maxiter;
    if (!converged && k < maxiter) begin_ls();  // (group-uniform; inert rows' values are never used)
  }
  while (__builtin_amdgcn_ballot_w64(pending) != 0ull) {
    double xt[S], g_t[S];
#pragma unroll
    for (int s = 0; s < S; ++s) xt[s] = fma(t_trial, pk[s], x[s]);
    const double phi_t = fg(xt, g_t, pending);
    const double dphi_t = dot(g_t, pk);
    if (!pending) continue;
    bool ls_end = false, ls_done = false, next_zoom = false;
    {
#pragma clang fp contract(off)  // NC
    if (!in_zoom) {
      const double a_i = t_trial;
      const bool s_z1 = (phi_t > phi0 + 1e-4 * a_i * dphi0) || ((phi_t >= phi_i1) && (li > 1));
      const bool s_i = (fabs(dphi_t) <= -0.9 * dphi0) && !s_z1;
      const bool s_z2 = (dphi_t >= 0.0) && !s_z1 && !s_i;
      if (s_i) {
        a_star = a_i;
        phi_star = phi_t;
#pragma unroll
        for (int s = 0; s < S; ++s) g_star[s] = g_t[s];
      }
      if (s_z1 || s_z2) {
        if (s_z1) {
          a_lo = a_i1; phi_lo = phi_i1; dphi_lo = dphi_i1;
          a_hi = a_i; phi_hi = phi_t; dphi_hi = dphi_t;
        } else {
          a_lo = a_i; phi_lo = phi_t; dphi_lo = dphi_t;
          a_hi = a_i1; phi_hi = phi_i1; dphi_hi = dphi_i1;
        }
        zj = 0;
        z_failed = false;
        a_rec = (a_lo + a_hi) / 2.0;
        phi_rec = (phi_lo + phi_hi) / 2.0;
        za = 1.0;
        zphi = phi_lo;
#pragma unroll
        for (int s = 0; s < S; ++s) g_star[s] = g[s];
        in_zoom = true;
      }
      ++li;
      a_i1 = a_i;
      phi_i1 = phi_t;
      dphi_i1 = dphi_t;
      if (in_zoom) {
        next_zoom = true;
      } else if (s_i) {
        ls_end = ls_done = true;
      } else if (li > 10) {
        ls_end = true;
      } else {
        t_trial = a_i1 * 2.0;
      }
    } else {
      const double a_j = t_trial;
      const bool hi_to_j = (phi_t > phi0 + 1e-4 * a_j * dphi0) || (phi_t >= phi_lo);
      const bool star_to_j = (fabs(dphi_t) <= -0.9 * dphi0) && !hi_to_j;
      const bool hi_to_lo = (dphi_t * (a_hi - a_lo) >= 0.0) && !hi_to_j && !star_to_j;
      const bool lo_to_j = !hi_to_j && !star_to_j;
      if (hi_to_j) {
        a_rec = a_hi;
        phi_rec = phi_hi;
        a_hi = a_j;
        phi_hi = phi_t;
        dphi_hi = dphi_t;
      }
      if (star_to_j) {
        za = a_j;
        zphi = phi_t;
#pragma unroll
        for (int s = 0; s < S; ++s) g_star[s] = g_t[s];
      }
      if (hi_to_lo) {
        a_rec = a_hi;
        phi_rec = phi_hi;
        a_hi = a_lo;
        phi_hi = phi_lo;
        dphi_hi = dphi_lo;
      }
      if (lo_to_j) {
        a_rec = a_lo;
        phi_rec = phi_lo;
        a_lo = a_j;
        phi_lo = phi_t;
        dphi_lo = dphi_t;
      }
      ++zj;
      z_failed = ((z_failed ? 1 : 0) | zj) >= 30;  // jax: `failed | j >= 30` (no parentheses)
      if (star_to_j || z_failed) {
        a_star = za;
        phi_star = zphi;
        ls_failed = ls_failed || z_failed;
        ls_end = ls_done = true;
      } else {
        next_zoom = true;
      }
    }
    if (next_zoom) zoom_top();  // one copy for both phases (BfgsFlat::advance)
    }
    if (!ls_end) continue;
    ls_status = ls_failed ? 1 : (li > 10 ? 3 : 0);
    failed = ls_failed || !ls_done;
    {
#pragma clang fp contract(off)  // NC
    double sk[S], yk[S];
#pragma unroll
    for (int s = 0; s < S; ++s) {
      sk[s] = a_star * pk[s];
      yk[s] = g_star[s] - g[s];
    }
    const double rho = 1.0 / dot(yk, sk);
    if (isfinite(rho)) {
      double hy[S];
#pragma unroll
      for (int s = 0; s < S; ++s) hy[s] = 0.0;
      if constexpr (kLdsv) {
        vx_store(yk, 0);
#pragma unroll
        for (int q = 0; q < MC / 2; ++q) {
          const double2 yq = vx_load2(0, q);
#pragma unroll
          for (int s = 0; s < S; ++s) {
            if constexpr (INSITE_REFINE_FUSEDUPD) {
              hy[s] = fma(Hr[s][2 * q], yq.x, hy[s]);
              hy[s] = fma(Hr[s][2 * q + 1], yq.y, hy[s]);
            } else {
              hy[s] += Hr[s][2 * q] * yq.x;
              hy[s] += Hr[s][2 * q + 1] * yq.y;
            }
          }
        }
      } else {
#pragma unroll
      for (int q = 0; q < MC; ++q) {
        const double yq = gat(yk, q);
#pragma unroll
        for (int s = 0; s < S; ++s) hy[s] += Hr[s][q] * yq;
      }
      }
      const double yhy = dot(yk, hy);  // sum_i yk_i hy_i (coord_sum's order)
      const double cs = rho * rho * yhy + rho;
      if constexpr (kLdsv && INSITE_REFINE_FUSEDUPD) {
        double w[S], u[S];
#pragma unroll
        for (int s = 0; s < S; ++s) {
          w[s] = -rho * hy[s];
          u[s] = fma(cs, sk[s], w[s]);
        }
        vx_store(u, 0);
        vx_store(sk, 1);
#pragma unroll
        for (int q = 0; q < MC / 2; ++q) {
          const double2 uq = vx_load2(0, q), sq = vx_load2(1, q);
#pragma unroll
          for (int s = 0; s < S; ++s) {
            Hr[s][2 * q] = fma(sk[s], uq.x, fma(w[s], sq.x, Hr[s][2 * q]));
            Hr[s][2 * q + 1] = fma(sk[s], uq.y, fma(w[s], sq.y, Hr[s][2 * q + 1]));
          }
        }
      } else if constexpr (kLdsv) {
        vx_store(hy, 0);
        vx_store(sk, 1);
#pragma unroll
        for (int q = 0; q < MC / 2; ++q) {
          const double2 hq = vx_load2(0, q), sq = vx_load2(1, q);
#pragma unroll
          for (int s = 0; s < S; ++s) {
            Hr[s][2 * q] = Hr[s][2 * q] - rho * (sk[s] * hq.x + hy[s] * sq.x) + cs * (sk[s] * sq.x);
            Hr[s][2 * q + 1] = Hr[s][2 * q + 1] - rho * (sk[s] * hq.y + hy[s] * sq.y) + cs * (sk[s] * sq.y);
          }
        }
      } else {
#pragma unroll
      for (int q = 0; q < MC; ++q) {
        const double hq = gat(hy, q), sq = gat(sk, q);
#pragma unroll
        for (int s = 0; s < S; ++s)
          Hr[s][q] = Hr[s][q] - rho * (sk[s] * hq + hy[s] * sq) + cs * (sk[s] * sq);
      }
      }
    }
    double gm = 0.0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      x[s] = x[s] + sk[s];
      g[s] = g_star[s];
    }
#pragma unroll
    for (int s = 0; s < S; ++s) gm = fmax(gm, fabs(g[s]));
#pragma unroll
    for (int off = 1; off < kCoopG; off <<= 1) gm = fmax(gm, __shfl_xor(gm, off));  // (max: any order)
    converged = gm < 1e-5;
    old_old = f;
    f = phi_star;
    ++k;
    pending = !converged && !failed && k < maxiter;
    }
    if (pending) begin_ls();
  }
  int status = -1, nit = 0;
  if (refine) {
    nit = k;
    status = converged ? 0 : (k == maxiter ? 1 : (failed ? 2 + ls_status : -1));
    if (status == 3 && ra.revert3) {
#pragma unroll
      for (int s = 0; s < S; ++s) x[s] = c0a[s];
    }
  }
  // ---- final Euler scan with every coefficient (insite_refine_kernel's, replicated in the group's lanes) ----
  double xf[MC];
#pragma unroll
  for (int i = 0; i < MC; ++i) xf[i] = kLdsv ? 0.0 : gat(x, i);
  if constexpr (kLdsv) {
    vx_store(x, 0);
#pragma unroll
    for (int q = 0; q < MC / 2; ++q) {
      const double2 xq = vx_load2(0, q);
      xf[2 * q] = xq.x;
      xf[2 * q + 1] = xq.y;
    }
  }
  auto coef_at = [&](int q) -> double {
    double c = ra.c0[q];
#pragma unroll
    for (int i = 0; i < MC; ++i)
      if (i < ra.m && ra.t_flat[i] == q) c = xf[i];
    return c;
  };
  if (!valid) return;
  double gam[NA][2];
#pragma unroll
  for (int a = 0; a < NA; ++a) gam[a][0] = gam[a][1] = 0.0;
  for (int q = 0; q < ra.n_coef; ++q) {
#pragma clang fp contract(off)  // NC
    const int code = ra.q_code[q], mk = ra.q_mask[q], ex = code >> 24;
    const double t = coef_at(q) * monomial_code(code & 0xffffff, uu);
#pragma unroll
    for (int a = 0; a < NA; ++a)
      if ((mk >> a) & 1)
#pragma unroll
        for (int e = 0; e <= 1; ++e)
          if (ex == e) gam[a][e] += t;
  }
  const double h = ra.dt / (double)ra.sub;
  double y = v_at(0);
  for (int kk = 0; kk < ra.T; ++kk) {
    const int ak = a_at(kk);
    double gk0 = gam[0][0], gk1 = gam[0][1];
#pragma unroll
    for (int a = 1; a < NA; ++a)
      if (ak == a) {
        gk0 = gam[a][0];
        gk1 = gam[a][1];
      }
    for (int s = 0; s < ra.sub; ++s) y = y + h * (gk0 + gk1 * y);
    if ((kk & (kCoopG - 1)) == j) ra.preds[PM ? p * ra.ldp + kk : (int64_t)kk * ra.ldp + p] = y;
  }
  if (ra.coef_out)
    for (int q = j; q < ra.n_coef; q += kCoopG) ra.coef_out[p * ra.n_coef + q] = coef_at(q);
  if (j == 0) {
    if (ra.status) ra.status[p] = status;
    if (ra.iters) ra.iters[p] = nit;
    if (ra.nfev) ra.nfev[p] = nev;
  }
}

// The dynamic kernel's queue heads: device words handed out round-robin per launch (zeroed on the launch's stream
// first); kRefineQueues launches may be in flight on independent streams at once.
constexpr int kRefineQueues = 64;
__device__ unsigned g_refine_queue[kRefineQueues];
unsigned* refine_queue_slot() {
  static std::atomic<unsigned> next{0};
  void* base = nullptr;
  if (hipGetSymbolAddress(&base, HIP_SYMBOL(g_refine_queue)) != hipSuccess || !base) return nullptr;
  return static_cast<unsigned*>(base) + (next.fetch_add(1u) % kRefineQueues);
}

template <int NA, int D>
void launch_refine(const RefineArgs& ra, dim3 grid, hipStream_t hs) {
  const int m = ra.m;
  // the windowed M <= 4 kernels (INSITE_REFINE_WIN): the reference's sequences (T <= 64: one 64-bit arm mask per
  // lane), identity lane order (the binned layout gathers rows instead), even ldv (16-B ring loads)
  const bool win = INSITE_REFINE_WIN && INSITE_REFINE_FLAT && NA == 2 && ra.T <= 64 && ra.T >= 2 && !ra.order &&
                   ra.ldv % 2 == 0 && ((uintptr_t)ra.V & 15u) == 0;
  if constexpr (D == 1 && NA == 2) {
    if (ra.pm) {  // insite_refine_rows_f64 checked m <= 3, T <= 64, the 16-B alignment of V
      const char* dv = getenv("INSITE_REFINE_DYN");
      const bool dyn = dv ? dv[0] == '1' : INSITE_REFINE_DYN != 0;
      if (dyn && ra.coef_out) {
        // a persistent grid: every resident block of the kernel (the occupancy query), capped by the row count
        int dev = 0, cus = 256, per_cu = 3;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
          cus = 256;
        hipError_t oe = m <= 2 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, insite_refine_dyn_kernel<2>, kBlock, 0)
                               : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, insite_refine_dyn_kernel<3>, kBlock, 0);
        if (oe != hipSuccess || per_cu < 1) per_cu = 3;
        int64_t nb = (int64_t)cus * per_cu;
        const char* gv = getenv("INSITE_REFINE_DYN_BLOCKS");
        if (gv && atoll(gv) > 0) nb = atoll(gv);
        const int64_t need = (ra.N + kBlock - 1) / kBlock;
        if (nb > need) nb = need;
        unsigned* queue = refine_queue_slot();
        if (queue && hipMemsetAsync(queue, 0, sizeof(unsigned), hs) == hipSuccess) {  // else: the static kernel
          const dim3 gd((unsigned)nb);
          const char* fv = getenv("INSITE_REFINE_DYN_REFILL");
          const int refill = fv && atoi(fv) > 0 ? atoi(fv) : INSITE_REFINE_DYN_REFILL;
          if (m <= 2) insite_refine_dyn_kernel<2><<<gd, kBlock, 0, hs>>>(ra, queue, refill);
          else insite_refine_dyn_kernel<3><<<gd, kBlock, 0, hs>>>(ra, queue, refill);
          const int staged_arm = (ra.lda % 4 == 0) && (((uintptr_t)ra.arm8 & 3u) == 0) && ra.lda <= 64;
          insite_refine_final_kernel<2><<<grid, kBlock, 0, hs>>>(ra, staged_arm);
          return;
        }
      }
      if (m <= 2) insite_refine_kernel<2, NA, D, true, true><<<grid, kBlock, 0, hs>>>(ra);
      else insite_refine_kernel<3, NA, D, true, true><<<grid, kBlock, 0, hs>>>(ra);
      return;
    }
    // (m = 4: the 16-entry H in LDS plus the ring would hold the CU to 2 blocks; the per-step-load kernel runs it)
    if (win && m <= 3) {
      if (m <= 2) insite_refine_kernel<2, NA, D, true><<<grid, kBlock, 0, hs>>>(ra);
      else insite_refine_kernel<3, NA, D, true><<<grid, kBlock, 0, hs>>>(ra);
      return;
    }
  }
  if constexpr (D == 1) {
    // the sparse models get a kernel sized to their active count (register budget: INSITE_REFINE_WPE4 waves)
    if (m <= 2) insite_refine_kernel<2, NA, D><<<grid, kBlock, 0, hs>>>(ra);
    else if (m == 3) insite_refine_kernel<3, NA, D><<<grid, kBlock, 0, hs>>>(ra);
    else if (m <= 4) insite_refine_kernel<4, NA, D><<<grid, kBlock, 0, hs>>>(ra);
    else if (m <= 6 && INSITE_REFINE_M6) insite_refine_kernel<6, NA, D><<<grid, kBlock, 0, hs>>>(ra);
    else if (m <= 8) {
      const char* cv = getenv("INSITE_REFINE_COOP8");
      const bool coop = cv ? cv[0] == '1' : INSITE_REFINE_COOP8 != 0;
      if (NA == 4 && ra.pm) {  // the row layout (refine_launch admitted it: COOP8, T <= kCoopStT)
        const dim3 gc((unsigned)((ra.N * kCoopG + kBlock - 1) / kBlock));
        insite_refine_coop_kernel<8, 4, true, true><<<gc, kBlock, 0, hs>>>(ra);
      } else if (NA == 4 && coop) {  // the sparse 4-arm models with 5-8 active terms: 8 lanes per row, one coordinate a lane
        const dim3 gc((unsigned)((ra.N * kCoopG + kBlock - 1) / kBlock));
        if (ra.T <= kCoopStT) insite_refine_coop_kernel<8, 4, true><<<gc, kBlock, 0, hs>>>(ra);
        else insite_refine_coop_kernel<8, 4, false><<<gc, kBlock, 0, hs>>>(ra);
      } else {
        insite_refine_kernel<8, NA, D><<<grid, kBlock, 0, hs>>>(ra);
      }
    }
    else if (m <= 16) {
      const char* cv = getenv("INSITE_REFINE_COOP");
      const bool coop = cv ? cv[0] == '1' : INSITE_REFINE_COOP != 0;
      if (NA == 4 && ra.pm) {  // the row layout (refine_launch admitted it: coop, T <= kCoopStT)
        const dim3 gc((unsigned)((ra.N * kCoopG + kBlock - 1) / kBlock));
        insite_refine_coop_kernel<16, 4, true, true><<<gc, kBlock, 0, hs>>>(ra);
      } else if (NA == 4 && coop) {  // the dense 4-arm models (int8 arms): 8 lanes per row
        const dim3 gc((unsigned)((ra.N * kCoopG + kBlock - 1) / kBlock));
        if (ra.T <= kCoopStT) insite_refine_coop_kernel<16, 4, true><<<gc, kBlock, 0, hs>>>(ra);
        else insite_refine_coop_kernel<16, 4, false><<<gc, kBlock, 0, hs>>>(ra);
      } else {
        insite_refine_kernel<16, NA, D><<<grid, kBlock, 0, hs>>>(ra);
      }
    }
    else if (m <= 36) insite_refine_kernel<36, NA, D><<<grid, kBlock, 0, hs>>>(ra);
    else insite_refine_kernel<kRefineMaxCoef, NA, D><<<grid, kBlock, 0, hs>>>(ra);
  } else {
    if (m <= 8) insite_refine_kernel<8, NA, D><<<grid, kBlock, 0, hs>>>(ra);
    else insite_refine_kernel<kRefineMaxCoef, NA, D><<<grid, kBlock, 0, hs>>>(ra);
  }
}

// Shared argument checks and launch.  Coefficient q of coef0 [n_coef] acts on the arms of mask[q] with
// state exponent exps[q][0] and static exponents exps[q][1..].
int32_t refine_launch(const double* V, int64_t ld_v, int32_t T, const uint32_t* arm_bits, const int8_t* arm8,
                      int64_t ld_arm, const double* u, const int32_t* seq_len, int64_t n_rows, int32_t n_statics,
                      int32_t n_coef, const double* coef0, const int32_t* mask, const int8_t* exps, int32_t n_arms,
                      double dt, double lam, int32_t tau, int32_t substeps, int32_t revert_on_zoom_fail,
                      double* preds, int64_t ld_p, double* coef_out, int32_t* status_out, int32_t* iters_out,
                      const int32_t* row_order, void* stream, int32_t* nfev_out = nullptr, bool pm = false) {
  const bool bits = arm8 == nullptr;
  // pm: the row layout of insite_refine_rows_f64 (patient-major V / arm8 / preds, leading dimensions >= T)
  const int64_t ld_min = pm ? T : n_rows;
  if (n_rows < 0 || T < 1 || n_arms < 1 || n_arms > (bits ? 2 : 4) || substeps < 1 || !(dt > 0.0) ||
      !(lam >= 0.0) || tau < 0 || ld_v < ld_min || ld_p < ld_min || n_statics < 0 ||
      n_statics > INSITE_MAX_STATICS || ld_arm < (pm ? T : (bits ? (n_rows + 31) / 32 : n_rows)) || !coef0 ||
      !mask || !exps || n_coef < 1 || (pm && bits))
    return INSITE_E_INVALID_ARG;
  if (n_coef > kRefineMaxCoef) return INSITE_E_UNSUPPORTED;
  RefineArgs ra{};
  int D = 1, m = 0;
  for (int q = 0; q < n_coef; ++q) {
    const int8_t* e = exps + (int64_t)q * (1 + n_statics);
    if (e[0] < 0) return INSITE_E_INVALID_ARG;
    if (e[0] > 4) return INSITE_E_UNSUPPORTED;
    int code = 0;
    for (int i = 0; i < n_statics; ++i) {
      if (e[1 + i] < 0 || e[1 + i] > 8) return INSITE_E_INVALID_ARG;
      code |= (int)e[1 + i] << (8 * i);
    }
    if (mask[q] < 0 || mask[q] >= (1 << n_arms)) return INSITE_E_INVALID_ARG;
    const double c = coef0[q];
    ra.c0[q] = c;
    ra.q_mask[q] = mask[q];
    ra.q_code[q] = code | ((int)e[0] << 24);
    if (c != 0.0 && e[0] > 1) D = 4;  // a non-affine term in the model: the state-polynomial kernels
    if (fabs(c) > 1e-3) {             // coef_sparse_mask (sindy.py:587)
      ra.t_flat[m] = q;
      ra.t_mask[m] = mask[q];
      ra.t_ex[m] = e[0];
      ra.t_ucode[m] = code;
      ++m;
    }
  }
  if (m <= 4) {  // RefineArgs::gmap (used by the M <= 4, D = 1 kernels)
    for (int i = 0; i < m; ++i)
      for (int a = 0; a < n_arms; ++a)
        if ((ra.t_mask[i] >> a) & 1) ra.gmap |= 1 << (i * 8 + a * 2 + (ra.t_ex[i] & 1));
  }
  if (pm && n_arms <= 2 &&
      (D != 1 || m > 3 || T < 2 || T > 64 || (ld_v & 1) || ((uintptr_t)V & 15u) || n_rows > INT32_MAX))
    return INSITE_E_UNSUPPORTED;  // the windowed row kernel's shape (the reference's sequences: T <= 64, <= 3 active)
  if (pm && n_arms > 2) {  // 3-4 arms: the cooperative kernel on the rows (the dense models, 9-16 active terms; the
                           // sparse 5-8-term ones where the 8-coordinate cooperative kernel is selected, COOP8)
    const char* cv = getenv(m <= 8 ? "INSITE_REFINE_COOP8" : "INSITE_REFINE_COOP");
    const bool coop = cv ? cv[0] == '1' : (m <= 8 ? INSITE_REFINE_COOP8 : INSITE_REFINE_COOP) != 0;
    if (D != 1 || m <= (INSITE_REFINE_M6 ? 6 : 4) || m > 16 || !coop || T > kCoopStT || n_rows > INT32_MAX)
      return INSITE_E_UNSUPPORTED;
  }
  if (n_rows == 0) return INSITE_OK;
  if (!V || (bits && !arm_bits) || !seq_len || !preds || (n_statics > 0 && !u)) return INSITE_E_INVALID_ARG;
  ra.V = V;
  ra.arm = arm_bits;
  ra.arm8 = arm8;
  ra.u = n_statics > 0 ? u : V;
  ra.sl = seq_len;
  ra.preds = preds;
  ra.coef_out = coef_out;
  ra.status = status_out;
  ra.iters = iters_out;
  ra.nfev = nfev_out;
  ra.order = row_order;
  ra.ldv = ld_v;
  ra.lda = ld_arm;
  ra.ldp = ld_p;
  ra.N = n_rows;
  ra.T = T;
  ra.tau = tau;
  ra.sub = substeps;
  ra.U = n_statics;
  ra.revert3 = revert_on_zoom_fail != 0;
  ra.A = n_arms;
  ra.n_coef = n_coef;
  ra.dt = dt;
  ra.lam = lam;
  ra.m = m;
  ra.pm = pm ? 1 : 0;
  ra.st16 = ((uintptr_t)preds & 15u) == 0 && (ld_p & 1) == 0;
  const dim3 grid((unsigned)((n_rows + kBlock - 1) / kBlock));
  hipStream_t hs = reinterpret_cast<hipStream_t>(stream);
  if (bits || (pm && n_arms <= 2)) {
    if (D == 1) launch_refine<2, 1>(ra, grid, hs);
    else launch_refine<2, 4>(ra, grid, hs);
  } else {
    if (D == 1) launch_refine<4, 1>(ra, grid, hs);
    else launch_refine<4, 4>(ra, grid, hs);
  }
  return launch_status();
}

// separate per-arm models [n_arms, F] over the library exps [F][1 + U]: coefficient (a, j) acts on arm a
int32_t refine_per_arm(const double* V, int64_t ld_v, int32_t T, const uint32_t* arm_bits, const int8_t* arm8,
                       int64_t ld_arm, const double* u, const int32_t* seq_len, int64_t n_rows, int32_t n_statics,
                       const int8_t* exps, int32_t n_terms, const double* coef0, int32_t n_arms, double dt, double lam,
                       int32_t tau, int32_t substeps, int32_t revert_on_zoom_fail, double* preds, int64_t ld_p,
                       double* coef_out, int32_t* status_out, int32_t* iters_out, const int32_t* row_order,
                       void* stream) {
  if (!exps || n_terms < 1 || n_arms < 1 || n_arms > INSITE_MAX_ARMS || n_statics < 0 ||
      n_statics > INSITE_MAX_STATICS)
    return INSITE_E_INVALID_ARG;
  const int n_coef = n_arms * n_terms;
  if (n_coef > kRefineMaxCoef) return INSITE_E_UNSUPPORTED;
  int32_t mask[kRefineMaxCoef];
  int8_t qe[kRefineMaxCoef * (1 + INSITE_MAX_STATICS)];
  for (int a = 0; a < n_arms; ++a)
    for (int j = 0; j < n_terms; ++j) {
      const int q = a * n_terms + j;
      mask[q] = 1 << a;
      std::memcpy(qe + q * (1 + n_statics), exps + j * (1 + n_statics), (size_t)(1 + n_statics));
    }
  return refine_launch(V, ld_v, T, arm_bits, arm8, ld_arm, u, seq_len, n_rows, n_statics, n_coef, coef0, mask, qe,
                       n_arms, dt, lam, tau, substeps, revert_on_zoom_fail, preds, ld_p, coef_out, status_out,
                       iters_out, row_order, stream);
}
}  // namespace

int32_t insite_refine_f64(const double* V, int64_t ld_v, int32_t T, const uint32_t* arm_bits, int64_t ld_arm,
                          const double* u, const int32_t* seq_len, int64_t n_rows, int32_t n_statics, const int8_t* exps,
                          int32_t n_terms, const double* coef0, int32_t n_arms, double dt, double lam, int32_t tau,
                          int32_t substeps, int32_t revert_on_zoom_fail, double* preds, int64_t ld_p,
                          double* coef_out, int32_t* status_out, int32_t* iters_out, const int32_t* row_order,
                          void* stream) {
  if (!arm_bits && n_rows > 0) return INSITE_E_INVALID_ARG;
  return refine_per_arm(V, ld_v, T, arm_bits, nullptr, ld_arm, u, seq_len, n_rows, n_statics, exps, n_terms, coef0,
                        n_arms, dt, lam, tau, substeps, revert_on_zoom_fail, preds, ld_p, coef_out, status_out,
                        iters_out, row_order, stream);
}

int32_t insite_refine_arms_f64(const double* V, int64_t ld_v, int32_t T, const int8_t* arm, int64_t ld_arm,
                               const double* u, const int32_t* seq_len, int64_t n_rows, int32_t n_statics,
                               const int8_t* exps, int32_t n_terms, const double* coef0, int32_t n_arms, double dt,
                               double lam, int32_t tau, int32_t substeps, int32_t revert_on_zoom_fail, double* preds,
                               int64_t ld_p, double* coef_out, int32_t* status_out, int32_t* iters_out,
                               const int32_t* row_order, void* stream) {
  if (!arm && n_rows > 0) return INSITE_E_INVALID_ARG;
  static const int8_t kNoArms = 0;  // non-null marker for the int8 format when n_rows == 0
  return refine_per_arm(V, ld_v, T, nullptr, arm ? arm : &kNoArms, ld_arm, u, seq_len, n_rows, n_statics, exps, n_terms, coef0,
                        n_arms, dt, lam, tau, substeps, revert_on_zoom_fail, preds, ld_p, coef_out, status_out,
                        iters_out, row_order, stream);
}

// Layout preparation for the refinement (the reference hands over patient-major [N, T] prev_outputs and per-step
// arms, sindy.py:555-566): one pass writes the time-major V [T, N] and the arms either bit-packed [T, ceil(N/32)]
// (a wave ballots its 64 patients' bits per step: two words, no int64 intermediates) or int8 [T, N].  A wave owns
// 64 patients and walks the steps in chunks of kPrepTc: the 64 x kPrepTc block is read row-segment by row-segment
// (4 rows of 128 B per load instruction) into LDS, then every lane reads its own row back and each store is a
// coalesced 512-B (64-B for int8) step row.  (A lane-per-row gather straight from HBM touched 64 lines per
// load instruction: 1.58 ms for the 1M x 60 INSITE set.)
namespace {
constexpr int kPrepTc = 16;
constexpr int kPrepLd = kPrepTc + 1;  // odd row stride: lane-per-row reads hit distinct banks
// per-row side arrays moved with the rows (ABI 8): lane l <- row r (prepare), row r <- lane l (finish)
struct RowGather {
  const double* u;
  int32_t U;
  double* u_out;
  const int32_t* sl;
  int32_t* sl_out;
  __device__ void gather(int64_t l, int64_t r) const {
    if (u_out)
      for (int i = 0; i < U; ++i) u_out[l * U + i] = u[r * U + i];
    if (sl_out) sl_out[l] = sl[r];
  }
};
struct RowScatter {
  const double* coef;
  int32_t nc;
  double* coef_out;
  const int32_t* st;
  int32_t* st_out;
  const int32_t* it;
  int32_t* it_out;
  __device__ void scatter(int64_t l, int64_t r) const {
    if (coef_out)
      for (int q = 0; q < nc; ++q) coef_out[r * nc + q] = coef[l * nc + q];
    if (st_out) st_out[r] = st[l];
    if (it_out) it_out[r] = it[l];
  }
};
__global__ void __launch_bounds__(kBlock) refine_prepare_kernel(const double* __restrict__ V, int64_t ld_v,
                                                                const int8_t* __restrict__ arm, int64_t ld_arm,
                                                                int64_t N, int32_t T, double* __restrict__ Vt,
                                                                int64_t ld_vt, uint32_t* __restrict__ bits,
                                                                int64_t ld_bits, int8_t* __restrict__ arm_t,
                                                                int64_t ld_armt, const int32_t* __restrict__ order,
                                                                RowGather rg) {
  __shared__ double sv[kWavesPerBlock][kWave * kPrepLd];
  __shared__ int sa[kWavesPerBlock][kWave * kPrepLd];
  const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
  const int64_t p0 = (int64_t)blockIdx.x * kBlock + wv * kWave;  // the wave's first patient
  const int64_t p = p0 + lane;
  const bool act = p < N;
  if (act) rg.gather(p, order ? (int64_t)order[p] : p);
  const int64_t w0 = p0 >> 5;  // the wave's two bit words
  double* lv = sv[wv];
  int* la = sa[wv];
  for (int t0 = 0; t0 < T; t0 += kPrepTc) {
    const int tc = T - t0 < kPrepTc ? T - t0 : kPrepTc;
#pragma unroll 4
    for (int j = 0; j < kWave * kPrepTc / kWave; ++j) {  // element e = j * 64 + lane of the 64 x kPrepTc block
      const int e = j * kWave + lane, r = e / kPrepTc, c = e % kPrepTc;
      const bool ok = c < tc && p0 + r < N;
      const int64_t row = ok ? (order ? (int64_t)order[p0 + r] : p0 + r) : 0;
      lv[r * kPrepLd + c] = ok ? V[row * ld_v + t0 + c] : 0.0;
      if (arm) la[r * kPrepLd + c] = ok ? (int)arm[row * ld_arm + t0 + c] : 0;
    }
    __syncthreads();
    for (int c = 0; c < tc; ++c) {
      const int64_t t = t0 + c;
      if (act) Vt[t * ld_vt + p] = lv[lane * kPrepLd + c];
      if (arm) {
        const int a = la[lane * kPrepLd + c];
        if (bits) {
          const unsigned long long m = __builtin_amdgcn_ballot_w64(act && a != 0);
          if (lane < 2 && (w0 + lane) * 32 < N) bits[t * ld_bits + w0 + lane] = (uint32_t)(m >> (32 * lane));
        } else if (act) {
          arm_t[t * ld_armt + p] = (int8_t)a;
        }
      }
    }
    __syncthreads();
  }
}

// The inverse for the refinement's outputs: time-major preds [T, ld_t] whose column l is row order[l] (or l) ->
// the reference's patient-major [N, ld_pm].  Same staging: coalesced 512-B step rows into LDS, then each load /
// store instruction writes 4 patients' 128-B row segments.
__global__ void __launch_bounds__(kBlock) refine_finish_kernel(const double* __restrict__ P, int64_t ld_t,
                                                               const int32_t* __restrict__ order, int64_t N, int32_t T,
                                                               double* __restrict__ out, int64_t ld_pm, RowScatter rs) {
  __shared__ double sv[kWavesPerBlock][kWave * kPrepLd];
  const int lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
  const int64_t p0 = (int64_t)blockIdx.x * kBlock + wv * kWave;
  const int64_t l = p0 + lane;
  if (l < N) rs.scatter(l, order ? (int64_t)order[l] : l);
  double* lv = sv[wv];
  for (int t0 = 0; t0 < T; t0 += kPrepTc) {
    const int tc = T - t0 < kPrepTc ? T - t0 : kPrepTc;
    for (int c = 0; c < tc; ++c) lv[lane * kPrepLd + c] = l < N ? P[(int64_t)(t0 + c) * ld_t + l] : 0.0;
    __syncthreads();
#pragma unroll 4
    for (int j = 0; j < kPrepTc; ++j) {
      const int e = j * kWave + lane, r = e / kPrepTc, c = e % kPrepTc;
      if (c < tc && p0 + r < N) {
        const int64_t row = order ? (int64_t)order[p0 + r] : p0 + r;
        out[row * ld_pm + t0 + c] = lv[r * kPrepLd + c];
      }
    }
    __syncthreads();
  }
}

// T <= 64 (the reference's sequences: 60 steps): one wave per block stages its 64 patients' WHOLE rows, so every
// cache line of V is consumed in one phase (the chunked form re-touched the lines a row segment shares with the
// next chunk after they had left the L2).  Load: one instruction per patient row (lanes = steps, up to 512 B
// contiguous); store: one instruction per step (lanes = patients, 512 B).  Measured slower than the chunked
// 4-wave form (INSITE step 5.03 vs 4.69 ms, profiles/r03/v37_insite_variants.txt: one wave per block at 35 KB of
// LDS leaves 4 waves per CU), so off by default; INSITE_PREP_ROWS=1 selects it for T <= 64.
#ifndef INSITE_PREP_ROWS
#define INSITE_PREP_ROWS 0
#endif
constexpr int kRowLd = kWave + 1;
__global__ void __launch_bounds__(kWave) refine_prepare_rows_kernel(const double* __restrict__ V, int64_t ld_v,
                                                                    const int8_t* __restrict__ arm, int64_t ld_arm,
                                                                    int64_t N, int32_t T, double* __restrict__ Vt,
                                                                    int64_t ld_vt, uint32_t* __restrict__ bits,
                                                                    int64_t ld_bits, int8_t* __restrict__ arm_t,
                                                                    int64_t ld_armt, const int32_t* __restrict__ order,
                                                                    RowGather rg) {
  __shared__ double lv[kWave * kRowLd];
  __shared__ int8_t la[kWave * kRowLd];
  const int lane = threadIdx.x;
  const int64_t p0 = (int64_t)blockIdx.x * kWave;
  const int nr = N - p0 < kWave ? (int)(N - p0) : kWave;
  if (lane < nr) rg.gather(p0 + lane, order ? (int64_t)order[p0 + lane] : p0 + lane);
  for (int r = 0; r < nr; ++r) {
    const int64_t row = order ? (int64_t)order[p0 + r] : p0 + r;
    if (lane < T) {
      lv[r * kRowLd + lane] = V[row * ld_v + lane];
      if (arm) la[r * kRowLd + lane] = arm[row * ld_arm + lane];
    }
  }
  __syncthreads();
  const int64_t p = p0 + lane;
  const bool act = lane < nr;
  const int64_t w0 = p0 >> 5;
  for (int t = 0; t < T; ++t) {
    if (act) Vt[(int64_t)t * ld_vt + p] = lv[lane * kRowLd + t];
    if (arm) {
      const int a = act ? (int)la[lane * kRowLd + t] : 0;
      if (bits) {
        const unsigned long long m = __builtin_amdgcn_ballot_w64(act && a != 0);
        if (lane < 2 && (w0 + lane) * 32 < N) bits[(int64_t)t * ld_bits + w0 + lane] = (uint32_t)(m >> (32 * lane));
      } else if (act) {
        arm_t[(int64_t)t * ld_armt + p] = (int8_t)a;
      }
    }
  }
}

__global__ void __launch_bounds__(kWave) refine_finish_rows_kernel(const double* __restrict__ P, int64_t ld_t,
                                                                   const int32_t* __restrict__ order, int64_t N,
                                                                   int32_t T, double* __restrict__ out, int64_t ld_pm,
                                                                   RowScatter rs) {
  __shared__ double lv[kWave * kRowLd];
  const int lane = threadIdx.x;
  const int64_t p0 = (int64_t)blockIdx.x * kWave;
  const int nr = N - p0 < kWave ? (int)(N - p0) : kWave;
  if (lane < nr) rs.scatter(p0 + lane, order ? (int64_t)order[p0 + lane] : p0 + lane);
  if (lane < nr)
    for (int t = 0; t < T; ++t) lv[lane * kRowLd + t] = P[(int64_t)t * ld_t + p0 + lane];
  __syncthreads();
  for (int r = 0; r < nr; ++r) {
    const int64_t row = order ? (int64_t)order[p0 + r] : p0 + r;
    if (lane < T) out[row * ld_pm + lane] = lv[r * kRowLd + lane];
  }
}
}  // namespace

extern "C" int32_t insite_refine_finish_f64(const double* preds_tm, int64_t ld_t, const int32_t* row_order,
                                            int64_t n_rows, int32_t T, double* preds_pm, int64_t ld_pm,
                                            const double* coef_lane, int32_t n_coef, double* coef_out,
                                            const int32_t* status_lane, int32_t* status_out, const int32_t* iters_lane,
                                            int32_t* iters_out, void* stream) {
  if (n_rows < 0 || T < 1 || !preds_tm || !preds_pm || ld_t < n_rows || ld_pm < T) return INSITE_E_INVALID_ARG;
  if ((coef_lane == nullptr) != (coef_out == nullptr) || (status_lane == nullptr) != (status_out == nullptr) ||
      (iters_lane == nullptr) != (iters_out == nullptr) || (coef_out && n_coef < 1))
    return INSITE_E_INVALID_ARG;
  if (n_rows == 0) return INSITE_OK;
  const RowScatter rs{coef_lane, n_coef, coef_out, status_lane, status_out, iters_lane, iters_out};
  if (INSITE_PREP_ROWS && T <= kWave) {
    refine_finish_rows_kernel<<<dim3((unsigned)((n_rows + kWave - 1) / kWave)), kWave, 0,
                                static_cast<hipStream_t>(stream)>>>(preds_tm, ld_t, row_order, n_rows, T, preds_pm, ld_pm,
                                                                    rs);
    return hipGetLastError() == hipSuccess ? INSITE_OK : INSITE_E_HIP;
  }
  const dim3 grid((unsigned)((n_rows + kBlock - 1) / kBlock));
  refine_finish_kernel<<<grid, kBlock, 0, static_cast<hipStream_t>(stream)>>>(preds_tm, ld_t, row_order, n_rows, T,
                                                                              preds_pm, ld_pm, rs);
  return hipGetLastError() == hipSuccess ? INSITE_OK : INSITE_E_HIP;
}

extern "C" int32_t insite_refine_prepare_f64(const double* V, int64_t ld_v, const int8_t* arm, int64_t ld_arm,
                                             int64_t n_rows, int32_t T, double* Vt, int64_t ld_vt, uint32_t* arm_bits,
                                             int64_t ld_bits, int8_t* arm_t, int64_t ld_armt,
                                             const int32_t* row_order, const double* u, int32_t n_statics,
                                             double* u_out, const int32_t* seq_len, int32_t* seq_len_out,
                                             void* stream) {
  if (n_rows < 0 || T < 1 || !V || !Vt || ld_v < T || ld_vt < n_rows) return INSITE_E_INVALID_ARG;
  if (arm && (ld_arm < T || (arm_bits == nullptr) == (arm_t == nullptr))) return INSITE_E_INVALID_ARG;
  if (arm_bits && ld_bits < (n_rows + 31) / 32) return INSITE_E_INVALID_ARG;
  if (arm_t && ld_armt < n_rows) return INSITE_E_INVALID_ARG;
  if ((u_out && (!u || n_statics < 1 || n_statics > INSITE_MAX_STATICS)) || (seq_len_out && !seq_len))
    return INSITE_E_INVALID_ARG;
  if (n_rows == 0) return INSITE_OK;
  const RowGather rg{u, n_statics, u_out, seq_len, seq_len_out};
  if (INSITE_PREP_ROWS && T <= kWave) {
    refine_prepare_rows_kernel<<<dim3((unsigned)((n_rows + kWave - 1) / kWave)), kWave, 0,
                                 static_cast<hipStream_t>(stream)>>>(
        V, ld_v, arm, ld_arm, n_rows, T, Vt, ld_vt, arm ? arm_bits : nullptr, ld_bits, arm ? arm_t : nullptr, ld_armt,
        row_order, rg);
    return hipGetLastError() == hipSuccess ? INSITE_OK : INSITE_E_HIP;
  }
  const dim3 grid((unsigned)((n_rows + kBlock - 1) / kBlock));
  refine_prepare_kernel<<<grid, kBlock, 0, static_cast<hipStream_t>(stream)>>>(
      V, ld_v, arm, ld_arm, n_rows, T, Vt, ld_vt, arm ? arm_bits : nullptr, ld_bits, arm ? arm_t : nullptr, ld_armt,
      row_order, rg);
  return hipGetLastError() == hipSuccess ? INSITE_OK : INSITE_E_HIP;
}

int32_t insite_refine_general_f64(const double* V, int64_t ld_v, int32_t T, const uint32_t* arm_bits,
                                  const int8_t* arm, int64_t ld_arm, const double* u, const int32_t* seq_len,
                                  int64_t n_rows, int32_t n_statics, int32_t n_coef, const double* coef0,
                                  const int32_t* coef_arm_mask, const int8_t* coef_exps, int32_t n_arms, double dt,
                                  double lam, int32_t tau, int32_t substeps, int32_t revert_on_zoom_fail,
                                  double* preds, int64_t ld_p, double* coef_out, int32_t* status_out,
                                  int32_t* iters_out, int32_t* nfev_out, const int32_t* row_order, void* stream) {
  if ((arm_bits == nullptr) == (arm == nullptr) && n_rows > 0) return INSITE_E_INVALID_ARG;
  static const int8_t kNoArms = 0;  // non-null marker for the int8 format when n_rows == 0
  return refine_launch(V, ld_v, T, arm_bits, arm_bits ? nullptr : (arm ? arm : &kNoArms), ld_arm, u, seq_len, n_rows, n_statics, n_coef,
                       coef0, coef_arm_mask, coef_exps, n_arms, dt, lam, tau, substeps, revert_on_zoom_fail, preds,
                       ld_p, coef_out, status_out, iters_out, row_order, stream, nfev_out);
}

int32_t insite_refine_rows_f64(const double* V, int64_t ld_v, int32_t T, const int8_t* arm, int64_t ld_arm,
                               const double* u, const int32_t* seq_len, int64_t n_rows, int32_t n_statics,
                               int32_t n_coef, const double* coef0, const int32_t* coef_arm_mask,
                               const int8_t* coef_exps, int32_t n_arms, double dt, double lam, int32_t tau,
                               int32_t substeps, int32_t revert_on_zoom_fail, double* preds, int64_t ld_p,
                               double* coef_out, int32_t* status_out, int32_t* iters_out, int32_t* nfev_out,
                               const int32_t* row_order, void* stream) {
  static const int8_t kNoArms = 0;
  if (!arm && n_rows > 0) return INSITE_E_INVALID_ARG;
  return refine_launch(V, ld_v, T, nullptr, arm ? arm : &kNoArms, ld_arm, u, seq_len, n_rows, n_statics, n_coef, coef0,
                       coef_arm_mask, coef_exps, n_arms, dt, lam, tau, substeps, revert_on_zoom_fail, preds, ld_p,
                       coef_out, status_out, iters_out, row_order, stream, nfev_out, true);
}
