// insite_ms.hip — multi-state (S > 1) path of the INSITE hot path on MI355X (gfx950): configuration C3
// of BASELINE.json (5-state coupled ODE + binary per-step treatment, fp32 storage, fp64 Gram).
//
// Kernels:
//   gram_ms_kernel     fused savgol(5,3) smoothing + FD4 derivatives of S states + degree-2 polynomial
//                      library over (x_1..x_S, a) + the Gram Y^T Z, Y = Theta, Z = [Theta | xdot], on
//                      v_mfma_f64_16x16x4f64.  Lane = patient; every step the wave stages its 64 library
//                      rows [Theta | xdot] (<= 32 doubles each) in LDS and issues 16 x 2 or 3 MFMAs (tiles
//                      Y0^T Z0, Y0^T Z1 of the 32 x 32 padded product; the Y1^T Z0 tile is the
//                      transpose of part of Y0^T Z1) and, for F > 16, the Y1^T Z1 tile (MsTail).
//                      Interior rows stream through compile-time register rings; the 4 + 4 edge rows per patient use the one-sided stencils from directly
//                      loaded end windows.  Replaces pysindy SmoothedFiniteDifference + PolynomialLibrary
//                      + X^T X (reference sindy.py:186-192) generalised to S states.
//   ms_finalize        fixed-order reduction of the per-block tile partials -> G [F, F], B [F, S].
//   stlsq_wave_kernel  one wavefront per target state: STLSQ (pkpd/utils.py:213-327 semantics) with a
//                      lane-per-row masked Cholesky in LDS (F <= 32, beyond the register-resident
//                      one-thread solver of insite_hip.hip).
//   rollout_ms_kernel  lane = patient, S-dimensional state in fp32 registers, RK4 / Euler of the dense
//                      degree-2 RHS, per-step treatment bits (32 steps per register via the half-wave bit
//                      transpose), non-temporal stores of [T][S][N] fp32 trajectories.
#include <hip/hiprtc.h>

#include <cmath>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "insite_common.h"

namespace {

constexpr int kMsMaxF = 32;       // library columns: Y has two 16-row MFMA tiles
constexpr int kMsMaxS = 8;        // states
constexpr int kMsRowStride = 33;  // LDS stride (doubles) of a staged [Theta | xdot | 0] row
constexpr int kMsMaxBlocks = 512;
constexpr int kMsTiles = 3;       // Y0^T Z0, Y0^T Z1, Y1^T Z1

// Number of degree-<=2 polynomial columns over n inputs (bias, linear, pairwise) in pysindy order.
__host__ __device__ constexpr int ms_cols(int n, bool inter) { return 1 + n + (inter ? n * (n - 1) / 2 : n * (n + 1) / 2); }

// Library columns over z = [1, x_1..x_S, a_1..a_NIN]: column index j -> (z index i, z index k),
// pysindy order (bias; linear; products by combinations(_with_replacement)).  Compile-time.
template <int NZ, bool INTER>  // NZ = S + NIN inputs
struct PolyCols {
  static constexpr int F = ms_cols(NZ, INTER);
  int ci[F], ck[F];
  constexpr PolyCols() : ci(), ck() {
    int j = 0;
    ci[j] = 0; ck[j] = 0; ++j;                    // 1
    for (int i = 0; i < NZ; ++i) { ci[j] = 1 + i; ck[j] = 0; ++j; }
    for (int i = 0; i < NZ; ++i)
      for (int k = INTER ? i + 1 : i; k < NZ; ++k) { ci[j] = 1 + i; ck[j] = 1 + k; ++j; }
  }
};

// Library row Theta[F] from z[NZ + 1] (z[0] = 1).
template <int NZ, bool INTER>
__device__ __forceinline__ void poly_row(const double (&z)[NZ + 1], double (&th)[PolyCols<NZ, INTER>::F]) {
  constexpr PolyCols<NZ, INTER> pc;
#pragma unroll
  for (int j = 0; j < PolyCols<NZ, INTER>::F; ++j) th[j] = pc.ck[j] == 0 ? z[pc.ci[j]] : z[pc.ci[j]] * z[pc.ck[j]];
}

// Fetch bit (lane & 31) of word row k of a TIME_MAJOR_BITS mask for patient p (edge rows only).
__device__ __forceinline__ double input_bit(const uint32_t* __restrict__ abits, int64_t lda, int k, int64_t p) {
  if (!abits) return 0.0;
  return (double)((abits[(int64_t)k * lda + (p >> 5)] >> (p & 31)) & 1u);
}

// The tail: rows 16.. of Y (F1 = F - 16 library columns) against Z1 = [Theta_16.. | xdot]
// (F = 22: 6 rows x 11 columns).  As a 16 x 16 f64 MFMA tile it has 16 - F1 padding rows (F = 22:
// 10 of 16, a third of the kernel's MFMA work; F <= 16: all of them, so it is never issued then).
// INSITE_MS_TAIL selects how it is computed when F > 16:
//   0  the 16 x 16 x 4 tile (16 MFMAs per 64 rows);
//   1  per-lane VALU FMAs into F1 (F1 + 1) / 2 + F1 S accumulators; at F = 22 the 51 accumulators
//      (102 VGPRs) push the occupancy-2 kernel into scratch (C3: 15.5 -> 33.2 ms; at occupancy 1
//      15.8 ms, the 16 x 16 tile at occupancy 1 18.7 ms);
//   2  v_mfma_f64_4x4x4f64 (4 blocks of 4 x 4 x 4; A[b][m][k] in lane 16k + 4b + m, B[b][k][n] in
//      lane 16k + 4b + n, D[b][m][n] in lane 16m + 4b + n: tools/probe/mfma_f64_4x4_probe.hip): the
//      tail cut into 4 x 4 blocks (row group rg < RG, column group cg >= rg: the upper triangle and
//      every xdot column; F = 22: 5 blocks), each block type one accumulator double per lane whose 4
//      MFMA blocks take different rows; 20 MFMAs of 1/4 the work per 64 rows (default).
#ifndef INSITE_MS_TAIL
#define INSITE_MS_TAIL 2
#endif
#ifndef INSITE_MS_WPE
#define INSITE_MS_WPE 2
#endif
constexpr int kTailMfma16 = 0, kTailValu = 1, kTailMfma4 = 2, kTailNone = 3;
template <int S, int F>
struct MsTail {
  static constexpr int F1 = F > 16 ? F - 16 : 0;
  static constexpr int mode = F1 == 0 ? kTailNone : INSITE_MS_TAIL;
  static constexpr int NACC = F1 * (F1 + 1) / 2 + F1 * S;                     // VALU accumulators
  static constexpr int RG = (F1 + 3) / 4, CG = (F1 + S + 3) / 4;             // 4 x 4 block grid
  static constexpr int NT4 = RG * CG - RG * (RG - 1) / 2;                     // blocks with cg >= rg
  static constexpr int NA = mode == kTailValu ? NACC : (mode == kTailMfma4 ? NT4 : 1);
  static_assert(mode != kTailMfma4 || 16 + 4 * CG <= kMsMaxF, "tail column groups must stay in the staged row");
};

// Stage this lane's library row into LDS and run the 16 x 2 (+ 16) MFMAs over the wave's 64 rows.
// Row layout: [Theta_0..Theta_{F-1}, xdot_0..xdot_{S-1}, 0 ...] (32 doubles).  A[m][k] = Y_m of row
// 4g + k (m = lane & 15, k = lane >> 4); B[k][n] = Z_n of the same row; C[(lane>>4) + 4j][lane & 15].
// The Y1^T Z1 tail as MsTail::mode selects (acc: VALU or 4 x 4 x 4 MFMA accumulators).
template <int S, int F>
__device__ __forceinline__ void ms_emit(double* __restrict__ wrow, const double* __restrict__ wbase, bool valid,
                                        const double (&th)[F], const double (&xd)[S], dbl4& c00, dbl4& c01,
                                        dbl4& c11, double (&acc)[MsTail<S, F>::NA], int lane) {
  static_assert(F + S <= kMsMaxF, "Theta + xdot must fit two 16-column tiles");
  using Tail = MsTail<S, F>;
  wave_lds_sync();  // every lane finished reading the previous rows
#pragma unroll
  for (int j = 0; j < kMsMaxF; ++j) {
    double v = 0.0;
    if (j < F) v = th[j];
    else if (j < F + S) v = xd[j - F];
    wrow[j] = valid ? v : 0.0;
  }
  wave_lds_sync();
  if constexpr (Tail::mode == kTailValu) {
    double y1[Tail::F1];
#pragma unroll
    for (int i = 0; i < Tail::F1; ++i) y1[i] = valid ? th[16 + i] : 0.0;
    int q = 0;
#pragma unroll
    for (int i = 0; i < Tail::F1; ++i) {
#pragma unroll
      for (int j = i; j < Tail::F1; ++j, ++q) acc[q] = fma(y1[i], th[16 + j], acc[q]);
#pragma unroll
      for (int s = 0; s < S; ++s, ++q) acc[q] = fma(y1[i], xd[s], acc[q]);
    }
  }
  const int m = lane & 15, k = lane >> 4;
  const bool y1ok = 16 + m < F;
#pragma unroll
  for (int g = 0; g < 16; ++g) {
    const double* src = wbase + (4 * g + k) * kMsRowStride;
    const double y0 = src[m];
    const double z1 = src[16 + m];
    c00 = __builtin_amdgcn_mfma_f64_16x16x4f64(y0, y0, c00, 0, 0, 0);
    c01 = __builtin_amdgcn_mfma_f64_16x16x4f64(y0, z1, c01, 0, 0, 0);
    if constexpr (Tail::mode == kTailMfma16) {
      const double y1 = y1ok ? z1 : 0.0;
      c11 = __builtin_amdgcn_mfma_f64_16x16x4f64(y1, z1, c11, 0, 0, 0);
    }
  }
  if constexpr (Tail::mode == kTailMfma4) {
    // lane = 16k + 4b + i: in pass r, block b reduces rows 16r + 4b + k; operand i of column group q is
    // Z1 column 4q + i (= Y1 row 4q + i for q < RG): one LDS read per group serves A and B
    const int kk = lane >> 4, bb = (lane >> 2) & 3, ii = lane & 3;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const double* src = wbase + (16 * r + 4 * bb + kk) * kMsRowStride + 16 + ii;
      double v[Tail::CG];
#pragma unroll
      for (int q = 0; q < Tail::CG; ++q) v[q] = src[4 * q];
      int t = 0;
#pragma unroll
      for (int rg = 0; rg < Tail::RG; ++rg)
#pragma unroll
        for (int cg = rg; cg < Tail::CG; ++cg, ++t) acc[t] = __builtin_amdgcn_mfma_f64_4x4x4f64(v[rg], v[cg], acc[t], 0, 0, 0);
    }
  }
}

// Smoothed values and derivatives of one short trajectory (5 <= LL <= 7 rows), every position
// resolved at compile time (scipy savgol mode='interp' edges, pysindy one-sided FD4 edges).
template <int LL>
__device__ __forceinline__ void ms_small(const double (&xv)[8], const GramW& w, double (&xs)[8], double (&xd)[8]) {
#pragma unroll
  for (int k = 0; k < LL; ++k) {
    if (k == 0) xs[k] = sg_pos0(xv[0], xv[1], xv[2], xv[3], xv[4]);
    else if (k == 1) xs[k] = sg_pos1(xv[0], xv[1], xv[2], xv[3], xv[4]);
    else if (k == LL - 2) xs[k] = sg_pos3(xv[LL - 5], xv[LL - 4], xv[LL - 3], xv[LL - 2], xv[LL - 1]);
    else if (k == LL - 1) xs[k] = sg_pos4(xv[LL - 5], xv[LL - 4], xv[LL - 3], xv[LL - 2], xv[LL - 1]);
    else xs[k] = sg_int(w, xv[k - 2], xv[k - 1], xv[k], xv[k + 1], xv[k + 2]);
  }
#pragma unroll
  for (int k = 0; k < LL; ++k) {
    if (k == 0) xd[k] = fd_pos0(xs[0], xs[1], xs[2], xs[3], xs[4]) * w.inv_dt;
    else if (k == 1) xd[k] = fd_pos1(xs[0], xs[1], xs[2], xs[3], xs[4]) * w.inv_dt;
    else if (k == LL - 2) xd[k] = fd_pos3(xs[LL - 5], xs[LL - 4], xs[LL - 3], xs[LL - 2], xs[LL - 1]) * w.inv_dt;
    else if (k == LL - 1) xd[k] = fd_pos4(xs[LL - 5], xs[LL - 4], xs[LL - 3], xs[LL - 2], xs[LL - 1]) * w.inv_dt;
    else xd[k] = fd_int(w, xs[k - 2], xs[k - 1], xs[k + 1], xs[k + 2]);
  }
  for (int k = LL; k < 8; ++k) xs[k] = xd[k] = 0.0;
}

// Lane = patient, work item = 64-patient tile (grid-stride).  Time-major SoA fp32 states
// x[(k * S + s) * ldx + p]; treatment bits abits[k * lda + p / 32] (TIME_MAJOR_BITS; NULL = no input
// column); rows[p] observation rows (>= 5 to contribute; NULL = n_steps).
//   interior rows r = 4 .. L-5: streamed, raw ring xr[8][S] (fp32, loads 4 steps ahead into the slot
//     just consumed), smoothed ring sr[8][S] (fp64); row r leaves at step t = r + 4
//   edge rows 0..3 and L-4..L-1 (all rows when L < 8): one-sided stencils from end windows
template <int S, int NIN, bool INTER>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(INSITE_MS_WPE)))
gram_ms_kernel(const float* __restrict__ x, int64_t ldx, int n_steps, const uint32_t* __restrict__ abits,
               int64_t lda, const int32_t* __restrict__ rows, int64_t N, GramW w, double* __restrict__ partial) {
  constexpr int NZ = S + NIN;
  constexpr int F = PolyCols<NZ, INTER>::F;
  __shared__ double stage[kWavesPerBlock * kWave * kMsRowStride];
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  double* wbase = stage + wid * kWave * kMsRowStride;
  double* wrow = wbase + lane * kMsRowStride;
  dbl4 c00 = {0.0, 0.0, 0.0, 0.0}, c01 = c00, c11 = c00;
  using Tail = MsTail<S, F>;
  double acc[Tail::NA];
#pragma unroll
  for (int q = 0; q < Tail::NA; ++q) acc[q] = 0.0;
  const int64_t n_tiles = (N + kWave - 1) / kWave;
  const int64_t sstride = ldx;              // between states of one step
  const int64_t kstride = (int64_t)S * ldx; // between steps

  for (int64_t tile = (int64_t)blockIdx.x * kWavesPerBlock + wid; tile < n_tiles;
       tile += (int64_t)gridDim.x * kWavesPerBlock) {
    const int64_t p0 = tile * kWave;
    const int64_t p = p0 + lane;
    const bool in = p < N;
    const int64_t pc = in ? p : N - 1;
    int L = rows ? rows[pc] : n_steps;
    if (L > n_steps) L = n_steps;
    if (!in || L < 5) L = 0;
    const int Lmax = wave_max_i(L);
    const float* xp = x + pc;
    auto ld = [&](int k, int s) -> double { return (double)xp[(int64_t)k * kstride + s * sstride]; };

    // ---------------- interior rows (L >= 9): r = 4 .. L-5 at steps t = 8 .. L-1 ----------------
    if (Lmax >= 9) {
      float xr[8][S];
      double sr[8][S];
      // treatment word of rows [32 g, 32 g + 32): one load per lane, transposed across the half-wave
      auto word = [&](int g) -> unsigned {
        if (!abits) return 0u;
        const int k = 32 * g + (lane & 31);
        const int kk = k < n_steps ? k : n_steps - 1;
        const int64_t col = (p0 >> 5) + (lane >> 5);
        const uint32_t v = col * 32 < N ? abits[(int64_t)kk * lda + col] : 0u;  // words past N: not read
        return bit_transpose32(v, lane);
      };
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int s = 0; s < S; ++s) xr[t][s] = xp[(int64_t)t * kstride + s * sstride];
      unsigned wcur = word(0);
      // steps are processed in blocks of 8 (compile-time ring slots); loads run 4 steps ahead
      for (int t0 = 0; t0 < Lmax; t0 += 8) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int t = t0 + i;
          if (t < Lmax) {  // uniform
            if (t >= 4) {
#pragma unroll
              for (int s = 0; s < S; ++s)
                sr[(i + 6) & 7][s] = sg_int(w, xr[(i + 4) & 7][s], xr[(i + 5) & 7][s], xr[(i + 6) & 7][s],
                                            xr[(i + 7) & 7][s], xr[i & 7][s]);  // xs[t - 2]
            }
            if (t >= 8) {  // row r = t - 4
              const int r = t - 4;
              if ((r & 31) == 0) wcur = word(r >> 5);
              double z[NZ + 1], xd[S];
              z[0] = 1.0;
#pragma unroll
              for (int s = 0; s < S; ++s) {
                z[1 + s] = (double)xr[(i + 4) & 7][s];  // raw x[r]: the library sees the raw states
                xd[s] = fd_int(w, sr[(i + 2) & 7][s], sr[(i + 3) & 7][s], sr[(i + 5) & 7][s], sr[(i + 6) & 7][s]);
              }
#pragma unroll
              for (int q = 0; q < NIN; ++q) z[1 + S + q] = (double)((wcur >> (r & 31)) & 1u);
              double th[F];
              poly_row<NZ, INTER>(z, th);
              ms_emit<S, F>(wrow, wbase, t <= L - 1, th, xd, c00, c01, c11, acc, lane);
            }
            // x[t + 4] is loaded straight into the slot x[t - 4] occupied (read above): the wait
            // for it falls 4 steps later, at its first use
            const int tn = t + 4 < n_steps ? t + 4 : n_steps - 1;
#pragma unroll
            for (int s = 0; s < S; ++s) xr[(i + 4) & 7][s] = xp[(int64_t)tn * kstride + s * sstride];
          }
        }
      }
    }

    // ---------------- edge rows: 0..3 and L-4..L-1 (all rows when 5 <= L < 8) ----------------
    if (Lmax >= 5) {
      // head window x[0..7] (clamped to the stored steps; values past L are never used)
#pragma unroll
      for (int part = 0; part < 2; ++part) {
        double xs[4][S], xdd[4][S];  // the 4 rows this part emits: raw states, derivatives
        int base = 0;  // first step of the window
        if (part == 1) base = L >= 8 ? L - 8 : 0;
#pragma unroll
        for (int s = 0; s < S; ++s) {
          double xv[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int k = base + j < n_steps ? base + j : n_steps - 1;
            xv[j] = ld(k, s);
          }
          double a8[8], d8[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) a8[j] = d8[j] = 0.0;
          if (L >= 8) {
            if (part == 0) {
              a8[0] = sg_pos0(xv[0], xv[1], xv[2], xv[3], xv[4]);
              a8[1] = sg_pos1(xv[0], xv[1], xv[2], xv[3], xv[4]);
#pragma unroll
              for (int k = 2; k < 6; ++k) a8[k] = sg_int(w, xv[k - 2], xv[k - 1], xv[k], xv[k + 1], xv[k + 2]);
              a8[6] = a8[7] = 0.0;
              d8[0] = fd_pos0(a8[0], a8[1], a8[2], a8[3], a8[4]) * w.inv_dt;
              d8[1] = fd_pos1(a8[0], a8[1], a8[2], a8[3], a8[4]) * w.inv_dt;
              d8[2] = fd_int(w, a8[0], a8[1], a8[3], a8[4]);
              d8[3] = fd_int(w, a8[1], a8[2], a8[4], a8[5]);
            } else {  // window index j <-> step L - 8 + j; rows L-4..L-1 = j 4..7
#pragma unroll
              for (int k = 2; k < 6; ++k) a8[k] = sg_int(w, xv[k - 2], xv[k - 1], xv[k], xv[k + 1], xv[k + 2]);
              a8[6] = sg_pos3(xv[3], xv[4], xv[5], xv[6], xv[7]);
              a8[7] = sg_pos4(xv[3], xv[4], xv[5], xv[6], xv[7]);
              a8[0] = a8[1] = 0.0;
              d8[4] = fd_int(w, a8[2], a8[3], a8[5], a8[6]);
              d8[5] = fd_int(w, a8[3], a8[4], a8[6], a8[7]);
              d8[6] = fd_pos3(a8[3], a8[4], a8[5], a8[6], a8[7]) * w.inv_dt;
              d8[7] = fd_pos4(a8[3], a8[4], a8[5], a8[6], a8[7]) * w.inv_dt;
            }
          } else if (L == 7) {
            ms_small<7>(xv, w, a8, d8);
          } else if (L == 6) {
            ms_small<6>(xv, w, a8, d8);
          } else {
            ms_small<5>(xv, w, a8, d8);
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            xs[q][s] = xv[4 * part + q];  // raw sample of the row (smoothing feeds x_dot only)
            xdd[q][s] = d8[4 * part + q];
          }
        }
        // slots: part 0 -> window rows 0..3; part 1 -> window rows 4..7 (L >= 8) or rows 4..L-1
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int j = 4 * part + q;  // window row
          const bool valid = (L >= 8) || (j < L);
          const int step = base + j;
          double z[NZ + 1], xd[S];
          z[0] = 1.0;
#pragma unroll
          for (int s = 0; s < S; ++s) {
            z[1 + s] = xs[q][s];
            xd[s] = xdd[q][s];
          }
#pragma unroll
          for (int qq = 0; qq < NIN; ++qq) z[1 + S + qq] = (L > 0 && step < n_steps) ? input_bit(abits, lda, step, pc) : 0.0;
          double th[F];
          poly_row<NZ, INTER>(z, th);
          ms_emit<S, F>(wrow, wbase, L > 0 && valid, th, xd, c00, c01, c11, acc, lane);
        }
      }
    }
  }

  // ---- block reduction (fixed order) -> partial[block][tile][256], canonical [row][col] ----
  __syncthreads();
  double* red = stage;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int e = ((lane >> 4) + 4 * j) * 16 + (lane & 15);
    red[(wid * kMsTiles + 0) * 256 + e] = c00[j];
    red[(wid * kMsTiles + 1) * 256 + e] = c01[j];
    red[(wid * kMsTiles + 2) * 256 + e] = c11[j];
  }
  if constexpr (Tail::mode == kTailValu) {
    // wave sums of the VALU tail into tile 2 ([row - 16][col - 16], both triangles), fixed order
    wave_lds_sync();  // after this wave's (zero) c11 writes
    double* t2 = red + (wid * kMsTiles + 2) * 256;
    int q = 0;
#pragma unroll
    for (int i = 0; i < Tail::F1; ++i) {
#pragma unroll
      for (int j = i; j < Tail::F1 + S; ++j, ++q) {
        double v = acc[q];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
        if (lane == 0) {
          const int c = j < Tail::F1 ? j : F - 16 + (j - Tail::F1);
          t2[i * 16 + c] = v;
          if (j < Tail::F1) t2[j * 16 + i] = v;
        }
      }
    }
  }
  if constexpr (Tail::mode == kTailMfma4) {
    // block sums (lanes 16m + 4b + n over b) into tile 2: entry (4 rg + m, 4 cg + n) is Y1 row 4 rg + m
    // against Z1 column 4 cg + n, i.e. tile 2 [4 rg + m][4 cg + n] (Z1 column j is tile column j since
    // xdot_s sits at Z column F + s = 16 + F1 + s); the skipped cg < rg blocks by symmetry
    wave_lds_sync();  // after this wave's (zero) c11 writes
    double* t2 = red + (wid * kMsTiles + 2) * 256;
    const int m = lane >> 4, n = lane & 3;
    int t = 0;
#pragma unroll
    for (int rg = 0; rg < Tail::RG; ++rg)
#pragma unroll
      for (int cg = rg; cg < Tail::CG; ++cg, ++t) {
        double v = acc[t];
        v += __shfl_xor(v, 4, kWave);
        v += __shfl_xor(v, 8, kWave);
        const int row = 4 * rg + m, col = 4 * cg + n;
        if (((lane >> 2) & 3) == 0 && row < Tail::F1 && col < Tail::F1 + S) {
          t2[row * 16 + col] = v;
          if (cg != rg && col < Tail::F1) t2[col * 16 + row] = v;
        }
      }
  }
  __syncthreads();
  for (int q = threadIdx.x; q < kMsTiles * 256; q += kBlock) {
    double s = red[q];
#pragma unroll
    for (int ww = 1; ww < kWavesPerBlock; ++ww) s += red[ww * kMsTiles * 256 + q];
    partial[(int64_t)blockIdx.x * kMsTiles * 256 + q] = s;
  }
}

// ---------------------------------------------------------------------------------------------
// gram_ms4_kernel: the same contraction cut entirely into 4 x 4 blocks (the default form)
// ---------------------------------------------------------------------------------------------
// Y^T Z with Y = Theta (F columns) and Z = [Theta | xdot] (F + S columns) is needed on the upper
// triangle of the Theta block and on every xdot column only.  As 16 x 16 x 4 tiles (gram_ms_kernel) the
// F = 22 system issues 592 FMA per row for 363 needed: the Y0^T Z0 tile computes its lower triangle,
// and the Y0^T Z1 tile and the tail carry padding rows / columns.  Cut into 4 x 4 blocks (row group
// rg < RG over Y, column group cg >= rg over Z) the same system is 27 blocks = 432 FMA per row, and on
// gfx950 v_mfma_f64_4x4x4f64 retires FMAs at the rate of the 16 x 16 x 4 form (tools/probe/
// mfma_f64_rate_probe.hip: 17 vs 64 cycles for 1/4 of the work), so the MFMA time drops by the FMA ratio.
// Operands: lane 16 k + 4 b + i of pass r holds row 16 r + 4 b + k, columns 4 q + i of the staged LDS
// row (one ds_read_b64 per column group serves A and B); block b of every MFMA takes different rows, so
// D[b][m][n] accumulates one quarter of the rows and the epilogue sums the four (lanes xor 4, 8).
// Interior derivatives: savgol(5, 3) then the 5-point FD is one 9-tap antisymmetric filter on the raw
// samples, xdot[r] = sum_n c_n (x[r+n] - x[r-n]) / dt, c = (37/105, 79/420, -3/35, 1/140) (the exact
// convolution of the two interior stencils), so the streamed interior needs only the raw fp32 ring
// (12 slots: x[t-8 .. t] live, x[t+3] prefetched) -- no smoothed fp64 ring, ~40 VGPRs fewer than the 16 x 16
// form, which spilled at occupancy 2.  Edge rows keep the one-sided stencils (window form, as before).
template <int S, int F>
struct Ms4 {
  static constexpr int RG = (F + 3) / 4;          // Y (Theta) column groups
  static constexpr int CG = (F + S + 3) / 4;      // Z ([Theta | xdot]) column groups
  static constexpr int NB = RG * CG - RG * (RG - 1) / 2;  // blocks with cg >= rg
  static_assert(4 * CG <= kMsMaxF, "staged row");
};
#ifndef INSITE_MS4_SCHED
#define INSITE_MS4_SCHED 1
#endif
constexpr int kMs4Stride = 29;   // LDS row stride (doubles): odd, stores conflict-free, 2-way on the reads
#ifndef INSITE_MS4_ABL_NOMFMA
#define INSITE_MS4_ABL_NOMFMA 0
#endif
#ifndef INSITE_MS4_ABL_NOEMIT
#define INSITE_MS4_ABL_NOEMIT 0
#endif
#ifndef INSITE_MS4Z_SYNC
#define INSITE_MS4Z_SYNC 1
#endif
#ifndef INSITE_MS4Z_MASKSEL
#define INSITE_MS4Z_MASKSEL 0
#endif
#ifndef INSITE_MS4_PRIO
#define INSITE_MS4_PRIO 0
#endif
#ifndef INSITE_MS4_RING
#define INSITE_MS4_RING 12
#endif
constexpr int kMs4Ring = INSITE_MS4_RING;
// INSITE_MS4_BUFLD (default 1): interior samples through a per-step buffer descriptor (SGPR address math) instead
// of per-lane 64-bit addresses -- with those the 256-VGPR kernel spilled its step index and reloaded it from
// scratch before every prefetch, and each reload's s_waitcnt vmcnt(0) drained the whole prefetch ring
#ifndef INSITE_MS4_BUFLD
#define INSITE_MS4_BUFLD 1
#endif  // raw-sample ring slots (interior): x[t-8 .. t] + kMs4Ring - 9 prefetched
constexpr double kMsC1 = 37.0 / 105.0, kMsC2 = 79.0 / 420.0, kMsC3 = -3.0 / 35.0, kMsC4 = 1.0 / 140.0;

// The library row is formed column by column straight into LDS (Theta_j = z_i z_k, pysindy order), so the
// F products are never live at once.
template <int S, int NZ, bool INTER>
__device__ __forceinline__ void ms_emit4(double* __restrict__ wrow, const double* __restrict__ wbase, bool valid,
                                         const double (&z)[NZ + 1], const double (&xd)[S],
                                         double (&acc)[Ms4<S, PolyCols<NZ, INTER>::F>::NB], int lane) {
  constexpr int F = PolyCols<NZ, INTER>::F;
  constexpr PolyCols<NZ, INTER> pc;
  using M4 = Ms4<S, F>;
  wave_lds_sync();  // every lane finished reading the previous rows
#pragma unroll
  for (int j = 0; j < 4 * M4::CG; ++j) {
    double v = 0.0;
    if (j < F) v = pc.ck[j] == 0 ? z[pc.ci[j]] : z[pc.ci[j]] * z[pc.ck[j]];
    else if (j < F + S) v = xd[j - F];
    wrow[j] = valid ? v : 0.0;
  }
  wave_lds_sync();
  const int kk = lane >> 4, bb = (lane >> 2) & 3, ii = lane & 3;
  const double* src0 = wbase + (4 * bb + kk) * kMs4Stride + ii;
  // operands of pass r + 1 are read from LDS before pass r's MFMAs issue (two sets live): the LDS
  // latency hides behind the 27-MFMA pass instead of stalling the wave at every pass
  double v[2][M4::CG];
#pragma unroll
  for (int q = 0; q < M4::CG; ++q) v[0][q] = src0[4 * q];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
#if INSITE_MS4_SCHED
    __builtin_amdgcn_sched_barrier(0);  // at most two passes' operands live (register budget, occupancy 2)
#endif
    if (r < 3) {
#pragma unroll
      for (int q = 0; q < M4::CG; ++q) v[(r + 1) & 1][q] = src0[16 * (r + 1) * kMs4Stride + 4 * q];
    }
    int t = 0;
#pragma unroll
    for (int rg = 0; rg < M4::RG; ++rg)
#pragma unroll
      for (int cg = rg; cg < M4::CG; ++cg, ++t)
#if INSITE_MS4_ABL_NOMFMA  // profiling-only ablation (timing without the matrix work; results wrong)
        if (rg == 0) acc[t] += v[r & 1][cg];
#else
        acc[t] = __builtin_amdgcn_mfma_f64_4x4x4f64(v[r & 1][rg], v[r & 1][cg], acc[t], 0, 0, 0);
#endif
  }
}

// ---- staged-factor form (default): the library products are formed by the READING lanes ----
// The full-row form above writes F + S doubles per row to LDS and every one is read back once: LDS stores
// are the expensive direction (ds_write_b64 ~85 B/clk/CU against ~256 B/clk for ds_read_b64), and the
// stores plus the 27 per-row column selects were a third of the kernel (tools/g_c3var.sh ablations).
// Here each lane stages only the NPURE = NZ + 1 + S "pure" values of its row,
//   [z_0 = valid, z_1 .. z_NZ, xdot_0 .. xdot_{S-1}]            (12 doubles for C3 instead of 27),
// and the MFMA operand of a lane (row R, column slot i of column group g) is read back as
//   pure group:    P[R][4 p + i]                  (consecutive positions: one read)
//   product group: P[R][posA(g, i)] * P[R][posB(g, i)]   (two reads + one multiply, pysindy product order)
// Column groups: the pure groups that hold a library column (z_0 .. z_NZ reach into them), then the
// product groups, then the xdot-only pure groups (Z side only).  Blocks (rg, cg >= rg) over that order
// cover every needed pair once (a xdot slot that falls in a Y-side group is read as a row, the pair
// written to B through the map below).  Products are exact in f64 (f32 factors); pad slots duplicate a
// real slot and are dropped by the map.
// LDS banking (stride 13, odd): in pass r the 32 lanes of a half-wave read rows {32 h + 4 m + r : m < 8},
// whose bank offsets 13 (4 m) mod 32 are distinct multiples of 4, so a read is conflict-free whenever the
// distinct positions one instruction touches differ mod 4 (true for the C3 layout; same-position lanes
// of a quad broadcast).  Stores: 16 consecutive lanes x stride 13 cover all 16 bank pairs.
template <int S, int NZ, bool INTER>
struct Ms4Z {
  static constexpr int F = PolyCols<NZ, INTER>::F;
  static constexpr int NPURE = NZ + 1 + S;
  static constexpr int NPROD = F - (NZ + 1);
  static constexpr int PG = (NPURE + 3) / 4;    // pure groups
  static constexpr int PY = NZ / 4 + 1;         // pure groups holding a library column
  static constexpr int QG = (NPROD + 3) / 4;    // product groups
  static constexpr int RG = PY + QG;            // Y side
  static constexpr int CG = PG + QG;            // Z side
  static constexpr int NB = RG * CG - RG * (RG - 1) / 2;
  static constexpr int STRIDE = (4 * PG) | 1;   // odd, >= every pure position
  static constexpr bool kCover = false;
  static_assert(4 * CG <= kMsMaxF, "column map");
  int pos_a[CG][4], pos_b[CG][4];  // staged positions of the factors (pure groups: pos_b unused)
  int col[4 * CG];                 // logical column of slot 4 g + i: 0..F-1 library, F..F+S-1 xdot, -1 pad
  bool prod[CG];
  __host__ __device__ constexpr Ms4Z() : pos_a(), pos_b(), col(), prod() {
    constexpr PolyCols<NZ, INTER> pc{};
    // pure position -> logical column: z_0 .. z_NZ are library columns 0 .. NZ, xdot_s is F + s
    auto pure_col = [](int p) { return p <= NZ ? p : (p < NPURE ? F + (p - NZ - 1) : -1); };
    for (int g = 0; g < CG; ++g) {
      const bool is_prod = g >= PY && g < PY + QG;
      prod[g] = is_prod;
      const int pgi = g < PY ? g : g - QG;  // pure group index
      for (int i = 0; i < 4; ++i) {
        if (is_prod) {
          const int qi = 4 * (g - PY) + i;
          const int j = qi < NPROD ? NZ + 1 + qi : NZ + 1 + 4 * (g - PY);  // pad: the group's first product
          pos_a[g][i] = pc.ci[j];
          pos_b[g][i] = pc.ck[j];
          col[4 * g + i] = qi < NPROD ? j : -1;
        } else {
          const int p = 4 * pgi + i;
          pos_a[g][i] = p;
          pos_b[g][i] = p;
          col[4 * g + i] = pure_col(p);
        }
      }
    }
  }
};

// Per-lane LDS read pointers of the staged-factor form (row R0(lane) of pass 0; pass r adds r rows).
// INSITE_MS4Z_PACK (default): the product groups' factor positions (< 256) packed 4 to a register and unpacked
// at each read (one bit-field extract), where 2 QG + 1 separate pointers pushed the 256-VGPR kernel into
// scratch reloads inside the MFMA passes (C3: 6 reloads per pass; -Rpass-analysis 84 B/lane).
#ifndef INSITE_MS4Z_PACK
#define INSITE_MS4Z_PACK 1
#endif
template <int QG>
struct Ms4ZPtr {
  const double* pure;    // &P[R0][i]
#if INSITE_MS4Z_PACK
  const double* row;                            // &P[R0][0]
  unsigned pa[(QG + 3) / 4], pb[(QG + 3) / 4];  // pos_a / pos_b of product group g in byte g % 4 of word g / 4
  __device__ const double* at_a(int g) const { return row + ((pa[g >> 2] >> (8 * (g & 3))) & 0xffu); }
  __device__ const double* at_b(int g) const { return row + ((pb[g >> 2] >> (8 * (g & 3))) & 0xffu); }
#else
  const double* qa[QG];  // &P[R0][pos_a(g, i)]
  const double* qb[QG];
  __device__ const double* at_a(int g) const { return qa[g]; }
  __device__ const double* at_b(int g) const { return qb[g]; }
#endif
};

template <int S, int NZ, bool INTER>
__device__ __forceinline__ Ms4ZPtr<Ms4Z<S, NZ, INTER>::QG> ms4z_ptrs(const double* wbase, int lane) {
  using LZ = Ms4Z<S, NZ, INTER>;
  constexpr LZ lz{};
  const int k = lane >> 4, b = (lane >> 2) & 3, i = lane & 3;
  const int r0 = 32 * (k >> 1) + 4 * (4 * (k & 1) + b);
  const double* row = wbase + r0 * LZ::STRIDE;
  Ms4ZPtr<LZ::QG> p;
  p.pure = row + i;
#if INSITE_MS4Z_PACK
  p.row = row;
#pragma unroll
  for (int q = 0; q < (LZ::QG + 3) / 4; ++q) p.pa[q] = p.pb[q] = 0u;
#endif
#pragma unroll
  for (int g = 0; g < LZ::QG; ++g) {
    int a = lz.pos_a[LZ::PY + g][0], bb = lz.pos_b[LZ::PY + g][0];
#pragma unroll
    for (int ii = 1; ii < 4; ++ii) {
      if (i == ii) {
        a = lz.pos_a[LZ::PY + g][ii];
        bb = lz.pos_b[LZ::PY + g][ii];
      }
    }
#if INSITE_MS4Z_PACK
    static_assert(4 * LZ::PG < 256, "factor positions fit a byte");
    p.pa[g >> 2] |= (unsigned)a << (8 * (g & 3));
    p.pb[g >> 2] |= (unsigned)bb << (8 * (g & 3));
#else
    p.qa[g] = row + a;
    p.qb[g] = row + bb;
#endif
  }
  return p;
}

// compiler-only ordering of LDS accesses (the hardware keeps one wave's DS instructions in order)
__device__ __forceinline__ void ms4z_order() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}
#ifndef INSITE_MS4_SKEW
#define INSITE_MS4_SKEW 0
#endif
#ifndef INSITE_MS4_SKEW_EARLY
#define INSITE_MS4_SKEW_EARLY 0
#endif

__device__ __forceinline__ void ms4z_sync() {
#if INSITE_MS4Z_SYNC
  wave_lds_sync();
#else
  // LDS executes one wave's DS instructions in issue order; only the compiler has to keep the order
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
#endif
}

// Stage one row's pure values: masked (invalid rows staged as zeros) ...
template <int S, int NZ, bool INTER>
__device__ __forceinline__ void ms4z_stage_masked(double* __restrict__ wrow, bool valid, const double (&z)[NZ + 1],
                                                  const double (&xd)[S]) {
  using LZ = Ms4Z<S, NZ, INTER>;
  wrow[0] = valid ? 1.0 : 0.0;
#pragma unroll
  for (int s = 1; s <= NZ; ++s) wrow[s] = valid ? z[s] : 0.0;
#pragma unroll
  for (int s = 0; s < S; ++s) wrow[NZ + 1 + s] = valid ? xd[s] : 0.0;
#pragma unroll
  for (int p = LZ::NPURE; p < 4 * LZ::PG; ++p) wrow[p] = 0.0;
}
// ... or as they are (the caller routes invalid rows elsewhere)
template <int S, int NZ, bool INTER>
__device__ __forceinline__ void ms4z_stage(double* __restrict__ wp, const double (&z)[NZ + 1], const double (&xd)[S]) {
  using LZ = Ms4Z<S, NZ, INTER>;
  wp[0] = 1.0;
#pragma unroll
  for (int s = 1; s <= NZ; ++s) wp[s] = z[s];
#pragma unroll
  for (int s = 0; s < S; ++s) wp[NZ + 1 + s] = xd[s];
#pragma unroll
  for (int p = LZ::NPURE; p < 4 * LZ::PG; ++p) wp[p] = 0.0;
}
template <int S, int NZ, bool INTER>
__device__ __forceinline__ void ms4z_zero(double* __restrict__ wrow) {
#pragma unroll
  for (int p = 0; p < 4 * Ms4Z<S, NZ, INTER>::PG; ++p) wrow[p] = 0.0;
}

// The 4 passes over the 64 staged rows: read / form the operands, 4 x 4 x 4 f64 blocks.
template <int S, int NZ, bool INTER>
__device__ __forceinline__ void ms4z_passes(const Ms4ZPtr<Ms4Z<S, NZ, INTER>::QG>& pp,
                                            double (&acc)[Ms4Z<S, NZ, INTER>::NB]) {
  using LZ = Ms4Z<S, NZ, INTER>;
  // operands of pass r + 1 are read before pass r's MFMAs issue (two sets live)
  double ra[2][LZ::CG], rb[2][LZ::QG];
  auto fetch = [&](int r, int slot) {
#pragma unroll
    for (int g = 0; g < LZ::CG; ++g) {
      if (g >= LZ::PY && g < LZ::PY + LZ::QG) {
        ra[slot][g] = pp.at_a(g - LZ::PY)[r * LZ::STRIDE];
        rb[slot][g - LZ::PY] = pp.at_b(g - LZ::PY)[r * LZ::STRIDE];
      } else {
        const int pgi = g < LZ::PY ? g : g - LZ::QG;
        ra[slot][g] = pp.pure[4 * pgi + r * LZ::STRIDE];
      }
    }
  };
  fetch(0, 0);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
#if INSITE_MS4_SCHED
    __builtin_amdgcn_sched_barrier(0);
#endif
    if (r < 3) fetch(r + 1, (r + 1) & 1);
    double v[LZ::CG];
#pragma unroll
    for (int g = 0; g < LZ::CG; ++g)
      v[g] = (g >= LZ::PY && g < LZ::PY + LZ::QG) ? ra[r & 1][g] * rb[r & 1][g - LZ::PY] : ra[r & 1][g];
    int t = 0;
#pragma unroll
    for (int rg = 0; rg < LZ::RG; ++rg)
#pragma unroll
      for (int cg = rg; cg < LZ::CG; ++cg, ++t)
#if INSITE_MS4_ABL_NOMFMA
        if (rg == 0) acc[t] += v[cg];
#else
        acc[t] = __builtin_amdgcn_mfma_f64_4x4x4f64(v[rg], v[cg], acc[t], 0, 0, 0);
#endif
  }
}

// ---- moment cover (C3, default): fewer blocks over the distinct moments ----
// The Theta | xdot column groups above issue 27 blocks (432 cells per row) for 363 entries, but those entries
// hold only 257 distinct moments: G entries are monomials z^g of degree <= 4 in z = (x_1..x_5, a), and a is
// 0/1 (a^2 = a), so the 253 G entries are 147 moments; B adds 110.  tools/ms4_cover.py searches operand groups
// -- each slot a product of <= 2 staged pure values (one LDS read, or two reads + one multiply; the same
// staging as Ms4Z) -- whose pairwise 4 x 4 blocks cover all 257, and emits the groups, the block list and the
// entry -> (block, m, n) map of ms4_finalize_cover (ms4_cover_c3.inc).  The products are exact in f64 wherever
// the old form's were (x and a are fp32 values: products of two are exact); only operands xdot * x would round
// once more, and the emitted cover has none.
#include "ms4_cover_c3.inc"
template <int S, int NZ, bool INTER>
struct Ms4Cover {
  using LZ = Ms4Z<S, NZ, INTER>;
  static_assert(S == 5 && NZ == 6 && INTER, "the emitted cover is the C3 library's");
  static constexpr int F = LZ::F, STRIDE = LZ::STRIDE, NG = kMs4CoverNG, NB = kMs4CoverNB;
  static constexpr bool kCover = true;
  static constexpr bool prod(int g) { return kMs4CoverProd[g] != 0; }
  static_assert(LZ::NPURE == 4 * LZ::PG, "every staged position holds a pure value (no pads)");
  static_assert(4 * LZ::PG < 256, "factor positions fit a byte");
};
struct Ms4CPtr {
  const double* row;  // &P[R0][0]
  unsigned pa[(kMs4CoverNG + 3) / 4], pb[(kMs4CoverNG + 3) / 4];
  __device__ const double* at_a(int g) const { return row + ((pa[g >> 2] >> (8 * (g & 3))) & 0xffu); }
  __device__ const double* at_b(int g) const { return row + ((pb[g >> 2] >> (8 * (g & 3))) & 0xffu); }
};
template <int S, int NZ, bool INTER>
__device__ __forceinline__ Ms4CPtr ms4c_ptrs(const double* wbase, int lane) {
  using LC = Ms4Cover<S, NZ, INTER>;
  const int k = lane >> 4, b = (lane >> 2) & 3, i = lane & 3;
  const int r0 = 32 * (k >> 1) + 4 * (4 * (k & 1) + b);  // the rows of Ms4Z's conflict-free read pattern
  Ms4CPtr p;
  p.row = wbase + r0 * LC::STRIDE;
#pragma unroll
  for (int q = 0; q < (LC::NG + 3) / 4; ++q) p.pa[q] = p.pb[q] = 0u;
#pragma unroll
  for (int g = 0; g < LC::NG; ++g) {
    unsigned a = kMs4CoverPA[g][0], bb = kMs4CoverPB[g][0];
#pragma unroll
    for (int ii = 1; ii < 4; ++ii) {
      if (i == ii) {
        a = kMs4CoverPA[g][ii];
        bb = kMs4CoverPB[g][ii];
      }
    }
    p.pa[g >> 2] |= a << (8 * (g & 3));
    p.pb[g >> 2] |= bb << (8 * (g & 3));
  }
  return p;
}
// Operands of one pass (rows r of the staged buffer at offset boff doubles): per group the first factor, and the
// second for the product groups.
template <int S, int NZ, bool INTER>
__device__ __forceinline__ void ms4c_fetch(const Ms4CPtr& pp, int off, double (&ra)[kMs4CoverNG],
                                           double (&rb)[kMs4CoverNG]) {
#pragma unroll
  for (int g = 0; g < kMs4CoverNG; ++g) {
    ra[g] = pp.at_a(g)[off];
    if (Ms4Cover<S, NZ, INTER>::prod(g)) rb[g] = pp.at_b(g)[off];
  }
}
// The 4 passes over the buffer at boff; PRE: pass 0's operands were fetched by the caller (ra0 / rb0), so their
// LDS latency hid behind the caller's own work.
template <int S, int NZ, bool INTER, bool PRE>
__device__ __forceinline__ void ms4c_passes(const Ms4CPtr& pp, int boff, const double (&ra0)[kMs4CoverNG],
                                            const double (&rb0)[kMs4CoverNG], double (&acc)[kMs4CoverNB]) {
  using LC = Ms4Cover<S, NZ, INTER>;
  double ra[2][LC::NG], rb[2][LC::NG];  // rb: product groups only; operands of pass r + 1 read during pass r
  if constexpr (PRE) {
#pragma unroll
    for (int g = 0; g < LC::NG; ++g) {
      ra[0][g] = ra0[g];
      rb[0][g] = rb0[g];
    }
  } else {
    ms4c_fetch<S, NZ, INTER>(pp, boff, ra[0], rb[0]);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
#if INSITE_MS4_SCHED
    __builtin_amdgcn_sched_barrier(0);
#endif
    if (r < 3) ms4c_fetch<S, NZ, INTER>(pp, boff + (r + 1) * LC::STRIDE, ra[(r + 1) & 1], rb[(r + 1) & 1]);
    double v[LC::NG];
#pragma unroll
    for (int g = 0; g < LC::NG; ++g) v[g] = LC::prod(g) ? ra[r & 1][g] * rb[r & 1][g] : ra[r & 1][g];
#pragma unroll
    for (int t = 0; t < LC::NB; ++t)
#if INSITE_MS4_ABL_NOMFMA
      if (t == 0) acc[t] += v[kMs4CoverBU[t]] + v[kMs4CoverBV[t]];
#else
      acc[t] = __builtin_amdgcn_mfma_f64_4x4x4f64(v[kMs4CoverBU[t]], v[kMs4CoverBV[t]], acc[t], 0, 0, 0);
#endif
  }
}
template <int S, int NZ, bool INTER>
__device__ __forceinline__ void ms4c_passes(const Ms4CPtr& pp, double (&acc)[kMs4CoverNB]) {
  double unused[kMs4CoverNG];
  ms4c_passes<S, NZ, INTER, false>(pp, 0, unused, unused, acc);
}

// The cover stages the same pure values, at the positions kMs4CoverStage gives (bank-conflict-free reads).
template <int S, int NZ>
__device__ __forceinline__ void ms4c_stage(double* __restrict__ wp, double one, const double (&z)[NZ + 1],
                                           const double (&xd)[S], bool valid) {
  wp[kMs4CoverStage[0]] = one;
#pragma unroll
  for (int s = 1; s <= NZ; ++s) wp[kMs4CoverStage[s]] = valid ? z[s] : 0.0;
#pragma unroll
  for (int s = 0; s < S; ++s) wp[kMs4CoverStage[NZ + 1 + s]] = valid ? xd[s] : 0.0;
}

// layout-generic per-lane read pointers, staging and passes
template <int S, int NZ, bool INTER, class M4>
__device__ __forceinline__ void ms4_stage(double* __restrict__ wp, const double (&z)[NZ + 1], const double (&xd)[S]) {
  if constexpr (M4::kCover) ms4c_stage<S, NZ>(wp, 1.0, z, xd, true);
  else ms4z_stage<S, NZ, INTER>(wp, z, xd);
}
template <int S, int NZ, bool INTER, class M4>
__device__ __forceinline__ auto ms4_ptrs(const double* wbase, int lane) {
  if constexpr (M4::kCover) return ms4c_ptrs<S, NZ, INTER>(wbase, lane);
  else return ms4z_ptrs<S, NZ, INTER>(wbase, lane);
}
template <int S, int NZ, bool INTER, class PP, int NBX>
__device__ __forceinline__ void ms4_passes(const PP& pp, double (&acc)[NBX]) {
  if constexpr (std::is_same<PP, Ms4CPtr>::value) ms4c_passes<S, NZ, INTER>(pp, acc);
  else ms4z_passes<S, NZ, INTER>(pp, acc);
}

template <int S, int NZ, bool INTER, class PP, int NBX>
__device__ __forceinline__ void ms_emit4z(double* __restrict__ wrow, const PP& pp, bool valid,
                                          const double (&z)[NZ + 1], const double (&xd)[S], double (&acc)[NBX]) {
  ms4z_sync();
  if constexpr (std::is_same<PP, Ms4CPtr>::value) ms4c_stage<S, NZ>(wrow, valid ? 1.0 : 0.0, z, xd, valid);
  else ms4z_stage_masked<S, NZ, INTER>(wrow, valid, z, xd);
  ms4z_sync();
  ms4_passes<S, NZ, INTER>(pp, acc);
}

// The full-row form's geometry in the same vocabulary (column map = identity over [Theta | xdot]).
template <int S, int NZ, bool INTER>
struct Ms4Full {
  static constexpr int F = PolyCols<NZ, INTER>::F;
  using M4 = Ms4<S, F>;
  static constexpr int RG = M4::RG, CG = M4::CG, NB = M4::NB, STRIDE = kMs4Stride;
  static constexpr bool kCover = false;
  int col[4 * CG];
  __host__ __device__ constexpr Ms4Full() : col() {
    for (int j = 0; j < 4 * CG; ++j) col[j] = j < F + S ? j : -1;
  }
};

#ifndef INSITE_MS4_FULLROW
#define INSITE_MS4_FULLROW 0
#endif
// INSITE_MS4_COVER (default 1): the C3 library (5 states + one binary input, interaction only) takes the moment
// cover; the other libraries (and INSITE_MS4_COVER=0) the Theta | xdot column groups
#ifndef INSITE_MS4_COVER
#define INSITE_MS4_COVER 1
#endif
template <int S, int NZ, bool INTER>
using Ms4Layout = typename std::conditional<
    INSITE_MS4_FULLROW != 0, Ms4Full<S, NZ, INTER>,
    typename std::conditional<INSITE_MS4_COVER != 0 && S == 5 && NZ == 6 && INTER, Ms4Cover<S, NZ, INTER>,
                              Ms4Z<S, NZ, INTER>>::type>::type;

template <int S, int NIN, bool INTER>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(INSITE_MS_WPE)))
gram_ms4_kernel(const float* __restrict__ x, int64_t ldx, int n_steps, const uint32_t* __restrict__ abits,
                int64_t lda, const int32_t* __restrict__ rows, int64_t N, GramW w, double* __restrict__ partial,
                int nchunk) {
  constexpr int NZ = S + NIN;
  using M4 = Ms4Layout<S, NZ, INTER>;
  // INSITE_MS4_SKEW (A/B, default off): the interior stages row t into one of two buffers while the passes run
  // over row t - 1 in the other, whose pass-0 operands are read ahead of the stores -- the staging stores and the
  // first reads no longer sit between the VALU work and the MFMAs.  Measured neutral-to-slower (7.92 / 7.93 ms
  // with the reads ahead of the stores / of the derivative work, vs 7.86 ms, profiles/r05/c3/): the LDS waits
  // (SQ_WAIT_INST_LDS ~237 cycles per wave-step) were already covered by the partner wave's MFMAs.
  constexpr bool kSkew = INSITE_MS4_SKEW && M4::kCover && !INSITE_MS4_FULLROW && !INSITE_MS4Z_MASKSEL;
  static_assert(kMs4Ring % 2 == 0, "buffer parity of step t = parity of its ring slot");
  constexpr int kBuf = kWave * M4::STRIDE;  // doubles per staged 64-row buffer
  // per wave: 64 staged rows (two buffers when skewed), then (staged-factor form) 64 trash rows that invalid
  // interior rows go to
  constexpr int kWaveStage = (INSITE_MS4_FULLROW ? 1 : kSkew ? 3 : 2) * kBuf;
  static_assert(M4::NB * 16 * kWavesPerBlock <= kWavesPerBlock * kWaveStage, "block reduction fits the stage");
  __shared__ double stage[kWavesPerBlock * kWaveStage];
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
#if INSITE_MS4_PRIO
  if (blockIdx.x >= gridDim.x / 2) __builtin_amdgcn_s_setprio(1);
#endif
  double* wbase = stage + wid * kWaveStage;
  double* wrow = wbase + lane * M4::STRIDE;
#if !INSITE_MS4_FULLROW
  const auto zptr = ms4_ptrs<S, NZ, INTER, M4>(wbase, lane);
#endif
  double acc[M4::NB];
#pragma unroll
  for (int q = 0; q < M4::NB; ++q) acc[q] = 0.0;
  const int64_t n_tiles = (N + kWave - 1) / kWave;
  const int64_t sstride = ldx;              // between states of one step
  const int64_t kstride = (int64_t)S * ldx; // between steps
  const double c1 = kMsC1 * w.inv_dt, c2 = kMsC2 * w.inv_dt, c3 = kMsC3 * w.inv_dt, c4 = kMsC4 * w.inv_dt;

  // work unit = (tile, chunk): the interior steps of a tile are cut into nchunk consecutive ranges so the
  // units divide evenly over the resident waves (ms4_chunks); chunk 0 also takes the tile's edge rows
  for (int64_t unit = (int64_t)blockIdx.x * kWavesPerBlock + wid; unit < n_tiles * nchunk;
       unit += (int64_t)gridDim.x * kWavesPerBlock) {
    const int64_t tile = unit / nchunk;
    const int chunk = (int)(unit - tile * nchunk);
    const int64_t p0 = tile * kWave;
    const int64_t p = p0 + lane;
    const bool in = p < N;
    const int64_t pc = in ? p : N - 1;
    int L = rows ? rows[pc] : n_steps;
    if (L > n_steps) L = n_steps;
    if (!in || L < 5) L = 0;
    const int Lmax = wave_max_i(L);
    const int tz = L > 8 ? L : 8;  // first interior step whose row lies past the lane's end
    const float* xp = x + pc;
    auto ld = [&](int k, int s) -> double { return (double)xp[(int64_t)k * kstride + s * sstride]; };

    // ---------------- interior rows (L >= 9): r = 4 .. L-5 at steps t = 8 .. L-1 ----------------
    // this chunk emits steps [ea, eb) and loads from ea - 8 (the 9-sample window of its first row)
    const int n_emit = Lmax - 8;
    const int ea = 8 + (int)((int64_t)n_emit * chunk / nchunk);
    const int eb = 8 + (int)((int64_t)n_emit * (chunk + 1) / nchunk);
    const int ts = ea - 8;
    const int tzc = tz > ea ? tz : ea;  // a lane already past its end zeroes its (stale) row at the first emit
    if (Lmax >= 9 && eb > ea) {
      float xr[kMs4Ring][S];
#if INSITE_MS4_BUFLD
      // the S state rows of step k through one wave-uniform descriptor based at (k, state 0, column p0):
      // SGPR address math per step, lanes past N read 0 (their rows are never emitted)
      const int tval = (int)(N - p0 < kWave ? N - p0 : kWave);
      const unsigned loff = p < N ? (unsigned)lane * 4u : kOOB;
      auto ld_step = [&](float (&dst)[S], int k) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(x + (int64_t)k * kstride + p0), (short)0, (int)(((int64_t)(S - 1) * sstride + tval) * 4), 0x00020000);
#pragma unroll
        for (int s = 0; s < S; ++s)
          dst[s] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, loff, (int)(s * sstride * 4), 0));
      };
#endif
      auto word = [&](int g) -> unsigned {  // treatment bits of rows [32 g, 32 g + 32), half-wave transpose
        if (!abits) return 0u;
        const int k = 32 * g + (lane & 31);
        const int kk = k < n_steps ? k : n_steps - 1;
        const int64_t col = (p0 >> 5) + (lane >> 5);
        const uint32_t v = col * 32 < N ? abits[(int64_t)kk * lda + col] : 0u;
        return bit_transpose32(v, lane);
      };
#pragma unroll
      for (int t = 0; t < kMs4Ring - 9; ++t) {
#if INSITE_MS4_BUFLD
        ld_step(xr[t], ts + t);
#else
#pragma unroll
        for (int s = 0; s < S; ++s) xr[t][s] = xp[(int64_t)(ts + t) * kstride + s * sstride];
#endif
      }
      unsigned wcur = word((ea - 4) >> 5);
      for (int t0 = ts; t0 < eb; t0 += kMs4Ring) {
#pragma unroll
        for (int i = 0; i < kMs4Ring; ++i) {
          const int t = t0 + i;
          if (t < eb) {  // uniform
            // x[t + PF] into the slot of x[t - 9 + ...] (no longer needed): its wait falls PF steps later
            constexpr int PF = kMs4Ring - 9;
            const int tn = t + PF < n_steps ? t + PF : n_steps - 1;
#if INSITE_MS4_BUFLD
            ld_step(xr[(i + PF) % kMs4Ring], tn);
#else
#pragma unroll
            for (int s = 0; s < S; ++s) xr[(i + PF) % kMs4Ring][s] = xp[(int64_t)tn * kstride + s * sstride];
#endif
            if (t >= ea) {  // row r = t - 4: raw x[r], xdot from x[r-4 .. r+4] (slots i-8 .. i)
              const int r = t - 4;
              // skewed: step t stages into buffer (t - ts) & 1 = i & 1 and passes over the other (row t - 1)
              const int cb = (i & 1) * kBuf, pbf = kBuf - cb;  // constants once unrolled
              // skewed: pass-0 operands of row t - 1 (read unconditionally -- at t == ea the stale buffer's
              // values go unused -- so they are not live across steps)
              double pa0[kMs4CoverNG], pb0[kMs4CoverNG];
#if INSITE_MS4_SKEW_EARLY
              if constexpr (kSkew) {
                ms4c_fetch<S, NZ, INTER>(zptr, pbf, pa0, pb0);
                __builtin_amdgcn_sched_barrier(0);  // issued before the derivative work
              }
#endif
              if ((r & 31) == 0) wcur = word(r >> 5);
              double z[NZ + 1], xd[S];
              z[0] = 1.0;
#pragma unroll
              for (int s = 0; s < S; ++s) {
                auto X = [&](int d) -> double { return (double)xr[(i + kMs4Ring + d) % kMs4Ring][s]; };  // x[t + d]
                z[1 + s] = X(-4);
                xd[s] = c1 * (X(-3) - X(-5)) + c2 * (X(-2) - X(-6)) + c3 * (X(-1) - X(-7)) + c4 * (X(0) - X(-8));
              }
#pragma unroll
              for (int q = 0; q < NIN; ++q) z[1 + S + q] = (double)((wcur >> (r & 31)) & 1u);
#if INSITE_MS4_ABL_NOEMIT  // profiling-only ablation (ring + derivative only; results wrong)
              double sink = 0.0;
#pragma unroll
              for (int s = 0; s < S; ++s) sink += z[1 + s] * xd[s];
              acc[0] += (t <= L - 1) ? sink + z[NZ] : 0.0;
#else
#if INSITE_MS4_FULLROW
              ms_emit4<S, NZ, INTER>(wrow, wbase, t <= L - 1, z, xd, acc, lane);
#elif INSITE_MS4Z_MASKSEL
              ms_emit4z<S, NZ, INTER>(wrow, zptr, t <= L - 1, z, xd, acc);
#else
              // rows past a lane's end go to its trash row; its staged row is zeroed once, at the first
              // such row (t == tz), and stays zero for the rest of the interior
              if constexpr (kSkew) {
                // the LDS executes one wave's DS instructions in issue order: the stores of row t cannot pass the
                // reads of row t - 2 (same buffer, step t - 1), and row t - 1's stores are complete before this
                // step's reads of it -- only the compiler's order is pinned here.  A lane past its end zeroes its
                // row in both buffers (steps tzc, tzc + 1), its rows go to the trash row.
#if !INSITE_MS4_SKEW_EARLY
                ms4c_fetch<S, NZ, INTER>(zptr, pbf, pa0, pb0);  // ahead of the stores
#endif
                ms4z_order();
                ms4_stage<S, NZ, INTER, M4>(t <= L - 1 ? wrow + cb : wrow + 2 * kBuf, z, xd);
                if (t == tzc || t == tzc + 1) ms4z_zero<S, NZ, INTER>(wrow + cb);
                ms4z_order();
                if (t > ea) ms4c_passes<S, NZ, INTER, true>(zptr, pbf, pa0, pb0, acc);
              } else {
                ms4z_sync();
                ms4_stage<S, NZ, INTER, M4>(t <= L - 1 ? wrow : wrow + kBuf, z, xd);
                if (t == tzc) ms4z_zero<S, NZ, INTER>(wrow);
                ms4z_sync();
                ms4_passes<S, NZ, INTER>(zptr, acc);
              }
#endif
#endif
            }
          }
        }
      }
      if constexpr (kSkew) {  // the chunk's last row (step eb - 1) has not had its passes
        ms4z_order();
        double unused[kMs4CoverNG];
        ms4c_passes<S, NZ, INTER, false>(zptr, ((eb - 1 - ts) & 1) * kBuf, unused, unused, acc);
      }
    }

    // ---------------- edge rows: 0..3 and L-4..L-1 (all rows when 5 <= L < 8) ----------------
    // one row at a time (its window re-read per row from the cache: 8 of ~500 rows per patient), so the
    // edge path holds one 8-sample window instead of 4 rows x S states of values and derivatives
    if (Lmax >= 5 && chunk == 0) {
      for (int j = 0; j < 8; ++j) {  // window row: part j / 4, position j % 4 within the part
        const int base = j < 4 ? 0 : (L >= 8 ? L - 8 : 0);
        const bool valid = (L >= 8) || (j < L);
        const int step = base + j;
        double z[NZ + 1], xd[S];
        z[0] = 1.0;
#pragma unroll
        for (int s = 0; s < S; ++s) {
          double xv[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const int k = base + q < n_steps ? base + q : n_steps - 1;
            xv[q] = ld(k, s);
          }
          double a8[8], d8[8];
          if (L >= 8) {
            // rows 0..3 from the head window, L-4..L-1 (window rows 4..7) from the tail window
#pragma unroll
            for (int k = 2; k < 6; ++k) a8[k] = sg_int(w, xv[k - 2], xv[k - 1], xv[k], xv[k + 1], xv[k + 2]);
            a8[0] = sg_pos0(xv[0], xv[1], xv[2], xv[3], xv[4]);
            a8[1] = sg_pos1(xv[0], xv[1], xv[2], xv[3], xv[4]);
            a8[6] = sg_pos3(xv[3], xv[4], xv[5], xv[6], xv[7]);
            a8[7] = sg_pos4(xv[3], xv[4], xv[5], xv[6], xv[7]);
            double d;
            switch (j) {
              case 0: d = fd_pos0(a8[0], a8[1], a8[2], a8[3], a8[4]) * w.inv_dt; break;
              case 1: d = fd_pos1(a8[0], a8[1], a8[2], a8[3], a8[4]) * w.inv_dt; break;
              case 2: d = fd_int(w, a8[0], a8[1], a8[3], a8[4]); break;
              case 3: d = fd_int(w, a8[1], a8[2], a8[4], a8[5]); break;
              case 4: d = fd_int(w, a8[2], a8[3], a8[5], a8[6]); break;
              case 5: d = fd_int(w, a8[3], a8[4], a8[6], a8[7]); break;
              case 6: d = fd_pos3(a8[3], a8[4], a8[5], a8[6], a8[7]) * w.inv_dt; break;
              default: d = fd_pos4(a8[3], a8[4], a8[5], a8[6], a8[7]) * w.inv_dt; break;
            }
            xd[s] = d;
          } else {
            if (L == 7) ms_small<7>(xv, w, a8, d8);
            else if (L == 6) ms_small<6>(xv, w, a8, d8);
            else ms_small<5>(xv, w, a8, d8);
            xd[s] = d8[j];
          }
          z[1 + s] = xv[j];  // raw sample of the row (smoothing feeds x_dot only)
        }
#pragma unroll
        for (int qq = 0; qq < NIN; ++qq) z[1 + S + qq] = (L > 0 && step < n_steps) ? input_bit(abits, lda, step, pc) : 0.0;
#if INSITE_MS4_FULLROW
        ms_emit4<S, NZ, INTER>(wrow, wbase, L > 0 && valid, z, xd, acc, lane);
#else
        ms_emit4z<S, NZ, INTER>(wrow, zptr, L > 0 && valid, z, xd, acc);
#endif
      }
    }
  }

  // ---- block partial (fixed order): partial[block][t * 16 + 4 m + n] = sum over waves and the 4 row quarters
  // b of D[b][m][n] of block type t ----
  __syncthreads();
  double* red = stage;
  const int m = lane >> 4, n = lane & 3;
#pragma unroll
  for (int t = 0; t < M4::NB; ++t) {
    double v = acc[t];
    v += __shfl_xor(v, 4, kWave);
    v += __shfl_xor(v, 8, kWave);
    if (((lane >> 2) & 3) == 0) red[(wid * M4::NB + t) * 16 + 4 * m + n] = v;
  }
  __syncthreads();
  for (int q = threadIdx.x; q < M4::NB * 16; q += kBlock) {
    double sum = red[q];
#pragma unroll
    for (int ww = 1; ww < kWavesPerBlock; ++ww) sum += red[ww * M4::NB * 16 + q];
    partial[(int64_t)blockIdx.x * M4::NB * 16 + q] = sum;
  }
}

// Fixed-order reduction of gram_ms4_kernel's block partials and scatter into G [F, F] and B [F, S]:
// entry (t, m, n) of block type t = (rg, cg) pairs Y slot 4 rg + m with Z slot 4 cg + n; the slot -> column
// map (library 0..F-1, xdot F..F+S-1, -1 pad) places it.  Diagonal blocks hold each pair twice: n >= m only.
struct Ms4Map {
  int col[kMsMaxF];
};
__global__ void __launch_bounds__(kWave) ms4_finalize(const double* __restrict__ partial, int nblk, int nb, int cgn,
                                                      int F, int S, Ms4Map map, double* __restrict__ G,
                                                      double* __restrict__ B) {
  const int q = blockIdx.x * kWave + threadIdx.x;
  if (q >= nb * 16) return;
  double v = 0.0;
  for (int g = 0; g < nblk; ++g) v += partial[(int64_t)g * nb * 16 + q];
  int t = q / 16, rg = 0;
  while (t >= cgn - rg) {  // block types enumerate rg-major, cg = rg .. cgn-1
    t -= cgn - rg;
    ++rg;
  }
  const int cg = rg + t;
  const int m = (q % 16) / 4, n = q % 4;
  if (cg == rg && n < m) return;
  const int a = map.col[4 * rg + m], b = map.col[4 * cg + n];
  if (a < 0 || b < 0) return;
  if (a < F && b < F) {
    G[(int64_t)a * F + b] = v;
    G[(int64_t)b * F + a] = v;
  } else if (a < F) {
    B[(int64_t)a * S + (b - F)] = v;
  } else if (b < F) {
    B[(int64_t)b * S + (a - F)] = v;
  }
}

// The moment cover's finalize: one lane per output entry (G row-major, then B row-major) reduces the partial
// its moment lives in, in block order (symmetric G entries read the same partial: bitwise equal halves).
__global__ void __launch_bounds__(kWave) ms4_finalize_cover(const double* __restrict__ partial, int nblk, int nb,
                                                            int F, double* __restrict__ G, double* __restrict__ B) {
  const int e = blockIdx.x * kWave + threadIdx.x;
  if (e >= kMs4CoverEntries) return;
  const int q = kMs4CoverMap[e];
  double v = 0.0;
  for (int g = 0; g < nblk; ++g) v += partial[(int64_t)g * nb * 16 + q];
  if (e < F * F) G[e] = v;
  else B[e - F * F] = v;
}

// Fixed-order reduction of the tile partials and scatter into G [F, F] (symmetric) and B [F, S].
__global__ void __launch_bounds__(kWave) ms_finalize(const double* __restrict__ partial, int nblk, int F, int S,
                                                     double* __restrict__ G, double* __restrict__ B) {
  const int q = blockIdx.x * kWave + threadIdx.x;  // tile entry, < 3 * 256
  if (q >= kMsTiles * 256) return;
  double v = 0.0;
  for (int g = 0; g < nblk; ++g) v += partial[(int64_t)g * kMsTiles * 256 + q];
  const int t = q / 256, e = q % 256, r = e / 16, c = e % 16;
  const int row = t == 2 ? 16 + r : r;        // Y row
  const int col = t == 0 ? c : 16 + c;        // Z column
  if (row >= F) return;
  if (col < F) {
    G[(int64_t)row * F + col] = v;
    if (t == 1) G[(int64_t)col * F + row] = v;  // the skipped Y1^T Z0 tile, by symmetry
  } else if (col < F + S) {
    B[(int64_t)row * S + (col - F)] = v;
  }
}

// ---------------------------------------------------------------------------------------------
// Wave-cooperative STLSQ for F <= 32 (one wavefront per target state)
// ---------------------------------------------------------------------------------------------
// Masked ridge solve (G_SS + alpha I) c_S = b_S with inactive rows/columns replaced by identity rows
// (the operations of the reduced solve on the active block, as masked_cholesky_solve in
// insite_hip.hip).  Lane i owns row i of M (LDS, row-major with stride kMsMaxF + 1); right-looking
// Cholesky, then forward/backward substitution.  Returns false if not positive definite.
__device__ bool wave_chol_solve(const double* __restrict__ G, const double* __restrict__ b, int bstride, int F,
                                unsigned m, double alpha, double* M, double* v, double* c, int lane) {
  constexpr int LD = kMsMaxF + 1;
  const bool row_on = lane < F;
  const bool ai = row_on && ((m >> lane) & 1u);
  if (row_on) {
    for (int j = 0; j < F; ++j) {
      const bool act = ai && ((m >> j) & 1u);
      double a = act ? G[(int64_t)lane * F + j] : 0.0;
      if (j == lane) a = ai ? a + alpha : 1.0;
      M[lane * LD + j] = a;
    }
    v[lane] = ai ? b[(int64_t)lane * bstride] : 0.0;
  }
  wave_lds_sync();
  bool ok = true;
  for (int j = 0; j < F; ++j) {
    double d = M[j * LD + j];
    if (!(d > 0.0)) {
      ok = false;
      d = 1e-300;
    }
    const double rd = 1.0 / sqrt(d);
    wave_lds_sync();
    if (lane > j && lane < F) M[lane * LD + j] *= rd;  // L[i][j]
    if (lane == j) M[j * LD + j] = d * rd;                // L[j][j] = sqrt(d)
    wave_lds_sync();
    if (lane > j && lane < F) {
      const double lij = M[lane * LD + j];
      for (int k = j + 1; k <= lane; ++k) M[lane * LD + k] = fma(-lij, M[k * LD + j], M[lane * LD + k]);
    }
    wave_lds_sync();
  }
  // forward: L z = v
  for (int j = 0; j < F; ++j) {
    const double zj = v[j] / M[j * LD + j];
    wave_lds_sync();
    if (lane == j) v[j] = zj;
    if (lane > j && lane < F) v[lane] = fma(-M[lane * LD + j], zj, v[lane]);
    wave_lds_sync();
  }
  // backward: L^T c = z
  for (int j = F - 1; j >= 0; --j) {
    const double cj = v[j] / M[j * LD + j];
    wave_lds_sync();
    if (lane == j) c[j] = ((m >> j) & 1u) ? cj : 0.0;
    if (lane < j) v[lane] = fma(-M[j * LD + lane], cj, v[lane]);
    wave_lds_sync();
  }
  return ok;
}

__global__ void __launch_bounds__(kWave)
stlsq_wave_kernel(const double* __restrict__ G, const double* __restrict__ B, int F, int n_sys, StlsqParams sp,
                  double* __restrict__ coef, int8_t* __restrict__ mask, int32_t* __restrict__ iters) {
  __shared__ double M[kMsMaxF * (kMsMaxF + 1)];
  __shared__ double v[kMsMaxF], c[kMsMaxF];
  const int s = blockIdx.x;
  const int lane = threadIdx.x;
  if (s >= n_sys) return;
  const double* b = B + s;  // column s of B [F, n_sys]
  const unsigned all = F >= 32 ? 0xffffffffu : ((1u << F) - 1u);
  unsigned ind = all, prev = all;
  bool ok = true;
  int it = 0;
  if (lane < kMsMaxF) c[lane] = 0.0;
  wave_lds_sync();
  for (int k = 0; k < sp.max_iter; ++k) {
    it = k + 1;
    if (ind == 0u) {
      if (lane < kMsMaxF) c[lane] = 0.0;
      wave_lds_sync();
      break;
    }
    ok &= wave_chol_solve(G, b, n_sys, F, ind, sp.alpha, M, v, c, lane);
    wave_lds_sync();
    const bool big_l = lane < F && fabs(c[lane]) >= sp.thr;
    if (lane < F && !big_l) c[lane] = 0.0;
    wave_lds_sync();
    const unsigned big = (unsigned)__builtin_amdgcn_readfirstlane((int)(uint32_t)__ballot(big_l));
    const unsigned pattern = (unsigned)__builtin_amdgcn_readfirstlane((int)(uint32_t)__ballot(lane < F && c[lane] != 0.0));
    ind = big;
    if (ind == all || pattern == prev) break;
    prev = pattern;
  }
  const unsigned sup = (unsigned)__builtin_amdgcn_readfirstlane((int)(uint32_t)__ballot(lane < F && fabs(c[lane]) > 1e-14));
  if (sp.unbias && sup) ok &= wave_chol_solve(G, b, n_sys, F, sup, 0.0, M, v, c, lane);
  wave_lds_sync();
  if (lane < F) {
    coef[(int64_t)s * F + lane] = c[lane];
    if (mask) mask[(int64_t)s * F + lane] = (int8_t)((sup >> lane) & 1u);
  }
  if (lane == 0 && iters) iters[s] = ok ? it : -1;
}

// ---------------------------------------------------------------------------------------------
// Multi-state rollout
// ---------------------------------------------------------------------------------------------
struct MsRollArgs {
  const float* y0;     // [S][ld0]
  const uint32_t* a;   // TIME_MAJOR_BITS [T][lda] (NULL: input column 0 throughout)
  const double* coef;  // [S][F]
  float* y;            // [T][S][ldy]
  int64_t ld0, lda, ldy, N;
  int32_t T, method, substeps;
  double dt, drop;
};

// f(y, a)[S] = C Theta(y, a) (dense over the library; coefficients |c| <= drop zeroed at setup).
template <int S, int NIN, bool INTER>
__device__ __forceinline__ void ms_rhs(const float (&y)[S], float a, const float (&cf)[S][PolyCols<S + NIN, INTER>::F],
                                       float (&f)[S]) {
  constexpr int NZ = S + NIN;
  constexpr PolyCols<NZ, INTER> pc;
  float z[NZ + 1];
  z[0] = 1.0f;
#pragma unroll
  for (int s = 0; s < S; ++s) z[1 + s] = y[s];
#pragma unroll
  for (int q = 0; q < NIN; ++q) z[1 + S + q] = a;
#pragma unroll
  for (int s = 0; s < S; ++s) f[s] = 0.0f;
#pragma unroll
  for (int j = 0; j < PolyCols<NZ, INTER>::F; ++j) {
    const float th = pc.ck[j] == 0 ? z[pc.ci[j]] : z[pc.ci[j]] * z[pc.ck[j]];
#pragma unroll
    for (int s = 0; s < S; ++s) f[s] = fmaf(cf[s][j], th, f[s]);
  }
}

template <int S, int NIN, bool INTER>
__global__ void __launch_bounds__(kBlock) rollout_ms_kernel(MsRollArgs ra) {
  constexpr int F = PolyCols<S + NIN, INTER>::F;
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int64_t p0 = ((int64_t)blockIdx.x * kWavesPerBlock + wid) * kWave;
  if (p0 >= ra.N) return;
  const int64_t p = p0 + lane;
  const bool act = p < ra.N;
  const int64_t pc = act ? p : ra.N - 1;
  float cf[S][F];
#pragma unroll
  for (int s = 0; s < S; ++s)
#pragma unroll
    for (int j = 0; j < F; ++j) {
      const double c = ra.coef[s * F + j];
      cf[s][j] = fabs(c) > ra.drop ? (float)c : 0.0f;
    }
  float y[S];
#pragma unroll
  for (int s = 0; s < S; ++s) y[s] = ra.y0[s * ra.ld0 + pc];
  const float h = (float)(ra.dt / ra.substeps);
  const float h2 = 0.5f * h, h6 = h / 6.0f;
  const int nvalid = (int)(ra.N - p0 < kWave ? ra.N - p0 : kWave);
  const unsigned yoff = act ? (unsigned)(lane * 4) : kOOB;
  const int64_t lda = ra.lda;
  auto word = [&](int g) -> unsigned {  // treatment bits of steps [32 g, 32 g + 32) for this lane
    if (!ra.a) return 0u;
    const int k = 32 * g + (lane & 31);
    const int kk = k < ra.T ? k : ra.T - 1;
    const int64_t col = (p0 >> 5) + (lane >> 5);
    const uint32_t v = col * 32 < ra.N ? ra.a[(int64_t)kk * lda + col] : 0u;  // words past N: not read
    return bit_transpose32(v, lane);
  };
  unsigned wnext = word(0);
  for (int k0 = 0; k0 < ra.T; k0 += 32) {
    const unsigned wcur = wnext;
    if (k0 + 32 < ra.T) wnext = word((k0 >> 5) + 1);  // one group ahead
    const int kend = ra.T - k0 < 32 ? ra.T - k0 : 32;
    for (int i = 0; i < kend; ++i) {
      const float a = (float)((wcur >> i) & 1u);
      for (int sub = 0; sub < ra.substeps; ++sub) {
        if (ra.method == INSITE_METHOD_EULER) {
          float f[S];
          ms_rhs<S, NIN, INTER>(y, a, cf, f);
#pragma unroll
          for (int s = 0; s < S; ++s) y[s] = fmaf(h, f[s], y[s]);
        } else {
          float k1[S], k2[S], k3[S], k4[S], t[S];
          ms_rhs<S, NIN, INTER>(y, a, cf, k1);
#pragma unroll
          for (int s = 0; s < S; ++s) t[s] = fmaf(h2, k1[s], y[s]);
          ms_rhs<S, NIN, INTER>(t, a, cf, k2);
#pragma unroll
          for (int s = 0; s < S; ++s) t[s] = fmaf(h2, k2[s], y[s]);
          ms_rhs<S, NIN, INTER>(t, a, cf, k3);
#pragma unroll
          for (int s = 0; s < S; ++s) t[s] = fmaf(h, k3[s], y[s]);
          ms_rhs<S, NIN, INTER>(t, a, cf, k4);
#pragma unroll
          for (int s = 0; s < S; ++s) y[s] = fmaf(h6, (k1[s] + 2.0f * k2[s]) + (2.0f * k3[s] + k4[s]), y[s]);
        }
      }
      const int k = k0 + i;
      // step row k: S contiguous runs of N floats; this wave's 64 columns through a range-checked
      // descriptor (lanes past N carry an out-of-range offset)
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(ra.y + (int64_t)k * S * ra.ldy + p0), (short)0, (int)(((int64_t)(S - 1) * ra.ldy + nvalid) * 4),
          0x00020000);
#pragma unroll
      for (int s = 0; s < S; ++s)
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, y[s]), rs, yoff + (unsigned)(s * ra.ldy * 4),
                                              0, kStoreAux);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// host helpers
// ---------------------------------------------------------------------------------------------
// The exponent table must be the pysindy PolynomialLibrary(degree 2, interaction_only) over S + NIN
// inputs (states first, then inputs); returns the matching interaction flag or -1.
int ms_library_kind(const int8_t* exps, int F, int S, int NIN) {
  const int n = S + NIN;
  for (int inter = 1; inter >= 0; --inter) {
    if (F != ms_cols(n, inter)) continue;
    bool ok = true;
    int j = 0;
    auto row_is = [&](int i, int k) {  // column with inputs i, k (-1 = none)
      for (int q = 0; q < n; ++q) {
        int e = (q == i) + (q == k);
        if (exps[j * n + q] != e) return false;
      }
      return true;
    };
    ok &= row_is(-1, -1);
    ++j;
    for (int i = 0; ok && i < n; ++i, ++j) ok &= row_is(i, -1);
    for (int i = 0; ok && i < n; ++i)
      for (int k = inter ? i + 1 : i; ok && k < n; ++k, ++j) ok &= row_is(i, k);
    if (ok) return inter;
  }
  return -1;
}

// Interior chunks per tile for gram_ms4_kernel: the count (<= 8, >= 48 emitted steps per chunk) whose
// units fill the last round of resident waves best (15625 tiles on 2048 waves: 7.6 tiles per wave as whole
// tiles, 30.5 of 31 rounds in quarter tiles).
inline int ms4_chunks(int64_t N, int n_steps, int grid) {
  const int64_t tiles = (N + kWave - 1) / kWave;
  const int64_t waves = (int64_t)grid * kWavesPerBlock;
  int best = 1;
  double best_eff = 0.0;
  for (int c = 1; c <= 8; ++c) {
    if (c > 1 && (n_steps - 8) / c < 48) break;
    const int64_t units = tiles * c;
    const int64_t rounds = (units + waves - 1) / waves;
    const double eff = (double)units / (double)(rounds * waves) - 0.004 * (c - 1);  // ~1 exposed load latency per chunk
    if (eff > best_eff + 1e-9) {
      best_eff = eff;
      best = c;
    }
  }
  return best;
}

inline int ms_grid(int64_t N) {
  int64_t tiles = (N + kWave - 1) / kWave;
  int64_t g = (tiles + kWavesPerBlock - 1) / kWavesPerBlock;
  // one resident round: 256 CUs x INSITE_MS_WPE blocks of 4 waves (one wave per SIMD per block)
  constexpr int kResident = 256 * INSITE_MS_WPE < kMsMaxBlocks ? 256 * INSITE_MS_WPE : kMsMaxBlocks;
  if (g > kResident) g = kResident;
  if (g < 1) g = 1;
  return (int)g;
}

// ---------------------------------------------------------------------------------------------
// Support-specialised S-state rollout, generated at run time (hipRTC).  A discovered model is sparse
// (C3: 11 of the 110 state x column coefficients), and the dense RHS keeps the rollout VALU-bound
// (SURVEY.md §7.3-4).  The generated kernel evaluates exactly the supported terms, column by column in
// library order: with the dropped terms contributing fmaf(0, th, f) = f, the sums are the dense ones.
// The coefficient VALUES stay device data (read once per wave into scalar registers); only the support
// pattern is compiled in.  If any coefficient outside the pattern is above the drop threshold the
// launch takes the embedded dense RHS instead, so a stale pattern can cost speed, never correctness.
// ---------------------------------------------------------------------------------------------
const char* kMsSparseTemplate = R"HIPSRC(
#define S @S@
#define NIN @NIN@
#define F @F@
#define METHOD @METHOD@
static __device__ __forceinline__ unsigned bit_transpose32(unsigned x, int lane) {
  const unsigned m[5] = {0x0000FFFFu, 0x00FF00FFu, 0x0F0F0F0Fu, 0x33333333u, 0x55555555u};
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const int sh = 16 >> k;
    const unsigned y = (unsigned)__shfl_xor((int)x, sh, 64);
    x = (lane & sh) ? ((x & ~m[k]) | ((y >> sh) & m[k])) : ((x & m[k]) | ((y << sh) & ~m[k]));
  }
  return x;
}
__constant__ int kCI[F] = {@CI@};
__constant__ int kCK[F] = {@CK@};
static __device__ __forceinline__ void rhs_dense(const float (&v)[S], float a, const float (&cf)[S][F], float (&f)[S]) {
  float z[S + NIN + 1];
  z[0] = 1.0f;
#pragma unroll
  for (int s = 0; s < S; ++s) z[1 + s] = v[s];
#pragma unroll
  for (int q = 0; q < NIN; ++q) z[1 + S + q] = a;
#pragma unroll
  for (int s = 0; s < S; ++s) f[s] = 0.0f;
#pragma unroll
  for (int j = 0; j < F; ++j) {
    const float th = kCK[j] == 0 ? z[kCI[j]] : z[kCI[j]] * z[kCK[j]];
#pragma unroll
    for (int s = 0; s < S; ++s) f[s] = fmaf(cf[s][j], th, f[s]);
  }
}
static __device__ __forceinline__ float coef_at(const double* c, int i, double drop) {
  const double v = c[i];
  return fabs(v) > drop ? (float)v : 0.0f;
}
extern "C" __global__ void __launch_bounds__(256) ms_rollout_sparse(
    const float* __restrict__ y0, long long ld0, const unsigned* __restrict__ abits, long long lda,
    const double* __restrict__ coef, float* __restrict__ yout, long long ldy, long long N, int T, int substeps,
    double dt, double drop) {
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const long long p0 = ((long long)blockIdx.x * 4 + wid) * 64;
  if (p0 >= N) return;
  const long long p = p0 + lane;
  const bool act = p < N;
  const long long pc = act ? p : N - 1;
  // pattern check: every coefficient outside the compiled support must be dropped
  const unsigned long long sup[2] = {@SUPLO@ull, @SUPHI@ull};
  bool viol = false;
  for (int t = lane; t < S * F; t += 64) {
    const bool in = (sup[t >> 6] >> (t & 63)) & 1ull;
    viol = viol || (!in && fabs(coef[t]) > drop);
  }
  const bool dense = __ballot(viol) != 0ull;
  float y[S];
#pragma unroll
  for (int s = 0; s < S; ++s) y[s] = y0[s * ld0 + pc];
  const float h = (float)(dt / substeps);
  const float h2 = 0.5f * h, h6 = h / 6.0f;
  const int nvalid = (int)(N - p0 < 64 ? N - p0 : 64);
  const unsigned yoff = act ? (unsigned)(lane * 4) : 0x80000000u;
  auto word = [&](int g) -> unsigned {
    if (!abits) return 0u;
    const int k = 32 * g + (lane & 31);
    const int kk = k < T ? k : T - 1;
    const long long col = (p0 >> 5) + (lane >> 5);
    const unsigned v = col * 32 < N ? abits[(long long)kk * lda + col] : 0u;
    return bit_transpose32(v, lane);
  };
  auto run = [&](auto&& rhs) {
    unsigned wnext = word(0);
    for (int k0 = 0; k0 < T; k0 += 32) {
      const unsigned wcur = wnext;
      if (k0 + 32 < T) wnext = word((k0 >> 5) + 1);
      const int kend = T - k0 < 32 ? T - k0 : 32;
      for (int i = 0; i < kend; ++i) {
        const float a = (float)((wcur >> i) & 1u);
        for (int sub = 0; sub < substeps; ++sub) {
          if (METHOD == 0) {
            float f[S];
            rhs(y, a, f);
#pragma unroll
            for (int s = 0; s < S; ++s) y[s] = fmaf(h, f[s], y[s]);
          } else {
            float k1[S], k2[S], k3[S], k4[S], t[S];
            rhs(y, a, k1);
#pragma unroll
            for (int s = 0; s < S; ++s) t[s] = fmaf(h2, k1[s], y[s]);
            rhs(t, a, k2);
#pragma unroll
            for (int s = 0; s < S; ++s) t[s] = fmaf(h2, k2[s], y[s]);
            rhs(t, a, k3);
#pragma unroll
            for (int s = 0; s < S; ++s) t[s] = fmaf(h, k3[s], y[s]);
            rhs(t, a, k4);
#pragma unroll
            for (int s = 0; s < S; ++s) y[s] = fmaf(h6, (k1[s] + 2.0f * k2[s]) + (2.0f * k3[s] + k4[s]), y[s]);
          }
        }
        const int k = k0 + i;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(yout + (long long)k * S * ldy + p0), (short)0, (int)(((long long)(S - 1) * ldy + nvalid) * 4),
            0x00020000);
#pragma unroll
        for (int s = 0; s < S; ++s)
          __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, y[s]), rs, yoff + (unsigned)(s * ldy * 4),
                                                0, @AUX@);
      }
    }
  };
  if (dense) {
    float cf[S][F];
#pragma unroll
    for (int s = 0; s < S; ++s)
#pragma unroll
      for (int j = 0; j < F; ++j) cf[s][j] = coef_at(coef, s * F + j, drop);
    run([&](const float (&v)[S], float a, float (&f)[S]) { rhs_dense(v, a, cf, f); });
  } else {
@COEFS@
    run([&](const float (&v)[S], float a, float (&f)[S]) {
      float z[S + NIN + 1];
      z[0] = 1.0f;
#pragma unroll
      for (int s = 0; s < S; ++s) z[1 + s] = v[s];
#pragma unroll
      for (int q = 0; q < NIN; ++q) z[1 + S + q] = a;
#pragma unroll
      for (int s = 0; s < S; ++s) f[s] = 0.0f;
@BODY@
    });
  }
}
)HIPSRC";

std::string ms_replace(std::string src, const std::string& key, const std::string& val) {
  for (size_t pos; (pos = src.find(key)) != std::string::npos;) src.replace(pos, key.size(), val);
  return src;
}

// Kernel source for one (S, NIN, method, support) — interaction-only degree-2 library.
template <int S, int NIN>
std::string ms_sparse_source(int method, const int8_t* support) {
  constexpr PolyCols<S + NIN, true> pc;
  constexpr int F = PolyCols<S + NIN, true>::F;
  std::string ci, ck, coefs, body;
  unsigned long long sup[2] = {0ull, 0ull};
  for (int j = 0; j < F; ++j) {
    ci += std::to_string(pc.ci[j]) + (j + 1 < F ? "," : "");
    ck += std::to_string(pc.ck[j]) + (j + 1 < F ? "," : "");
  }
  for (int j = 0; j < F; ++j) {  // column order = the dense kernel's summation order
    bool any = false;
    std::string col;
    for (int st = 0; st < S; ++st) {
      const int t = st * F + j;
      if (!support[t]) continue;
      sup[t >> 6] |= 1ull << (t & 63);
      coefs += "    const float c" + std::to_string(t) + " = coef_at(coef, " + std::to_string(t) + ", drop);\n";
      col += "        f[" + std::to_string(st) + "] = fmaf(c" + std::to_string(t) + ", th, f[" + std::to_string(st) + "]);\n";
      any = true;
    }
    if (!any) continue;
    const std::string th = pc.ck[j] == 0 ? "z[" + std::to_string(pc.ci[j]) + "]"
                                         : "z[" + std::to_string(pc.ci[j]) + "] * z[" + std::to_string(pc.ck[j]) + "]";
    body += "      {\n        const float th = " + th + ";\n" + col + "      }\n";
  }
  std::string src = kMsSparseTemplate;
  src = ms_replace(src, "@S@", std::to_string(S));
  src = ms_replace(src, "@NIN@", std::to_string(NIN));
  src = ms_replace(src, "@F@", std::to_string(F));
  src = ms_replace(src, "@METHOD@", std::to_string(method == INSITE_METHOD_EULER ? 0 : 1));
  src = ms_replace(src, "@CI@", ci);
  src = ms_replace(src, "@CK@", ck);
  src = ms_replace(src, "@SUPLO@", std::to_string(sup[0]));
  src = ms_replace(src, "@SUPHI@", std::to_string(sup[1]));
  src = ms_replace(src, "@AUX@", std::to_string(kStoreAux));
  src = ms_replace(src, "@COEFS@", coefs);
  src = ms_replace(src, "@BODY@", body);
  return src;
}

// Compiled kernels, one per (device, source), compiled once under the lock.  A support that fails to
// compile or load is remembered as nullptr (the caller then takes the dense kernel and the compile is not
// retried).  The cache is bounded: past kMsJitMax entries new supports run the dense kernel (a model
// family has few distinct supports; the entries' modules stay loaded for the process lifetime).
constexpr size_t kMsJitMax = 64;
struct MsJitCache {
  std::mutex mu;
  std::map<std::pair<int, std::string>, hipFunction_t> fns;
};
MsJitCache& ms_jit_cache() {
  static MsJitCache c;
  return c;
}

hipFunction_t ms_jit_function(const std::string& src) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  MsJitCache& c = ms_jit_cache();
  std::lock_guard<std::mutex> lk(c.mu);
  const auto key = std::make_pair(dev, src);
  auto it = c.fns.find(key);
  if (it != c.fns.end()) return it->second;
  if (c.fns.size() >= kMsJitMax) return nullptr;
  hipFunction_t fn = nullptr;
  // the target is the current device's own ISA (gcnArchName, e.g. "gfx950:sramecc+:xnack-")
  hipDeviceProp_t prop;
  std::string arch = "--offload-arch=gfx950";
  if (hipGetDeviceProperties(&prop, dev) == hipSuccess && prop.gcnArchName[0])
    arch = std::string("--offload-arch=") + std::string(prop.gcnArchName).substr(0, std::string(prop.gcnArchName).find(':'));
  hiprtcProgram prog;
  std::vector<char> code;
  if (hiprtcCreateProgram(&prog, src.c_str(), "insite_ms_sparse.hip", 0, nullptr, nullptr) == HIPRTC_SUCCESS) {
    const char* opts[] = {arch.c_str(), "-O3", "-std=c++17", "-ffp-contract=fast-honor-pragmas"};
    if (hiprtcCompileProgram(prog, 4, opts) == HIPRTC_SUCCESS) {
      size_t n = 0;
      if (hiprtcGetCodeSize(prog, &n) == HIPRTC_SUCCESS && n > 0) {
        code.resize(n);
        if (hiprtcGetCode(prog, code.data()) != HIPRTC_SUCCESS) code.clear();
      }
    }
    hiprtcDestroyProgram(&prog);
  }
  hipModule_t mod = nullptr;
  if (!code.empty() && hipModuleLoadData(&mod, code.data()) == hipSuccess) {
    if (hipModuleGetFunction(&fn, mod, "ms_rollout_sparse") != hipSuccess) {
      fn = nullptr;
      (void)hipModuleUnload(mod);
    }
  }
  (void)hipGetLastError();  // a failed compile / load must not leak into the caller's launch status
  c.fns.emplace(key, fn);   // nullptr remembered: the dense kernel serves this support
  return fn;
}

}  // namespace

extern "C" {

size_t insite_gram_ms_workspace_bytes(int64_t n_patients) {
  return (size_t)ms_grid(n_patients) * kMsTiles * 256 * sizeof(double);
}

int32_t insite_gram_ms_f32(const float* x, int64_t ldx, int32_t n_steps, int32_t n_states, const uint32_t* inp_bits,
                           int64_t ld_bits, const int32_t* rows, int64_t n_patients, const int8_t* exps,
                           int32_t n_terms, int32_t fd_kind, double dt, double* G_out, double* B_out, void* workspace,
                           size_t workspace_bytes, void* stream) {
  if (n_states != 5) return INSITE_E_UNSUPPORTED;  // instantiated for the C3 system
  if (n_patients < 0 || n_steps < 0 || ldx < n_patients || !(dt > 0.0) || !G_out || !B_out || !exps)
    return INSITE_E_INVALID_ARG;
  if (fd_kind != INSITE_FD_SMOOTHED4) return INSITE_E_UNSUPPORTED;
  const int nin = inp_bits ? 1 : 0;
  if (inp_bits && ld_bits < (n_patients + 31) / 32) return INSITE_E_INVALID_ARG;
  const int inter = ms_library_kind(exps, n_terms, n_states, nin);
  if (inter < 0) return INSITE_E_UNSUPPORTED;
  if (n_terms + n_states > kMsMaxF) return INSITE_E_UNSUPPORTED;
  if (!workspace || workspace_bytes < insite_gram_ms_workspace_bytes(n_patients)) return INSITE_E_WORKSPACE;
  if (n_patients > 0 && !x) return INSITE_E_INVALID_ARG;
  // the per-step buffer descriptor (INSITE_MS4_BUFLD) spans the S state rows of one step with 32-bit byte
  // offsets (s * ldx * 4 and its size): refuse cohorts whose step block leaves that range
  if ((int64_t)n_states * ldx * 4 > (int64_t)INT32_MAX) return INSITE_E_UNSUPPORTED;
  hipStream_t hs = reinterpret_cast<hipStream_t>(stream);
  double* part = static_cast<double*>(workspace);
  const int grid = ms_grid(n_patients);
  GramW w;
  w.sg0 = 17.0 / 35.0;
  w.sg1 = 12.0 / 35.0;
  w.sg2 = -3.0 / 35.0;
  w.inv_dt = 1.0 / dt;
  w.fd1 = (2.0 / 3.0) * w.inv_dt;
  w.fd2 = (-1.0 / 12.0) * w.inv_dt;
  if (nin == 1 && inter != 1) return INSITE_E_UNSUPPORTED;  // 5 states + input, full degree 2: F + S > 32
#ifdef INSITE_MS_V1  // the 16 x 16 x 4 tile form (A/B builds, tools/build_ablation.sh)
  if (n_patients == 0 || n_steps < 5) {
    if (hipMemsetAsync(part, 0, (size_t)grid * kMsTiles * 256 * sizeof(double), hs) != hipSuccess) return INSITE_E_HIP;
  } else if (nin == 1) {
    gram_ms_kernel<5, 1, true><<<grid, kBlock, 0, hs>>>(x, ldx, n_steps, inp_bits, ld_bits, rows, n_patients, w, part);
  } else if (inter == 1) {
    gram_ms_kernel<5, 0, true><<<grid, kBlock, 0, hs>>>(x, ldx, n_steps, nullptr, 0, rows, n_patients, w, part);
  } else {
    gram_ms_kernel<5, 0, false><<<grid, kBlock, 0, hs>>>(x, ldx, n_steps, nullptr, 0, rows, n_patients, w, part);
  }
  int32_t st = launch_status();
  if (st != INSITE_OK) return st;
  ms_finalize<<<(kMsTiles * 256 + kWave - 1) / kWave, kWave, 0, hs>>>(part, grid, n_terms, n_states, G_out, B_out);
#else
  int nb = 0, cgn = 0;
  bool cover = false;
  Ms4Map map{};
  auto geom = [&](auto m4) {
    using M4 = decltype(m4);
    static_assert(M4::NB * 16 <= kMsTiles * 256, "workspace holds the block partials");
    nb = M4::NB;
    if constexpr (M4::kCover) {
      cover = true;
    } else {
      cgn = M4::CG;
      for (int j = 0; j < kMsMaxF; ++j) map.col[j] = j < 4 * M4::CG ? m4.col[j] : -1;
    }
  };
#ifdef INSITE_MS4_NCHUNK
  const int nchunk = INSITE_MS4_NCHUNK;
#else
  const int nchunk = ms4_chunks(n_patients, n_steps, grid);
#endif
  if (nin == 1) geom(Ms4Layout<5, 6, true>{});
  else if (inter == 1) geom(Ms4Layout<5, 5, true>{});
  else geom(Ms4Layout<5, 5, false>{});
  if (n_patients == 0 || n_steps < 5) {
    if (hipMemsetAsync(part, 0, (size_t)grid * nb * 16 * sizeof(double), hs) != hipSuccess) return INSITE_E_HIP;
  } else if (nin == 1) {
    gram_ms4_kernel<5, 1, true><<<grid, kBlock, 0, hs>>>(x, ldx, n_steps, inp_bits, ld_bits, rows, n_patients, w, part,
                                                              nchunk);
  } else if (inter == 1) {
    gram_ms4_kernel<5, 0, true><<<grid, kBlock, 0, hs>>>(x, ldx, n_steps, nullptr, 0, rows, n_patients, w, part,
                                                              nchunk);
  } else {
    gram_ms4_kernel<5, 0, false><<<grid, kBlock, 0, hs>>>(x, ldx, n_steps, nullptr, 0, rows, n_patients, w, part,
                                                              nchunk);
  }
  int32_t st = launch_status();
  if (st != INSITE_OK) return st;
  if (cover) {
    if (n_terms * n_terms + n_terms * n_states != kMs4CoverEntries) return INSITE_E_INVALID_ARG;
    ms4_finalize_cover<<<(kMs4CoverEntries + kWave - 1) / kWave, kWave, 0, hs>>>(part, grid, nb, n_terms, G_out, B_out);
  } else {
    ms4_finalize<<<(nb * 16 + kWave - 1) / kWave, kWave, 0, hs>>>(part, grid, nb, cgn, n_terms, n_states, map, G_out,
                                                                  B_out);
  }
#endif
  return launch_status();
}

int32_t insite_stlsq_wave_f64(const double* G, const double* B, int32_t n_terms, int32_t n_targets, double threshold,
                              double alpha, int32_t max_iter, int32_t unbias, double* coef_out, int8_t* mask_out,
                              int32_t* iters_out, void* stream) {
  if (n_terms < 1 || n_terms > kMsMaxF || n_targets < 0 || !G || !B || !coef_out || max_iter < 1)
    return INSITE_E_INVALID_ARG;
  if (n_targets == 0) return INSITE_OK;
  StlsqParams sp{threshold, alpha, max_iter, unbias, 1};
  stlsq_wave_kernel<<<n_targets, kWave, 0, reinterpret_cast<hipStream_t>(stream)>>>(G, B, n_terms, n_targets, sp,
                                                                                     coef_out, mask_out, iters_out);
  return launch_status();
}

int32_t insite_rollout_ms_f32(const float* y0, int64_t ld_y0, const uint32_t* inp_bits, int64_t ld_bits,
                              const double* coef, const int8_t* exps, int32_t n_terms, int32_t n_states,
                              int64_t n_rows, int32_t T, double dt, int32_t method, int32_t substeps,
                              double drop_below, float* y_out, int64_t ld_y, void* stream) {
  if (n_states != 5) return INSITE_E_UNSUPPORTED;
  if (n_rows < 0 || T < 0 || substeps < 1 || !(dt >= 0.0) || ld_y0 < n_rows || ld_y < n_rows || !exps)
    return INSITE_E_INVALID_ARG;
  if (inp_bits && ld_bits < (n_rows + 31) / 32) return INSITE_E_INVALID_ARG;
  if (method != INSITE_METHOD_EULER && method != INSITE_METHOD_RK4) return INSITE_E_UNSUPPORTED;
  const int nin = inp_bits ? 1 : 0;
  const int inter = ms_library_kind(exps, n_terms, n_states, nin);
  if (inter != 1) return INSITE_E_UNSUPPORTED;
  if (n_rows == 0 || T == 0) return INSITE_OK;
  if (!y0 || !coef || !y_out) return INSITE_E_INVALID_ARG;
  if ((int64_t)n_states * ld_y * 4 >= ((int64_t)1 << 31)) return INSITE_E_UNSUPPORTED;  // 32-bit step offsets
  MsRollArgs ra{y0, inp_bits, coef, y_out, ld_y0, ld_bits, ld_y, n_rows, T, method, substeps, dt, drop_below};
  const int64_t waves = (n_rows + kWave - 1) / kWave;
  const dim3 grid((unsigned)((waves + kWavesPerBlock - 1) / kWavesPerBlock));
  hipStream_t hs = reinterpret_cast<hipStream_t>(stream);
  if (nin == 1) rollout_ms_kernel<5, 1, true><<<grid, kBlock, 0, hs>>>(ra);
  else rollout_ms_kernel<5, 0, true><<<grid, kBlock, 0, hs>>>(ra);
  return launch_status();
}

int32_t insite_rollout_ms_sparse_f32(const float* y0, int64_t ld_y0, const uint32_t* inp_bits, int64_t ld_bits,
                                     const double* coef, const int8_t* support, const int8_t* exps, int32_t n_terms,
                                     int32_t n_states, int64_t n_rows, int32_t T, double dt, int32_t method,
                                     int32_t substeps, double drop_below, float* y_out, int64_t ld_y, void* stream) {
  if (n_states != 5) return INSITE_E_UNSUPPORTED;
  if (n_rows < 0 || T < 0 || substeps < 1 || !(dt >= 0.0) || ld_y0 < n_rows || ld_y < n_rows || !exps || !support)
    return INSITE_E_INVALID_ARG;
  if (inp_bits && ld_bits < (n_rows + 31) / 32) return INSITE_E_INVALID_ARG;
  if (method != INSITE_METHOD_EULER && method != INSITE_METHOD_RK4) return INSITE_E_UNSUPPORTED;
  const int nin = inp_bits ? 1 : 0;
  if (ms_library_kind(exps, n_terms, n_states, nin) != 1) return INSITE_E_UNSUPPORTED;
  if (n_rows == 0 || T == 0) return INSITE_OK;
  if (!y0 || !coef || !y_out) return INSITE_E_INVALID_ARG;
  if ((int64_t)n_states * ld_y * 4 >= ((int64_t)1 << 31)) return INSITE_E_UNSUPPORTED;  // 32-bit step offsets
  const std::string src = nin ? ms_sparse_source<5, 1>(method, support) : ms_sparse_source<5, 0>(method, support);
  hipFunction_t fn = ms_jit_function(src);
  if (!fn)  // no specialised kernel for this support (compile / load failure, cache full): dense RHS
    return insite_rollout_ms_f32(y0, ld_y0, inp_bits, ld_bits, coef, exps, n_terms, n_states, n_rows, T, dt, method,
                                 substeps, drop_below, y_out, ld_y, stream);
  long long ld0 = ld_y0, lda = ld_bits, ldy = ld_y, N = n_rows;
  int Ti = T, sub = substeps;
  double dti = dt, drop = drop_below;
  const unsigned* ab = inp_bits;
  void* args[] = {(void*)&y0, &ld0, (void*)&ab, &lda, (void*)&coef, (void*)&y_out, &ldy, &N, &Ti, &sub, &dti, &drop};
  const int64_t waves = (n_rows + kWave - 1) / kWave;
  const unsigned grid = (unsigned)((waves + kWavesPerBlock - 1) / kWavesPerBlock);
  if (hipModuleLaunchKernel(fn, grid, 1, 1, kBlock, 1, 1, 0, reinterpret_cast<hipStream_t>(stream), args, nullptr) !=
      hipSuccess)
    return INSITE_E_HIP;
  return INSITE_OK;
}

}  // extern "C"
