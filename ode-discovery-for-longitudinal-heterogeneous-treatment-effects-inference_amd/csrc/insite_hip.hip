// insite_hip.hip — MI355X (gfx950, CDNA4) kernels + C ABI for the INSITE ODE-discovery hot path.
//
// Kernels (DESIGN.md §3 gives the roofline and algorithmic bytes of each):
//   gram_kernel        fused savgol(5,3) smoothing + 4th-order finite differences + polynomial
//                      library + per-arm Gram/moment accumulation.  Lane = patient; the patients'
//                      rows are staged [64 patients x KT steps] through LDS so every HBM load is a
//                      coalesced 16-B-per-lane row segment, then each lane streams its own row
//                      through a 9-deep register window.  Theta is affine in x for a fixed patient
//                      (polynomial library over [x, u] with u constant per patient), so a patient's
//                      Gram block is A(u) M A(u)^T with M the 2x2 (+2 moment) matrix of the smoothed
//                      series: per row the lane only updates 4 running moments; the per-patient
//                      A M A^T expansion is done cooperatively (one Gram entry per lane) from LDS.
//                      Replaces pysindy SmoothedFiniteDifference + PolynomialLibrary + the X^T X of
//                      sklearn's ridge (reference sindy.py:190-192).
//   gram_finalize      fixed-order reduction of the per-block partials -> G[A,F,F], b[A,F].
//   stlsq_kernel       one STLSQ system per thread; masked Cholesky in registers (pkpd/utils.py:213-327).
//   rollout_kernel     lane = patient, ODE state in registers; per-step int8 arm staged through LDS;
//                      outputs staged [64 x KT] through LDS and stored as contiguous row segments
//                      (sindy.py:413-431, pkpd/utils.py:68-94).
//   sse_kernel         masked squared-error sums for the RMSE metrics (time_varying_model.py:236-313).
//
// All reductions are fixed-order (bitwise reproducible for a fixed problem size).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstring>

#include "insite_hip.h"

namespace {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWave * kWavesPerBlock;
constexpr int kMaxEntries = 64;       // Gram + moment entries, one per lane
constexpr int kGramMaxBlocks = 1024;  // fixed cap -> deterministic reduction order
constexpr int kPsStride = 17;         // per-patient LDS scratch row (odd -> conflict-free)

// Polynomial library over [x, u_0..u_{U-1}] (one state, U statics), pysindy column order.
struct LibDesc {
  int32_t F;   // columns
  int32_t U;   // statics
  int32_t nG;  // F(F+1)/2 Gram entries (upper triangle, row-major)
  int32_t nE;  // nG + F
  int8_t ex[INSITE_MAX_TERMS];
  int8_t eu[INSITE_MAX_TERMS][INSITE_MAX_STATICS];
  int8_t ei[kMaxEntries];
  int8_t ek[kMaxEntries];  // -1 => moment entry b[ei]
};

// ---------------------------------------------------------------------------------------------
// stencil weights (oracle/insite_ref.py SAVGOL_5_3 / FD4; scipy savgol_filter mode='interp',
// pysindy FiniteDifference(order=4) with one-sided 5-point end stencils)
// ---------------------------------------------------------------------------------------------
#define SGC(a, b, c, d, e, den) a / den, b / den, c / den, d / den, e / den
__device__ __forceinline__ double dot5(double w0, double w1, double w2, double w3, double w4,
                                       double a, double b, double c, double d, double e) {
  return w0 * a + w1 * b + w2 * c + w3 * d + w4 * e;
}

__device__ __forceinline__ double sg_interior(double a, double b, double c, double d, double e) {
  return dot5(SGC(-3.0, 12.0, 17.0, 12.0, -3.0, 35.0), a, b, c, d, e);
}
__device__ __forceinline__ double sg_pos0(double a, double b, double c, double d, double e) {
  return dot5(SGC(69.0, 4.0, -6.0, 4.0, -1.0, 70.0), a, b, c, d, e);
}
__device__ __forceinline__ double sg_pos1(double a, double b, double c, double d, double e) {
  return dot5(SGC(2.0, 27.0, 12.0, -8.0, 2.0, 35.0), a, b, c, d, e);
}
__device__ __forceinline__ double sg_pos3(double a, double b, double c, double d, double e) {
  return dot5(SGC(2.0, -8.0, 12.0, 27.0, 2.0, 35.0), a, b, c, d, e);
}
__device__ __forceinline__ double sg_pos4(double a, double b, double c, double d, double e) {
  return dot5(SGC(-1.0, 4.0, -6.0, 4.0, 69.0, 70.0), a, b, c, d, e);
}
__device__ __forceinline__ double fd_interior(double a, double b, double /*c*/, double d, double e) {
  return (1.0 / 12.0) * a + (-2.0 / 3.0) * b + (2.0 / 3.0) * d + (-1.0 / 12.0) * e;
}
__device__ __forceinline__ double fd_pos0(double a, double b, double c, double d, double e) {
  return dot5(-25.0 / 12.0, 4.0, -3.0, 4.0 / 3.0, -0.25, a, b, c, d, e);
}
__device__ __forceinline__ double fd_pos1(double a, double b, double c, double d, double e) {
  return dot5(-0.25, -5.0 / 6.0, 1.5, -0.5, 1.0 / 12.0, a, b, c, d, e);
}
__device__ __forceinline__ double fd_pos3(double a, double b, double c, double d, double e) {
  return dot5(-1.0 / 12.0, 0.5, -1.5, 5.0 / 6.0, 0.25, a, b, c, d, e);
}
__device__ __forceinline__ double fd_pos4(double a, double b, double c, double d, double e) {
  return dot5(0.25, -4.0 / 3.0, 3.0, -4.0, 25.0 / 12.0, a, b, c, d, e);
}

// LDS hand-off between lanes of ONE wavefront: DS instructions of a wave execute in order, so
// only the compiler must be kept from reordering across this point.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}

__device__ __forceinline__ int wave_min_i(int v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = min(v, __shfl_xor(v, off, kWave));
  return v;
}
__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = max(v, __shfl_xor(v, off, kWave));
  return v;
}

__device__ __forceinline__ double monomial(const LibDesc& lib, int j, const double* u) {
  double m = 1.0;
  for (int i = 0; i < lib.U; ++i)
    for (int e = 0; e < lib.eu[j][i]; ++e) m *= u[i];
  return m;
}

// =============================================================================================
// Discovery: fused smoothing + FD + library + Gram
// =============================================================================================
template <int KT, int VEC, int NARM, bool SMOOTH>
__global__ void __launch_bounds__(kBlock)
gram_kernel(const double* __restrict__ x, int64_t ldx, const double* __restrict__ u,
            const int8_t* __restrict__ arm, const int32_t* __restrict__ rows, int64_t N,
            double inv_dt, LibDesc lib, double* __restrict__ partial) {
  constexpr int kRowStride = KT + 1;  // odd (KT even): lane-per-row reads are bank-conflict free
  __shared__ double smem[kWavesPerBlock * kWave * kRowStride];
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  double* xt = smem + wid * (kWave * kRowStride);

  double acc[NARM];
#pragma unroll
  for (int a = 0; a < NARM; ++a) acc[a] = 0.0;
  const int my_i = lane < lib.nE ? lib.ei[lane] : 0;
  const int my_k = lane < lib.nE ? lib.ek[lane] : 0;
  const int my_exi = lib.ex[my_i];
  const int my_exk = my_k >= 0 ? lib.ex[my_k] : 0;

  const int64_t n_tiles = (N + kWave - 1) / kWave;
  for (int64_t tile = (int64_t)blockIdx.x * kWavesPerBlock + wid; tile < n_tiles;
       tile += (int64_t)gridDim.x * kWavesPerBlock) {
    const int64_t p0 = tile * kWave;
    const int64_t p = p0 + lane;
    int L = 0;
    if (p < N) {
      L = rows[p];
      if (L > ldx) L = (int)ldx;
      if (L < 5) L = 0;  // too short for the 5-point stencils: contributes nothing
    }
    const int Lmin = wave_min_i(L);
    const int Lmax = wave_max_i(L);
    const int steps = Lmax > 0 ? Lmax + 8 : 0;  // delay line: xs lags 4, d lags 8

    double r0 = 0, r1 = 0, r2 = 0, r3 = 0, r4 = 0, r5 = 0, r6 = 0, r7 = 0, r8 = 0;  // raw x[t-8..t]
    double s0 = 0, s1 = 0, s2 = 0, s3 = 0, s4 = 0, s5 = 0, s6 = 0, s7 = 0, s8 = 0;  // xs[t-12..t-4]
    double Sx = 0, Sxx = 0, Sd = 0, Sdx = 0;

    for (int t0 = 0; t0 < steps; t0 += KT) {
      // ---- stage x[p0..p0+63][t0..t0+KT) into LDS: coalesced VEC*8-byte row segments ----
      if (t0 < Lmax) {
        constexpr int LPR = KT / VEC;      // lanes per row
        constexpr int RPI = kWave / LPR;   // rows per wave instruction
        const int cl = (lane % LPR) * VEC;
        const int64_t col = t0 + cl;
        double v[kWave / RPI][VEC];
#pragma unroll
        for (int it = 0; it < kWave / RPI; ++it) {
          const int r = it * RPI + lane / LPR;
          const int64_t pr = p0 + r;
          if (pr < N && col < Lmax) {
            if constexpr (VEC == 2) {
              const double2 w = *reinterpret_cast<const double2*>(x + pr * ldx + col);
              v[it][0] = w.x;
              v[it][1] = w.y;
            } else {
              v[it][0] = x[pr * ldx + col];
            }
          } else {
#pragma unroll
            for (int q = 0; q < VEC; ++q) v[it][q] = 0.0;
          }
        }
        wave_lds_sync();  // previous tile's reads done
#pragma unroll
        for (int it = 0; it < kWave / RPI; ++it) {
          const int r = it * RPI + lane / LPR;
#pragma unroll
          for (int q = 0; q < VEC; ++q) xt[r * kRowStride + cl + q] = v[it][q];
        }
        wave_lds_sync();
      }

#pragma unroll
      for (int i = 0; i < KT; ++i) {
        const int t = t0 + i;
        if (t < steps) {
          double xv = (t < L) ? xt[lane * kRowStride + i] : 0.0;
          r0 = r1; r1 = r2; r2 = r3; r3 = r4; r4 = r5; r5 = r6; r6 = r7; r7 = r8; r8 = xv;
          // xs[k], k = t - 4
          const int k = t - 4;
          double xs;
          if constexpr (SMOOTH) {
            xs = sg_interior(r2, r3, r4, r5, r6);
            if (k == 0) xs = sg_pos0(r4, r5, r6, r7, r8);
            if (k == 1) xs = sg_pos1(r3, r4, r5, r6, r7);
            if (k >= Lmin - 2) {
              const double e3 = sg_pos3(r1, r2, r3, r4, r5);
              const double e4 = sg_pos4(r0, r1, r2, r3, r4);
              xs = (k == L - 2) ? e3 : xs;
              xs = (k == L - 1) ? e4 : xs;
            }
          } else {
            xs = r4;
          }
          s0 = s1; s1 = s2; s2 = s3; s3 = s4; s4 = s5; s5 = s6; s6 = s7; s7 = s8; s8 = xs;
          // d[kd], kd = t - 8 (derivative of xs)
          const int kd = t - 8;
          if (kd >= 0) {
            double dv = fd_interior(s2, s3, s4, s5, s6);
            if (kd == 0) dv = fd_pos0(s4, s5, s6, s7, s8);
            if (kd == 1) dv = fd_pos1(s3, s4, s5, s6, s7);
            if (kd >= Lmin - 2) {
              const double e3 = fd_pos3(s1, s2, s3, s4, s5);
              const double e4 = fd_pos4(s0, s1, s2, s3, s4);
              dv = (kd == L - 2) ? e3 : dv;
              dv = (kd == L - 1) ? e4 : dv;
            }
            dv *= inv_dt;
            double xk = s4;
            if (kd >= Lmin) {
              const bool in = kd < L;
              xk = in ? xk : 0.0;
              dv = in ? dv : 0.0;
            }
            Sx += xk;
            Sxx = fma(xk, xk, Sxx);
            Sd += dv;
            Sdx = fma(dv, xk, Sdx);
          }
        }
      }
    }

    // ---- per-patient Gram block A(u) M A(u)^T, one (entry) per lane, patients via LDS ----
    double uu[INSITE_MAX_STATICS] = {0.0, 0.0, 0.0};
    if (L > 0)
      for (int i = 0; i < lib.U; ++i) uu[i] = u[p * lib.U + i];
    wave_lds_sync();
    double* ps = xt;  // reuse the x tile: 64 x kPsStride doubles
    for (int j = 0; j < lib.F; ++j) ps[lane * kPsStride + j] = monomial(lib, j, uu);
    ps[lane * kPsStride + 9] = (double)L;  // moment x^0
    ps[lane * kPsStride + 10] = Sx;        // moment x^1
    ps[lane * kPsStride + 11] = Sxx;       // moment x^2
    ps[lane * kPsStride + 12] = Sd;        // moment xdot * x^0
    ps[lane * kPsStride + 13] = Sdx;       // moment xdot * x^1
    ps[lane * kPsStride + 14] = (L > 0) ? (double)arm[p] : -1.0;
    wave_lds_sync();
    if (lane < lib.nE) {
      const int moff = my_k >= 0 ? 9 + my_exi + my_exk : 12 + my_exi;
      for (int q = 0; q < kWave; ++q) {
        const double* row = ps + q * kPsStride;
        double w = row[my_i] * row[moff];
        if (my_k >= 0) w *= row[my_k];
        const int a = (int)row[14];
#pragma unroll
        for (int aa = 0; aa < NARM; ++aa) acc[aa] += (a == aa) ? w : 0.0;
      }
    }
    wave_lds_sync();
  }

  // ---- block reduction (fixed order) -> partial[block][NARM][64] ----
  __syncthreads();
  double* red = smem;
#pragma unroll
  for (int a = 0; a < NARM; ++a) red[(wid * NARM + a) * kWave + lane] = acc[a];
  __syncthreads();
  if (wid == 0) {
#pragma unroll
    for (int a = 0; a < NARM; ++a) {
      double s = red[(0 * NARM + a) * kWave + lane];
#pragma unroll
      for (int w = 1; w < kWavesPerBlock; ++w) s += red[(w * NARM + a) * kWave + lane];
      partial[((int64_t)blockIdx.x * NARM + a) * kWave + lane] = s;
    }
  }
}

__global__ void __launch_bounds__(kBlock)
gram_finalize(const double* __restrict__ partial, int nblk, int narm_pad, int n_arms, LibDesc lib,
              double* __restrict__ G, double* __restrict__ b) {
  __shared__ double red[kBlock];
  const int a = blockIdx.x / lib.nE;
  const int e = blockIdx.x % lib.nE;
  if (a >= n_arms) return;
  double s = 0.0;
  for (int g = threadIdx.x; g < nblk; g += kBlock) s += partial[((int64_t)g * narm_pad + a) * kWave + e];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int off = kBlock / 2; off > 0; off >>= 1) {
    if (threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const int i = lib.ei[e], k = lib.ek[e];
    if (k >= 0) {
      G[((int64_t)a * lib.F + i) * lib.F + k] = red[0];
      G[((int64_t)a * lib.F + k) * lib.F + i] = red[0];
    } else {
      b[(int64_t)a * lib.F + i] = red[0];
    }
  }
}

// =============================================================================================
// STLSQ on Gram systems (pkpd/utils.py:213-327 semantics), one system per thread
// =============================================================================================
// Solve (G_SS + alpha I) c_S = b_S for the support mask `m` with the inactive rows/columns
// replaced by identity rows: the Cholesky factor stays block diagonal, so the active block
// performs exactly the operations of the reduced solve.  Returns false if not positive definite.
template <int F>
__device__ bool masked_cholesky_solve(const double (&g)[F][F], const double (&rhs)[F], unsigned m,
                                      double alpha, double (&c)[F]) {
  double l[F][F];
  bool ok = true;
#pragma unroll
  for (int i = 0; i < F; ++i) {
#pragma unroll
    for (int j = 0; j <= i; ++j) {
      const bool act = ((m >> i) & 1u) && ((m >> j) & 1u);
      double a = act ? g[i][j] : 0.0;
      if (i == j) a = ((m >> i) & 1u) ? a + alpha : 1.0;
#pragma unroll
      for (int q = 0; q < j; ++q) a -= l[i][q] * l[j][q];
      if (i == j) {
        if (!(a > 0.0)) {
          ok = false;
          a = 1e-300;
        }
        l[i][i] = sqrt(a);
      } else {
        l[i][j] = a / l[j][j];
      }
    }
  }
  double z[F];
#pragma unroll
  for (int i = 0; i < F; ++i) {
    double s = ((m >> i) & 1u) ? rhs[i] : 0.0;
#pragma unroll
    for (int q = 0; q < i; ++q) s -= l[i][q] * z[q];
    z[i] = s / l[i][i];
  }
#pragma unroll
  for (int i = F - 1; i >= 0; --i) {
    double s = z[i];
#pragma unroll
    for (int q = i + 1; q < F; ++q) s -= l[q][i] * c[q];
    c[i] = s / l[i][i];
  }
#pragma unroll
  for (int i = 0; i < F; ++i)
    if (!((m >> i) & 1u)) c[i] = 0.0;
  return ok;
}

template <int F>
__global__ void __launch_bounds__(kBlock)
stlsq_kernel(const double* __restrict__ G, const double* __restrict__ b, int64_t n_sys, double thr,
             double alpha, int max_iter, int unbias, double* __restrict__ coef,
             int8_t* __restrict__ mask, int32_t* __restrict__ iters) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_sys) return;
  double g[F][F], rhs[F], c[F];
#pragma unroll
  for (int i = 0; i < F; ++i) {
    rhs[i] = b[s * F + i];
    c[i] = 0.0;
#pragma unroll
    for (int j = 0; j < F; ++j) g[i][j] = G[(s * F + i) * F + j];
  }
  const unsigned all = (1u << F) - 1u;
  unsigned ind = all, prev = all;
  bool ok = true;
  int it = 0;
  for (int k = 0; k < max_iter; ++k) {
    it = k + 1;
    if (ind == 0u) {
#pragma unroll
      for (int i = 0; i < F; ++i) c[i] = 0.0;
      break;
    }
    ok &= masked_cholesky_solve<F>(g, rhs, ind, alpha, c);
    unsigned big = 0u;
#pragma unroll
    for (int i = 0; i < F; ++i) {
      if (fabs(c[i]) >= thr) big |= 1u << i;
      else c[i] = 0.0;
    }
    ind = big;
    unsigned pattern = 0u;
#pragma unroll
    for (int i = 0; i < F; ++i)
      if (c[i] != 0.0) pattern |= 1u << i;
    if (ind == all || pattern == prev) break;
    prev = pattern;
  }
  unsigned sup = 0u;
#pragma unroll
  for (int i = 0; i < F; ++i)
    if (fabs(c[i]) > 1e-14) sup |= 1u << i;
  if (unbias && sup) ok &= masked_cholesky_solve<F>(g, rhs, sup, 0.0, c);
#pragma unroll
  for (int i = 0; i < F; ++i) {
    coef[s * F + i] = c[i];
    if (mask) mask[s * F + i] = (int8_t)((sup >> i) & 1u);
  }
  if (iters) iters[s] = ok ? it : -1;
}

// =============================================================================================
// Batched rollout: lane = patient
// =============================================================================================
struct RolloutArgs {
  const double* y0;
  const double* u;
  const int8_t* arm;
  const double* coef;
  double* y;
  int64_t lda, ldy, coef_stride, N;
  int32_t T, substeps, A;
  double dt, drop;
};

template <int METHOD, int NARM, bool PERROW, int AVEC, int KT>
__global__ void __launch_bounds__(kBlock) rollout_kernel(RolloutArgs ra, LibDesc lib) {
  static_assert(KT == 32, "write-out mapping assumes 32-step tiles");
  constexpr int kYStride = KT + 1;           // doubles, odd -> conflict-free lane-per-row writes
  constexpr int kAStrideW = (KT + 4) / 4;    // arm row stride in dwords (odd)
  __shared__ double ysm[kWavesPerBlock * kWave * kYStride];
  __shared__ uint32_t asm_[kWavesPerBlock * kWave * kAStrideW];
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = threadIdx.x / kWave;
  double* yt = ysm + wid * (kWave * kYStride);
  uint32_t* at = asm_ + wid * (kWave * kAStrideW);
  uint8_t* at8 = reinterpret_cast<uint8_t*>(at);

  const int64_t p0 = ((int64_t)blockIdx.x * kWavesPerBlock + wid) * kWave;
  if (p0 >= ra.N) return;  // whole wave idle (no block-level sync below)
  const int64_t p = p0 + lane;
  const bool active = p < ra.N;

  // ---- prologue: f_a(y) = alpha_a + beta_a * y for this patient's statics ----
  double uu[INSITE_MAX_STATICS] = {0.0, 0.0, 0.0};
  if (active)
    for (int i = 0; i < lib.U; ++i) uu[i] = ra.u[p * lib.U + i];
  double alpha[NARM], beta[NARM];
  const double* cbase = ra.coef + (PERROW ? (active ? p : 0) * ra.coef_stride : 0);
#pragma unroll
  for (int a = 0; a < NARM; ++a) {
    alpha[a] = 0.0;
    beta[a] = 0.0;
    if (a >= ra.A) continue;  // padded arm slot (n_arms = 3 -> NARM = 4)
    for (int j = 0; j < lib.F; ++j) {
      const double c = cbase[a * lib.F + j];
      if (fabs(c) > ra.drop) {
        const double t = c * monomial(lib, j, uu);
        if (lib.ex[j] == 0) alpha[a] += t;
        else beta[a] += t;
      }
    }
  }
  double y = active ? ra.y0[p] : 0.0;
  const double h = ra.dt / (double)ra.substeps;
  const double h2 = 0.5 * h;
  const double h6 = h / 6.0;

  for (int t0 = 0; t0 < ra.T; t0 += KT) {
    // ---- stage arm[p0..p0+63][t0..t0+KT) (int8) into LDS ----
    {
      constexpr int LPR = KT / AVEC;
      constexpr int RPI = kWave / LPR;
      const int cl = (lane % LPR) * AVEC;
      const int64_t col = t0 + cl;
      uint32_t v[kWave / RPI];
#pragma unroll
      for (int it = 0; it < kWave / RPI; ++it) {
        const int64_t pr = p0 + it * RPI + lane / LPR;
        v[it] = 0u;
        if (pr < ra.N && col < ra.T) {
          if constexpr (AVEC == 4) v[it] = *reinterpret_cast<const uint32_t*>(ra.arm + pr * ra.lda + col);
          else v[it] = (uint8_t)ra.arm[pr * ra.lda + col];
        }
      }
      wave_lds_sync();
#pragma unroll
      for (int it = 0; it < kWave / RPI; ++it) {
        const int r = it * RPI + lane / LPR;
        if constexpr (AVEC == 4) at[r * kAStrideW + cl / 4] = v[it];
        else at8[r * kAStrideW * 4 + cl] = (uint8_t)v[it];
      }
      wave_lds_sync();
    }
    // ---- integrate KT observation intervals ----
    uint32_t a4 = 0u;
#pragma unroll
    for (int i = 0; i < KT; ++i) {
      if ((i & 3) == 0) a4 = at[lane * kAStrideW + i / 4];
      if (t0 + i < ra.T) {
        const int a = (int)((a4 >> (8 * (i & 3))) & 0xffu);
        double al = alpha[0], be = beta[0];
#pragma unroll
        for (int aa = 1; aa < NARM; ++aa) {
          al = (a == aa) ? alpha[aa] : al;
          be = (a == aa) ? beta[aa] : be;
        }
        if constexpr (METHOD == INSITE_METHOD_EULER) {
          for (int s = 0; s < ra.substeps; ++s) {
            const double f = fma(be, y, al);
            y = fma(f, h, y);
          }
        } else {
          for (int s = 0; s < ra.substeps; ++s) {
            const double k1 = fma(be, y, al);
            const double k2 = fma(be, fma(h2, k1, y), al);
            const double k3 = fma(be, fma(h2, k2, y), al);
            const double k4 = fma(be, fma(h, k3, y), al);
            y = fma(h6, (k1 + 2.0 * k2) + (2.0 * k3 + k4), y);
          }
        }
        yt[lane * kYStride + i] = y;
      }
    }
    wave_lds_sync();
    // ---- write-out: two 256-byte row segments per wave instruction ----
#pragma unroll
    for (int j = 0; j < kWave / 2; ++j) {
      const int r = 2 * j + (lane >> 5);
      const int c = lane & 31;
      const int64_t pr = p0 + r;
      const int tc = t0 + c;
      const double v = yt[r * kYStride + c];
      if (pr < ra.N && tc < ra.T) ra.y[pr * ra.ldy + tc] = v;
    }
    wave_lds_sync();
  }
}

// =============================================================================================
// Masked squared-error sums (metrics)
// =============================================================================================
__global__ void __launch_bounds__(kBlock)
sse_kernel(const double* __restrict__ pred, int64_t ldp, double scale, double shift,
           const double* __restrict__ target, const double* __restrict__ active, int64_t n_rows,
           int T, double* __restrict__ part /* [grid][2T+2] */) {
  __shared__ double red[2][kBlock];
  const int W = 2 * T + 2;
  double* out = part + (int64_t)blockIdx.x * W;
  double last_s = 0.0, last_c = 0.0;
  for (int t = threadIdx.x; t < T; t += kBlock) {
    double s = 0.0, c = 0.0;
    for (int64_t r = blockIdx.x; r < n_rows; r += gridDim.x) {
      const double av = active[r * T + t];
      const double d = fma(pred[r * ldp + t], scale, shift) - target[r * T + t];
      const double e = d * d * av;
      s += e;
      c += av;
      const double an = (t + 1 < T) ? active[r * T + t + 1] : 0.0;
      const double lw = av - an;  // reference: active - shift(active)  (time_varying_model.py:267-268)
      last_s += d * d * lw;
      last_c += lw;
    }
    out[t] = s;
    out[T + t] = c;
  }
  red[0][threadIdx.x] = last_s;
  red[1][threadIdx.x] = last_c;
  __syncthreads();
  for (int off = kBlock / 2; off > 0; off >>= 1) {
    if (threadIdx.x < off) {
      red[0][threadIdx.x] += red[0][threadIdx.x + off];
      red[1][threadIdx.x] += red[1][threadIdx.x + off];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[2 * T] = red[0][0];
    out[2 * T + 1] = red[1][0];
  }
}

__global__ void __launch_bounds__(kBlock)
sse_finalize(const double* __restrict__ part, int nblk, int T, double* __restrict__ per_step,
             double* __restrict__ per_cnt, double* __restrict__ last) {
  const int W = 2 * T + 2;
  for (int c = blockIdx.x * kBlock + threadIdx.x; c < W; c += gridDim.x * kBlock) {
    double s = 0.0;
    for (int g = 0; g < nblk; ++g) s += part[(int64_t)g * W + c];
    if (c < T) per_step[c] = s;
    else if (c < 2 * T) per_cnt[c - T] = s;
    else last[c - 2 * T] = s;
  }
}

// =============================================================================================
// host helpers
// =============================================================================================
int build_lib(const int8_t* exps, int32_t F, int32_t U, LibDesc* lib) {
  if (!exps || F < 1 || F > INSITE_MAX_TERMS || U < 0 || U > INSITE_MAX_STATICS) return INSITE_E_INVALID_ARG;
  std::memset(lib, 0, sizeof(*lib));
  lib->F = F;
  lib->U = U;
  for (int j = 0; j < F; ++j) {
    const int8_t ex = exps[j * (1 + U)];
    if (ex < 0) return INSITE_E_INVALID_ARG;
    if (ex > INSITE_MAX_STATE_DEGREE) return INSITE_E_UNSUPPORTED;
    lib->ex[j] = ex;
    for (int i = 0; i < U; ++i) {
      const int8_t e = exps[j * (1 + U) + 1 + i];
      if (e < 0 || e > 8) return INSITE_E_INVALID_ARG;
      lib->eu[j][i] = e;
    }
  }
  int e = 0;
  for (int i = 0; i < F; ++i)
    for (int k = i; k < F; ++k) {
      lib->ei[e] = (int8_t)i;
      lib->ek[e] = (int8_t)k;
      ++e;
    }
  lib->nG = e;
  for (int i = 0; i < F; ++i) {
    lib->ei[e] = (int8_t)i;
    lib->ek[e] = -1;
    ++e;
  }
  lib->nE = e;
  return e <= kMaxEntries ? INSITE_OK : INSITE_E_UNSUPPORTED;
}

inline int narm_pad(int n_arms) { return n_arms <= 1 ? 1 : (n_arms <= 2 ? 2 : 4); }

inline int gram_grid(int64_t N) {
  const int64_t tiles = (N + kWave - 1) / kWave;
  int64_t g = (tiles + kWavesPerBlock - 1) / kWavesPerBlock;
  if (g < 1) g = 1;
  if (g > kGramMaxBlocks) g = kGramMaxBlocks;
  return (int)g;
}

inline int sse_grid(int64_t n_rows) {
  int64_t g = (n_rows + 63) / 64;
  if (g < 1) g = 1;
  if (g > 1024) g = 1024;
  return (int)g;
}

inline int32_t launch_status() { return hipGetLastError() == hipSuccess ? INSITE_OK : INSITE_E_HIP; }

template <int NARM>
void launch_gram(bool vec2, bool smooth, dim3 grid, hipStream_t st, const double* x, int64_t ldx,
                 const double* u, const int8_t* arm, const int32_t* rows, int64_t N, double inv_dt,
                 const LibDesc& lib, double* part) {
  constexpr int KT = 32;
  if (vec2) {
    if (smooth) gram_kernel<KT, 2, NARM, true><<<grid, kBlock, 0, st>>>(x, ldx, u, arm, rows, N, inv_dt, lib, part);
    else gram_kernel<KT, 2, NARM, false><<<grid, kBlock, 0, st>>>(x, ldx, u, arm, rows, N, inv_dt, lib, part);
  } else {
    if (smooth) gram_kernel<KT, 1, NARM, true><<<grid, kBlock, 0, st>>>(x, ldx, u, arm, rows, N, inv_dt, lib, part);
    else gram_kernel<KT, 1, NARM, false><<<grid, kBlock, 0, st>>>(x, ldx, u, arm, rows, N, inv_dt, lib, part);
  }
}

template <int METHOD, int NARM, bool PERROW>
void launch_rollout_a(bool avec4, dim3 grid, hipStream_t st, const RolloutArgs& ra, const LibDesc& lib) {
  if (avec4) rollout_kernel<METHOD, NARM, PERROW, 4, 32><<<grid, kBlock, 0, st>>>(ra, lib);
  else rollout_kernel<METHOD, NARM, PERROW, 1, 32><<<grid, kBlock, 0, st>>>(ra, lib);
}

template <int METHOD, int NARM>
void launch_rollout_p(bool perrow, bool avec4, dim3 grid, hipStream_t st, const RolloutArgs& ra,
                      const LibDesc& lib) {
  if (perrow) launch_rollout_a<METHOD, NARM, true>(avec4, grid, st, ra, lib);
  else launch_rollout_a<METHOD, NARM, false>(avec4, grid, st, ra, lib);
}

template <int METHOD>
void launch_rollout_m(int narm, bool perrow, bool avec4, dim3 grid, hipStream_t st,
                      const RolloutArgs& ra, const LibDesc& lib) {
  if (narm == 1) launch_rollout_p<METHOD, 1>(perrow, avec4, grid, st, ra, lib);
  else if (narm == 2) launch_rollout_p<METHOD, 2>(perrow, avec4, grid, st, ra, lib);
  else launch_rollout_p<METHOD, 4>(perrow, avec4, grid, st, ra, lib);
}

}  // namespace

// =============================================================================================
// C ABI
// =============================================================================================
extern "C" {

int32_t insite_abi_version(void) { return INSITE_ABI_VERSION; }

const char* insite_strerror(int32_t code) {
  switch (code) {
    case INSITE_OK: return "ok";
    case INSITE_E_INVALID_ARG: return "invalid argument";
    case INSITE_E_UNSUPPORTED: return "unsupported configuration for this ABI version";
    case INSITE_E_WORKSPACE: return "workspace too small";
    case INSITE_E_HIP: return "HIP launch error";
    default: return "unknown error";
  }
}

int32_t insite_poly_library(int32_t n_statics, int32_t degree, int32_t interaction_only,
                            int8_t* exps_out, int32_t max_terms, int32_t* n_terms) {
  if (n_statics < 0 || n_statics > INSITE_MAX_STATICS || degree < 0 || degree > 8 || !exps_out ||
      !n_terms)
    return INSITE_E_INVALID_ARG;
  const int n_in = 1 + n_statics;
  int count = 0;
  // enumerate combinations (with replacement unless interaction_only) of input indices, by
  // degree, in lexicographic (itertools) order
  for (int deg = 0; deg <= degree; ++deg) {
    int idx[16];
    if (deg > 16) return INSITE_E_UNSUPPORTED;
    for (int q = 0; q < deg; ++q) idx[q] = interaction_only ? q : 0;
    if (interaction_only && deg > n_in) break;
    while (true) {
      if (count >= max_terms) return INSITE_E_UNSUPPORTED;
      int8_t* row = exps_out + (int64_t)count * n_in;
      for (int q = 0; q < n_in; ++q) row[q] = 0;
      for (int q = 0; q < deg; ++q) row[idx[q]] += 1;
      ++count;
      // next combination
      int q = deg - 1;
      if (interaction_only) {
        while (q >= 0 && idx[q] == n_in - deg + q) --q;
        if (q < 0) break;
        ++idx[q];
        for (int r = q + 1; r < deg; ++r) idx[r] = idx[r - 1] + 1;
      } else {
        while (q >= 0 && idx[q] == n_in - 1) --q;
        if (q < 0) break;
        ++idx[q];
        for (int r = q + 1; r < deg; ++r) idx[r] = idx[q];
      }
    }
  }
  *n_terms = count;
  return INSITE_OK;
}

size_t insite_gram_workspace_bytes(int64_t n_patients, int32_t n_arms, int32_t n_terms) {
  (void)n_terms;
  if (n_patients < 0 || n_arms < 1 || n_arms > INSITE_MAX_ARMS) return 0;
  return (size_t)gram_grid(n_patients) * (size_t)narm_pad(n_arms) * kWave * sizeof(double);
}

int32_t insite_gram_f64(const double* x, int64_t ldx, const double* u, const int8_t* arm,
                        const int32_t* rows, int64_t n_patients, int32_t n_statics, int32_t n_arms,
                        const int8_t* exps, int32_t n_terms, int32_t fd_kind, double dt,
                        double* G_out, double* b_out, void* workspace, size_t workspace_bytes,
                        void* stream) {
  if (n_patients < 0 || !G_out || !b_out || n_arms < 1 || n_arms > INSITE_MAX_ARMS || ldx < 1 ||
      !(dt > 0.0))
    return INSITE_E_INVALID_ARG;
  if (n_patients > 0 && (!x || !arm || !rows || (n_statics > 0 && !u))) return INSITE_E_INVALID_ARG;
  if (fd_kind != INSITE_FD_SMOOTHED4 && fd_kind != INSITE_FD_ORDER4) return INSITE_E_UNSUPPORTED;
  LibDesc lib;
  int32_t st = build_lib(exps, n_terms, n_statics, &lib);
  if (st != INSITE_OK) return st;
  if (workspace_bytes < insite_gram_workspace_bytes(n_patients, n_arms, n_terms) || !workspace)
    return INSITE_E_WORKSPACE;
  hipStream_t hs = reinterpret_cast<hipStream_t>(stream);
  const int grid = gram_grid(n_patients);
  const int na = narm_pad(n_arms);
  double* part = static_cast<double*>(workspace);
  const bool vec2 = (ldx % 2 == 0) && ((reinterpret_cast<uintptr_t>(x) & 15u) == 0);
  const bool smooth = fd_kind == INSITE_FD_SMOOTHED4;
  const double inv_dt = 1.0 / dt;
  if (na == 1) launch_gram<1>(vec2, smooth, dim3(grid), hs, x, ldx, u, arm, rows, n_patients, inv_dt, lib, part);
  else if (na == 2) launch_gram<2>(vec2, smooth, dim3(grid), hs, x, ldx, u, arm, rows, n_patients, inv_dt, lib, part);
  else launch_gram<4>(vec2, smooth, dim3(grid), hs, x, ldx, u, arm, rows, n_patients, inv_dt, lib, part);
  st = launch_status();
  if (st != INSITE_OK) return st;
  gram_finalize<<<dim3(n_arms * lib.nE), kBlock, 0, hs>>>(part, grid, na, n_arms, lib, G_out, b_out);
  return launch_status();
}

int32_t insite_stlsq_f64(const double* G, const double* b, int64_t n_sys, int32_t n_terms,
                         double threshold, double alpha, int32_t max_iter, int32_t unbias,
                         double* coef_out, int8_t* mask_out, int32_t* iters_out, void* stream) {
  if (n_sys < 0 || max_iter < 0 || !(threshold >= 0.0) || !(alpha >= 0.0)) return INSITE_E_INVALID_ARG;
  if (n_sys == 0) return INSITE_OK;
  if (!G || !b || !coef_out) return INSITE_E_INVALID_ARG;
  hipStream_t hs = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid((unsigned)((n_sys + kBlock - 1) / kBlock));
  switch (n_terms) {
#define INSITE_STLSQ_CASE(FF)                                                                   \
  case FF:                                                                                      \
    stlsq_kernel<FF><<<grid, kBlock, 0, hs>>>(G, b, n_sys, threshold, alpha, max_iter, unbias,  \
                                              coef_out, mask_out, iters_out);                   \
    break;
    INSITE_STLSQ_CASE(1)
    INSITE_STLSQ_CASE(2)
    INSITE_STLSQ_CASE(3)
    INSITE_STLSQ_CASE(4)
    INSITE_STLSQ_CASE(5)
    INSITE_STLSQ_CASE(6)
    INSITE_STLSQ_CASE(7)
    INSITE_STLSQ_CASE(8)
    INSITE_STLSQ_CASE(9)
#undef INSITE_STLSQ_CASE
    default:
      return INSITE_E_UNSUPPORTED;
  }
  return launch_status();
}

int32_t insite_rollout_f64(const double* y0, const double* u, const int8_t* arm, int64_t ld_arm,
                           const double* coef, int64_t coef_row_stride, const int8_t* exps,
                           int32_t n_terms, int64_t n_rows, int32_t T, int32_t n_statics,
                           int32_t n_arms, double dt, int32_t method, int32_t substeps,
                           double drop_below, double* y_out, int64_t ld_y, void* stream) {
  if (n_rows < 0 || T < 0 || n_arms < 1 || n_arms > INSITE_MAX_ARMS || substeps < 1 ||
      !(dt >= 0.0) || ld_arm < T || ld_y < T || coef_row_stride < 0)
    return INSITE_E_INVALID_ARG;
  if (method != INSITE_METHOD_EULER && method != INSITE_METHOD_RK4) return INSITE_E_UNSUPPORTED;
  if (n_rows == 0 || T == 0) return INSITE_OK;
  if (!y0 || !arm || !coef || !y_out || (n_statics > 0 && !u)) return INSITE_E_INVALID_ARG;
  LibDesc lib;
  int32_t st = build_lib(exps, n_terms, n_statics, &lib);
  if (st != INSITE_OK) return st;
  if (coef_row_stride != 0 && coef_row_stride < (int64_t)n_arms * n_terms) return INSITE_E_INVALID_ARG;
  RolloutArgs ra;
  ra.y0 = y0;
  ra.u = u;
  ra.arm = arm;
  ra.coef = coef;
  ra.y = y_out;
  ra.lda = ld_arm;
  ra.ldy = ld_y;
  ra.coef_stride = coef_row_stride;
  ra.N = n_rows;
  ra.T = T;
  ra.substeps = substeps;
  ra.A = n_arms;
  ra.dt = dt;
  ra.drop = drop_below;
  const bool avec4 = (ld_arm % 4 == 0) && ((reinterpret_cast<uintptr_t>(arm) & 3u) == 0);
  const int64_t waves = (n_rows + kWave - 1) / kWave;
  const dim3 grid((unsigned)((waves + kWavesPerBlock - 1) / kWavesPerBlock));
  hipStream_t hs = reinterpret_cast<hipStream_t>(stream);
  const bool perrow = coef_row_stride != 0;
  const int na = narm_pad(n_arms);
  if (method == INSITE_METHOD_EULER) launch_rollout_m<INSITE_METHOD_EULER>(na, perrow, avec4, grid, hs, ra, lib);
  else launch_rollout_m<INSITE_METHOD_RK4>(na, perrow, avec4, grid, hs, ra, lib);
  return launch_status();
}

size_t insite_masked_sse_workspace_bytes(int64_t n_rows, int32_t T) {
  if (n_rows < 0 || T < 0) return 0;
  return (size_t)sse_grid(n_rows) * (size_t)(2 * T + 2) * sizeof(double);
}

int32_t insite_masked_sse_f64(const double* pred, int64_t ld_pred, double scale, double shift,
                              const double* target, const double* active, int64_t n_rows,
                              int32_t T, double* per_step_out, double* per_step_cnt_out,
                              double* last_out, void* workspace, size_t workspace_bytes,
                              void* stream) {
  if (n_rows < 0 || T < 1 || ld_pred < T || !per_step_out || !per_step_cnt_out || !last_out)
    return INSITE_E_INVALID_ARG;
  if (n_rows > 0 && (!pred || !target || !active)) return INSITE_E_INVALID_ARG;
  if (!workspace || workspace_bytes < insite_masked_sse_workspace_bytes(n_rows, T)) return INSITE_E_WORKSPACE;
  hipStream_t hs = reinterpret_cast<hipStream_t>(stream);
  const int grid = sse_grid(n_rows);
  double* part = static_cast<double*>(workspace);
  sse_kernel<<<dim3(grid), kBlock, 0, hs>>>(pred, ld_pred, scale, shift, target, active, n_rows, T, part);
  int32_t st = launch_status();
  if (st != INSITE_OK) return st;
  const int W = 2 * T + 2;
  sse_finalize<<<dim3((W + kBlock - 1) / kBlock), kBlock, 0, hs>>>(part, grid, T, per_step_out,
                                                                    per_step_cnt_out, last_out);
  return launch_status();
}

}  // extern "C"
