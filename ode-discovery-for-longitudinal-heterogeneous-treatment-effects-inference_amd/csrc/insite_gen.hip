// insite_gen.hip — the general one-state library path on MI355X (gfx950): libraries whose columns
// are not affine in the state and libraries with per-step treatment inputs.
//
//   * the degree-4 ablation library (reference run.py:208 ABLATION_MORE_COMPLEX_BASIS_FUNCTIONS ->
//     PolynomialLibrary(degree=4, interaction_only=False), sindy.py:185-186): x up to x^4, F = 35 over
//     (x0, u0, u1);
//   * the joint ("one ODE") model (run.py:198-201 ABLATION_ONE_ODE -> joint_model + multilabel
//     treatments; DE format pkpd/utils.py:486-497, 639-672): ONE regression whose library inputs are
//     (x0, the per-step binary treatment(s), the statics), F = 11 for EQ_4 / cancer_sim.
//
// Kernels:
//   gen_deriv_kernel     element (step k, patient p): x_dot[k][p] by the reference's differentiation
//                        method (savgol(5,3) + one-sided/central FD4, FD4, FD1, savgol(2,1) + FD1) into a
//                        time-major scratch array (coalesced writes; x read in either layout).
//   gen_moments_kernel   lane = patient: per treatment combination c of the step inputs the power
//                        moments S[c][e] = sum x^e (e <= 2D) and T[c][e] = sum x_dot x^e (e <= D) over the
//                        patient's rows.  A column is m_j(u) * (input bits)^tau_j * x^{e_j}, so
//                        Theta_p^T Theta_p and Theta_p^T x_dot_p are fixed linear maps of these moments.
//   gen_contract_kernel  thread = Gram/moment entry (group g, columns i <= k, or b_i), block row = patient
//                        chunk: sum over the chunk's patients of m_i m_k S[c][e_i + e_k] (+ b) staged
//                        through LDS, one partial per (chunk, entry).
//   gen_finalize_kernel  fixed-order sum of the chunk partials -> G [n_groups, F, F], b [n_groups, F].
//   gen_stlsq_wave_kernel one wavefront per system: STLSQ (pkpd/utils.py:213-327 semantics) with a
//                        lane-per-row masked Cholesky in LDS, F <= 64 (64-bit lane masks).
//   gen_rollout_kernel   lane = patient: stage-evaluated Euler / RK4 of the polynomial RHS
//                        f_a(y) = sum_e P_a[e] y^e (Horner, e <= 4) with the per-step arm; the affine
//                        interval propagator of insite_hip.hip does not apply when D > 1.
// This path is memory-light (the moments are ~14 doubles per patient) and not a BASELINE bench
// configuration; it exists so the reference's ablation models run on the GPU, parity-tested against
// oracle/insite_ref.py (which evaluates Theta explicitly).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstring>

#include "insite_common.h"

namespace {

constexpr int kGenMaxF = 64;
constexpr int kGenMaxDeg = 4;
constexpr int kGenMaxIn = 2;  // binary per-step inputs: combinations NC = 1 << n_in <= 4
constexpr int kGenMaxNC = 1 << kGenMaxIn;
constexpr int kGenMaxU = INSITE_MAX_STATICS;
constexpr int kGenNS = 2 * kGenMaxDeg + 1;  // S moments per combination
constexpr int kGenNT = kGenMaxDeg + 1;      // T moments per combination
constexpr int kGenHdr = 1 + kGenMaxU;       // record header: group, u[0..2]
constexpr int kGenRec = kGenHdr + kGenMaxNC * (kGenNS + kGenNT);  // 60 doubles per patient
constexpr int kGenChunks = 256;             // patient chunks (fixed: deterministic reduction order)
constexpr int kGenTile = 32;                // patients staged per LDS tile in the contraction

struct GenLib {
  int32_t F, U, n_in, D, nG, nEg;
  int8_t ex[kGenMaxF];             // exponent of x
  int8_t tin[kGenMaxF];            // bitmask of the step inputs with exponent >= 1 (binary inputs)
  int8_t eu[kGenMaxF][kGenMaxU];   // exponents of the statics
};

// ---------------------------------------------------------------------------------------------
// derivative
// ---------------------------------------------------------------------------------------------
struct XView {
  const double* x;
  int64_t sp, sk;  // x(p, k) = x[p * sp + k * sk]
  __device__ __forceinline__ double at(int64_t p, int k) const { return x[p * sp + (int64_t)k * sk]; }
};

// savgol_filter(window 5, polyorder 3, mode='interp') at position j of a row of L >= 5 samples
__device__ double sg53_at(const XView& v, int64_t p, int j, int L) {
  if (j <= 1) {
    const double a = v.at(p, 0), b = v.at(p, 1), c = v.at(p, 2), d = v.at(p, 3), e = v.at(p, 4);
    return j == 0 ? sg_pos0(a, b, c, d, e) : sg_pos1(a, b, c, d, e);
  }
  if (j >= L - 2) {
    const double a = v.at(p, L - 5), b = v.at(p, L - 4), c = v.at(p, L - 3), d = v.at(p, L - 2), e = v.at(p, L - 1);
    return j == L - 2 ? sg_pos3(a, b, c, d, e) : sg_pos4(a, b, c, d, e);
  }
  return sg_interior(v.at(p, j - 2), v.at(p, j - 1), v.at(p, j), v.at(p, j + 1), v.at(p, j + 2));
}

// savgol_filter(window 2, polyorder 1): (x_i + x_{i+1}) / 2, the end samples unchanged
__device__ double sg21_at(const XView& v, int64_t p, int j, int L) {
  if (j == 0 || j == L - 1) return v.at(p, j);
  return 0.5 * (v.at(p, j) + v.at(p, j + 1));
}

// the smoothed (or raw) series the differentiation method sees
__device__ __forceinline__ double series_at(const XView& v, int64_t p, int j, int L, int fd) {
  if (fd == INSITE_FD_SMOOTHED4) return sg53_at(v, p, j, L);
  if (fd == INSITE_FD_SMOOTHED1) return sg21_at(v, p, j, L);
  return v.at(p, j);
}

__global__ void __launch_bounds__(kBlock)
gen_deriv_kernel(XView xv, const int32_t* __restrict__ rows, int n_steps, int64_t N, int fd, int min_rows, double inv_dt,
                 double* __restrict__ d, int64_t ldd) {
  const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const int k = blockIdx.y;
  if (p >= N) return;
  int L = rows[p] < n_steps ? rows[p] : n_steps;
  if (L < min_rows || k >= L) return;
  double r;
  if (fd == INSITE_FD_SMOOTHED4 || fd == INSITE_FD_ORDER4) {
    // pysindy FiniteDifference(order=4): central 5-point interior, one-sided 5-point at the 2 + 2 ends
    if (k <= 1) {
      const double a = series_at(xv, p, 0, L, fd), b = series_at(xv, p, 1, L, fd), c = series_at(xv, p, 2, L, fd),
                   dd = series_at(xv, p, 3, L, fd), e = series_at(xv, p, 4, L, fd);
      r = (k == 0 ? fd_pos0(a, b, c, dd, e) : fd_pos1(a, b, c, dd, e)) * inv_dt;
    } else if (k >= L - 2) {
      const double a = series_at(xv, p, L - 5, L, fd), b = series_at(xv, p, L - 4, L, fd),
                   c = series_at(xv, p, L - 3, L, fd), dd = series_at(xv, p, L - 2, L, fd),
                   e = series_at(xv, p, L - 1, L, fd);
      r = (k == L - 2 ? fd_pos3(a, b, c, dd, e) : fd_pos4(a, b, c, dd, e)) * inv_dt;
    } else {
      r = fd_interior(series_at(xv, p, k - 2, L, fd), series_at(xv, p, k - 1, L, fd), 0.0,
                      series_at(xv, p, k + 1, L, fd), series_at(xv, p, k + 2, L, fd)) * inv_dt;
    }
  } else {
    // FiniteDifference(order=1): forward difference, backward at the last sample
    const int k0 = k < L - 1 ? k : L - 2;
    r = (series_at(xv, p, k0 + 1, L, fd) - series_at(xv, p, k0, L, fd)) * inv_dt;
  }
  d[(int64_t)k * ldd + p] = r;
}

// ---------------------------------------------------------------------------------------------
// per-patient moments
// ---------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(kBlock)
gen_moments_kernel(XView xv, const double* __restrict__ d, int64_t ldd, const int8_t* __restrict__ sin_, int64_t in_sp,
                   int64_t in_sk, const int8_t* __restrict__ group, const double* __restrict__ u, int U,
                   const int32_t* __restrict__ rows, int n_steps, int64_t N, int D, int n_in, int min_rows,
                   double* __restrict__ rec) {
  const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (p >= N) return;
  int L = rows[p] < n_steps ? rows[p] : n_steps;
  const bool on = L >= min_rows;
  double S[kGenMaxNC][kGenNS], T[kGenMaxNC][kGenNT];
#pragma unroll
  for (int c = 0; c < kGenMaxNC; ++c) {
#pragma unroll
    for (int e = 0; e < kGenNS; ++e) S[c][e] = 0.0;
#pragma unroll
    for (int e = 0; e < kGenNT; ++e) T[c][e] = 0.0;
  }
  const int cmask = (1 << n_in) - 1;
  if (on) {
    for (int k = 0; k < L; ++k) {
      const double x = xv.at(p, k);
      const double dk = d[(int64_t)k * ldd + p];
      const int code = n_in ? ((int)sin_[p * in_sp + (int64_t)k * in_sk] & cmask) : 0;
      double pw[kGenNS];
      pw[0] = 1.0;
#pragma unroll
      for (int e = 1; e < kGenNS; ++e) pw[e] = pw[e - 1] * x;
#pragma unroll
      for (int c = 0; c < kGenMaxNC; ++c) {
        const double w = (c == code) ? 1.0 : 0.0;  // compile-time combination slots: no dynamic indexing
#pragma unroll
        for (int e = 0; e < kGenNS; ++e) S[c][e] = fma(w, e <= 2 * D ? pw[e] : 0.0, S[c][e]);
#pragma unroll
        for (int e = 0; e < kGenNT; ++e) T[c][e] = fma(w * dk, e <= D ? pw[e] : 0.0, T[c][e]);
      }
    }
  }
  double* r = rec + p * kGenRec;
  r[0] = on ? (double)(group ? group[p] : 0) : -1.0;
#pragma unroll
  for (int t = 0; t < kGenMaxU; ++t) r[1 + t] = t < U ? u[p * U + t] : 0.0;
#pragma unroll
  for (int c = 0; c < kGenMaxNC; ++c) {
#pragma unroll
    for (int e = 0; e < kGenNS; ++e) r[kGenHdr + c * (kGenNS + kGenNT) + e] = S[c][e];
#pragma unroll
    for (int e = 0; e < kGenNT; ++e) r[kGenHdr + c * (kGenNS + kGenNT) + kGenNS + e] = T[c][e];
  }
}

// Treatment-segment moments (the cancer_sim / EQ_5 DE format, pkpd/utils.py:433-462, 607-637, with a general
// library: the degree-4 ablation on those datasets, sindy.py:185-186 + run.py:96-104, 208).  Lane = patient,
// one walk over its samples j < L = seq_len: sample j (arm a_j) is a row (x_j, d_j), d_j the forward
// difference of its segment ((xs_{j+1} - xs_j) / dt); when sample j + 1 closes the segment (j + 1 = L or
// a_{j+1} != a_j) it is a row of the same arm with the backward difference d_j -- the index form of the
// reference's walk (oracle/segments_ref.segment_bounds).  SMOOTH1: savgol(2, 1) inside a segment,
// xs_i = (x_i + x_{i+1}) / 2 except at its first and last sample (raw); the library takes the raw x.
// Arm a's power moments go to record slot a (the contraction reads slot g for group g).
__global__ void __launch_bounds__(kBlock)
gen_seg_moments_kernel(XView xv, const int8_t* __restrict__ arm, int64_t asp, int64_t ask,
                       const int32_t* __restrict__ seq_len, int n_steps, const double* __restrict__ u, int U, int64_t N,
                       int D, int n_arms, int smooth1, double inv_dt, double* __restrict__ rec) {
  const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (p >= N) return;
  int L = seq_len[p];
  if (L > n_steps - 1) L = n_steps - 1;
  if (L < 0) L = 0;
  double S[kGenMaxNC][kGenNS], T[kGenMaxNC][kGenNT];
#pragma unroll
  for (int c = 0; c < kGenMaxNC; ++c) {
#pragma unroll
    for (int e = 0; e < kGenNS; ++e) S[c][e] = 0.0;
#pragma unroll
    for (int e = 0; e < kGenNT; ++e) T[c][e] = 0.0;
  }
  int aprev = -1;
  for (int j = 0; j < L; ++j) {
    const int aj = (int)arm[p * asp + (int64_t)j * ask];
    const bool start = j == 0 || aj != aprev;
    const bool end = j + 1 == L || (int)arm[p * asp + (int64_t)(j + 1) * ask] != aj;
    aprev = aj;
    const double xj = xv.at(p, j), xj1 = xv.at(p, j + 1);
    double xs0 = xj, xs1 = xj1;
    if (smooth1) {
      if (!start) xs0 = 0.5 * (xj + xj1);
      if (!end) xs1 = 0.5 * (xj1 + xv.at(p, j + 2));
    }
    const double dj = (xs1 - xs0) * inv_dt;
    if (aj < 0 || aj >= n_arms) continue;
#pragma unroll
    for (int r = 0; r < 2; ++r) {  // the sample, then (segment end) the closing sample
      if (r == 1 && !end) break;
      const double x = r == 0 ? xj : xj1;
      double pw[kGenNS];
      pw[0] = 1.0;
#pragma unroll
      for (int e = 1; e < kGenNS; ++e) pw[e] = pw[e - 1] * x;
#pragma unroll
      for (int c = 0; c < kGenMaxNC; ++c) {
        const double w = (c == aj) ? 1.0 : 0.0;  // compile-time arm slots: no dynamic indexing
#pragma unroll
        for (int e = 0; e < kGenNS; ++e) S[c][e] = fma(w, e <= 2 * D ? pw[e] : 0.0, S[c][e]);
#pragma unroll
        for (int e = 0; e < kGenNT; ++e) T[c][e] = fma(w * dj, e <= D ? pw[e] : 0.0, T[c][e]);
      }
    }
  }
  double* r = rec + p * kGenRec;
  r[0] = L >= 1 ? 0.0 : -1.0;
#pragma unroll
  for (int t = 0; t < kGenMaxU; ++t) r[1 + t] = t < U ? u[p * U + t] : 0.0;
#pragma unroll
  for (int c = 0; c < kGenMaxNC; ++c) {
#pragma unroll
    for (int e = 0; e < kGenNS; ++e) r[kGenHdr + c * (kGenNS + kGenNT) + e] = S[c][e];
#pragma unroll
    for (int e = 0; e < kGenNT; ++e) r[kGenHdr + c * (kGenNS + kGenNT) + kGenNS + e] = T[c][e];
  }
}

// ---------------------------------------------------------------------------------------------
// contraction + finalize
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ double static_mono(const GenLib& lib, int j, const double* uu) {
  double m = 1.0;
  for (int t = 0; t < lib.U; ++t)
    for (int e = 0; e < lib.eu[j][t]; ++e) m *= uu[t];
  return m;
}

// entry e of a group: (i, k) of the upper triangle in row-major order, then b_i (k = -1)
__device__ __forceinline__ void decode_entry(const GenLib& lib, int e, int& i, int& k) {
  if (e >= lib.nG) {
    i = e - lib.nG;
    k = -1;
    return;
  }
  i = 0;
  int rem = e;
  while (rem >= lib.F - i) {
    rem -= lib.F - i;
    ++i;
  }
  k = i + rem;
}

__global__ void __launch_bounds__(kBlock)
gen_contract_kernel(const double* __restrict__ rec, int64_t N, GenLib lib, int n_groups, int64_t chunk,
                    int slot_groups, double* __restrict__ part) {
  __shared__ double srec[kGenTile * kGenRec];
  __shared__ double smon[kGenTile * kGenMaxF];
  const int NE = n_groups * lib.nEg;
  const int E = blockIdx.x * kBlock + threadIdx.x;
  const bool ent = E < NE;
  int g = 0, i = 0, k = -1;
  if (ent) {
    g = E / lib.nEg;
    decode_entry(lib, E - g * lib.nEg, i, k);
  }
  const int NC = 1 << lib.n_in;
  const int eik = ent ? (k >= 0 ? lib.ex[i] + lib.ex[k] : lib.ex[i]) : 0;
  const int need = ent ? (k >= 0 ? (lib.tin[i] | lib.tin[k]) : lib.tin[i]) : 0;  // inputs that must be on
  const int moff = k >= 0 ? eik : kGenNS + eik;
  double acc = 0.0;
  const int64_t p_lo = (int64_t)blockIdx.y * chunk;
  const int64_t p_hi = p_lo + chunk < N ? p_lo + chunk : N;
  for (int64_t t0 = p_lo; t0 < p_hi; t0 += kGenTile) {
    const int nq = (int)(p_hi - t0 < kGenTile ? p_hi - t0 : kGenTile);
    __syncthreads();
    for (int q = threadIdx.x; q < nq * kGenRec; q += kBlock) srec[q] = rec[t0 * kGenRec + q];
    __syncthreads();
    for (int q = threadIdx.x; q < nq * lib.F; q += kBlock) {
      const int pq = q / lib.F, j = q - pq * lib.F;
      smon[pq * kGenMaxF + j] = static_mono(lib, j, srec + pq * kGenRec + 1);
    }
    __syncthreads();
    if (ent) {
      for (int q = 0; q < nq; ++q) {
        const double* r = srec + q * kGenRec;
        if (slot_groups ? (r[0] < 0.0) : ((int)r[0] != g)) continue;
        const double m = smon[q * kGenMaxF + i] * (k >= 0 ? smon[q * kGenMaxF + k] : 1.0);
        double s = 0.0;
        if (slot_groups) {  // segment records: group g's moments sit in slot g
          s = r[kGenHdr + g * (kGenNS + kGenNT) + moff];
        } else {
          for (int c = 0; c < NC; ++c)  // combinations in which every needed (binary) input is on
            if ((need & ~c) == 0) s += r[kGenHdr + c * (kGenNS + kGenNT) + moff];
        }
        acc = fma(m, s, acc);
      }
    }
  }
  if (ent) part[(int64_t)blockIdx.y * NE + E] = acc;
}

__global__ void __launch_bounds__(kBlock)
gen_finalize_kernel(const double* __restrict__ part, int n_chunks, GenLib lib, int n_groups, double* __restrict__ G,
                    double* __restrict__ b) {
  const int NE = n_groups * lib.nEg;
  const int E = blockIdx.x * kBlock + threadIdx.x;
  if (E >= NE) return;
  double s = 0.0;
  for (int c = 0; c < n_chunks; ++c) s += part[(int64_t)c * NE + E];
  const int g = E / lib.nEg;
  int i, k;
  decode_entry(lib, E - g * lib.nEg, i, k);
  const int64_t F = lib.F;
  if (k >= 0) {
    G[(g * F + i) * F + k] = s;
    G[(g * F + k) * F + i] = s;
  } else {
    b[g * F + i] = s;
  }
}

// ---------------------------------------------------------------------------------------------
// STLSQ, F <= 64: one wavefront per system, lane i owns row i of the masked ridge matrix
// ---------------------------------------------------------------------------------------------
typedef unsigned long long u64;

__device__ bool gen_wave_chol_solve(const double* __restrict__ G, const double* __restrict__ b, int F, u64 m,
                                    double alpha, double* M, double* v, double* c, int lane) {
  constexpr int LD = kGenMaxF + 1;
  const bool row_on = lane < F;
  const bool ai = row_on && ((m >> lane) & 1ull);
  if (row_on) {
    for (int j = 0; j < F; ++j) {
      const bool act = ai && ((m >> j) & 1ull);
      double a = act ? G[(int64_t)lane * F + j] : 0.0;
      if (j == lane) a = ai ? a + alpha : 1.0;  // inactive rows: identity (the reduced solve's operations)
      M[lane * LD + j] = a;
    }
    v[lane] = ai ? b[lane] : 0.0;
  }
  wave_lds_sync();
  bool ok = true;
  for (int j = 0; j < F; ++j) {
    double dg = M[j * LD + j];
    if (!(dg > 0.0)) {
      ok = false;
      dg = 1e-300;
    }
    const double rd = 1.0 / sqrt(dg);
    wave_lds_sync();
    if (lane > j && lane < F) M[lane * LD + j] *= rd;
    if (lane == j) M[j * LD + j] = dg * rd;
    wave_lds_sync();
    if (lane > j && lane < F) {
      const double lij = M[lane * LD + j];
      for (int q = j + 1; q <= lane; ++q) M[lane * LD + q] = fma(-lij, M[q * LD + j], M[lane * LD + q]);
    }
    wave_lds_sync();
  }
  for (int j = 0; j < F; ++j) {
    const double zj = v[j] / M[j * LD + j];
    wave_lds_sync();
    if (lane == j) v[j] = zj;
    if (lane > j && lane < F) v[lane] = fma(-M[lane * LD + j], zj, v[lane]);
    wave_lds_sync();
  }
  for (int j = F - 1; j >= 0; --j) {
    const double cj = v[j] / M[j * LD + j];
    wave_lds_sync();
    if (lane == j) c[j] = ((m >> j) & 1ull) ? cj : 0.0;
    if (lane < j) v[lane] = fma(-M[j * LD + lane], cj, v[lane]);
    wave_lds_sync();
  }
  return ok;
}

__global__ void __launch_bounds__(kWave)
gen_stlsq_wave_kernel(const double* __restrict__ G, const double* __restrict__ B, int F, int n_sys, StlsqParams sp,
                      double* __restrict__ coef, int8_t* __restrict__ mask, int32_t* __restrict__ iters) {
  __shared__ double M[kGenMaxF * (kGenMaxF + 1)];
  __shared__ double v[kGenMaxF], c[kGenMaxF];
  const int s = blockIdx.x;
  const int lane = threadIdx.x;
  if (s >= n_sys) return;
  const double* Gs = G + (int64_t)s * F * F;
  const double* bs = B + (int64_t)s * F;
  const u64 all = F >= 64 ? ~0ull : ((1ull << F) - 1ull);
  u64 ind = all, prev = all;
  bool ok = true;
  int it = 0;
  c[lane] = 0.0;
  wave_lds_sync();
  for (int k = 0; k < sp.max_iter; ++k) {
    it = k + 1;
    if (ind == 0ull) {  // empty support: zeros (pkpd/utils.py:275-281)
      c[lane] = 0.0;
      wave_lds_sync();
      break;
    }
    ok &= gen_wave_chol_solve(Gs, bs, F, ind, sp.alpha, M, v, c, lane);
    wave_lds_sync();
    const bool big_l = lane < F && fabs(c[lane]) >= sp.thr;
    if (lane < F && !big_l) c[lane] = 0.0;
    wave_lds_sync();
    const u64 big = __ballot(big_l);
    const u64 pattern = __ballot(lane < F && c[lane] != 0.0);
    ind = big;
    if (ind == all || pattern == prev) break;  // stop rule (pkpd/utils.py:308-310)
    prev = pattern;
  }
  const u64 sup = __ballot(lane < F && fabs(c[lane]) > 1e-14);
  if (sp.unbias && sup) {
    // minimum-norm unbias over exactly duplicated columns (lstsq's solution; see stlsq_solve in insite_hip.hip):
    // lane k finds the first earlier active column equal to its own, one representative per group is solved
    // and its coefficient split equally
    int rep = lane;
    if (lane < F && ((sup >> lane) & 1ull)) {
      const double gkk = Gs[(int64_t)lane * F + lane], bk = bs[lane];
      for (int i = 0; i < lane; ++i)
        if (((sup >> i) & 1ull) && Gs[(int64_t)i * F + i] == gkk && Gs[(int64_t)lane * F + i] == gkk && bs[i] == bk) {
          rep = i;
          break;
        }
    }
    const u64 solve = sup & ~__ballot(rep != lane);
    ok &= gen_wave_chol_solve(Gs, bs, F, solve, 0.0, M, v, c, lane);
    wave_lds_sync();
    if (solve != sup) {
      // a representative is its own first equal column, so rep chains have length one
      int cnt = 0;
      for (int k = 0; k < F; ++k) cnt += __shfl(rep, k) == lane && ((sup >> k) & 1ull) ? 1 : 0;
      const double ci = lane < F ? c[lane] : 0.0;
      wave_lds_sync();
      if (lane < F && cnt > 1) c[lane] = ci / (double)cnt;
      wave_lds_sync();
      if (lane < F && rep != lane) c[lane] = c[rep];
    }
  }
  wave_lds_sync();
  if (lane < F) {
    coef[(int64_t)s * F + lane] = c[lane];
    if (mask) mask[(int64_t)s * F + lane] = (int8_t)((sup >> lane) & 1ull);
  }
  if (lane == 0 && iters) iters[s] = ok ? it : -1;
}

// ---------------------------------------------------------------------------------------------
// stage-evaluated rollout of a polynomial RHS (state degree D <= 4)
// ---------------------------------------------------------------------------------------------
struct GenRollArgs {
  const double* y0;
  const double* u;
  const int8_t* arm;
  const double* coef;
  double* y;
  int64_t a_sp, a_sk, y_sp, y_sk, coef_stride, N;
  int32_t T, substeps, A;
  double dt, drop;
};

__device__ __forceinline__ double horner4(const double (&P)[kGenMaxDeg + 1], double y) {
  return fma(fma(fma(fma(P[4], y, P[3]), y, P[2]), y, P[1]), y, P[0]);
}

template <int METHOD>
__global__ void __launch_bounds__(kBlock) gen_rollout_kernel(GenRollArgs ra, GenLib lib) {
  const int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (p >= ra.N) return;
  double uu[kGenMaxU];
#pragma unroll
  for (int t = 0; t < kGenMaxU; ++t) uu[t] = t < lib.U ? ra.u[p * lib.U + t] : 0.0;
  double P[INSITE_MAX_ARMS][kGenMaxDeg + 1];
  const double* cb = ra.coef + ra.coef_stride * p;
#pragma unroll
  for (int a = 0; a < INSITE_MAX_ARMS; ++a) {
#pragma unroll
    for (int e = 0; e <= kGenMaxDeg; ++e) P[a][e] = 0.0;
    if (a < ra.A)
      for (int j = 0; j < lib.F; ++j) {
        const double c = cb[a * lib.F + j];
        if (fabs(c) > ra.drop) {
          const double t = c * static_mono(lib, j, uu);
#pragma unroll
          for (int e = 0; e <= kGenMaxDeg; ++e)
            if (lib.ex[j] == e) P[a][e] += t;
        }
      }
  }
  double y = ra.y0[p];
  const double h = ra.dt / (double)ra.substeps;
  for (int k = 0; k < ra.T; ++k) {
    const int a = ra.arm[p * ra.a_sp + (int64_t)k * ra.a_sk];
    double Q[kGenMaxDeg + 1];
#pragma unroll
    for (int e = 0; e <= kGenMaxDeg; ++e) {
      double q = P[0][e];
#pragma unroll
      for (int aa = 1; aa < INSITE_MAX_ARMS; ++aa) q = (a == aa) ? P[aa][e] : q;
      Q[e] = q;
    }
    for (int s = 0; s < ra.substeps; ++s) {
      if constexpr (METHOD == INSITE_METHOD_EULER) {
        y = fma(horner4(Q, y), h, y);  // y + f(y) h (pkpd/utils.py:68-71)
      } else {
        const double k1 = horner4(Q, y);
        const double k2 = horner4(Q, fma(0.5 * h, k1, y));
        const double k3 = horner4(Q, fma(0.5 * h, k2, y));
        const double k4 = horner4(Q, fma(h, k3, y));
        y = fma(h / 6.0, (k1 + 2.0 * k2) + (2.0 * k3 + k4), y);
      }
    }
    ra.y[p * ra.y_sp + (int64_t)k * ra.y_sk] = y;
  }
}

int32_t build_gen_lib(const int8_t* exps, int32_t F, int32_t n_in, int32_t U, GenLib* lib) {
  if (!exps || F < 1 || F > kGenMaxF || n_in < 0 || n_in > kGenMaxIn || U < 0 || U > kGenMaxU)
    return INSITE_E_INVALID_ARG;
  std::memset(lib, 0, sizeof(*lib));
  lib->F = F;
  lib->U = U;
  lib->n_in = n_in;
  const int W = 1 + n_in + U;
  for (int j = 0; j < F; ++j) {
    const int8_t ex = exps[j * W];
    if (ex < 0) return INSITE_E_INVALID_ARG;
    if (ex > kGenMaxDeg) return INSITE_E_UNSUPPORTED;
    lib->ex[j] = ex;
    if (ex > lib->D) lib->D = ex;
    for (int i = 0; i < n_in; ++i) {
      const int8_t e = exps[j * W + 1 + i];
      if (e < 0) return INSITE_E_INVALID_ARG;
      if (e > 0) lib->tin[j] |= (int8_t)(1 << i);  // binary input: b^e = b
    }
    for (int t = 0; t < U; ++t) {
      const int8_t e = exps[j * W + 1 + n_in + t];
      if (e < 0 || e > 8) return INSITE_E_INVALID_ARG;
      lib->eu[j][t] = e;
    }
  }
  lib->nG = F * (F + 1) / 2;
  lib->nEg = lib->nG + F;
  return INSITE_OK;
}

size_t gen_rec_bytes(int64_t N) { return ((size_t)N * kGenRec * sizeof(double) + 255) & ~(size_t)255; }
size_t gen_d_bytes(int64_t N, int32_t n_steps) { return ((size_t)N * n_steps * sizeof(double) + 255) & ~(size_t)255; }

}  // namespace

extern "C" {

size_t insite_gen_gram_workspace_bytes(int64_t n_patients, int32_t n_steps, int32_t n_groups, int32_t n_terms) {
  if (n_patients < 0 || n_steps < 0 || n_groups < 1 || n_terms < 1) return 0;
  const size_t NE = (size_t)n_groups * ((size_t)n_terms * (n_terms + 1) / 2 + n_terms);
  return gen_d_bytes(n_patients, n_steps) + gen_rec_bytes(n_patients) + (size_t)kGenChunks * NE * sizeof(double);
}

int32_t insite_gen_gram_f64(const double* x, int64_t ldx, int32_t layout, int32_t n_steps, const double* u,
                            int32_t n_statics, const int8_t* step_in, int64_t ld_in, int32_t n_inputs,
                            const int8_t* group, int32_t n_groups, const int32_t* rows, int64_t n_patients,
                            const int8_t* exps, int32_t n_terms, int32_t fd_kind, double dt, double* G_out,
                            double* b_out, void* workspace, size_t workspace_bytes, void* stream) {
  if (layout != INSITE_LAYOUT_PATIENT_MAJOR && layout != INSITE_LAYOUT_TIME_MAJOR) return INSITE_E_INVALID_ARG;
  if (n_patients < 0 || n_steps < 0 || n_groups < 1 || n_groups > INSITE_MAX_ARMS || !(dt > 0.0) || !G_out || !b_out)
    return INSITE_E_INVALID_ARG;
  if (fd_kind < INSITE_FD_SMOOTHED4 || fd_kind > INSITE_FD_SMOOTHED1) return INSITE_E_INVALID_ARG;
  GenLib lib;
  int32_t st = build_gen_lib(exps, n_terms, n_inputs, n_statics, &lib);
  if (st != INSITE_OK) return st;
  const bool tm = layout == INSITE_LAYOUT_TIME_MAJOR;
  if (tm ? ldx < n_patients : ldx < n_steps) return INSITE_E_INVALID_ARG;
  if (n_inputs > 0 && (!step_in || (tm ? ld_in < n_patients : ld_in < n_steps))) return INSITE_E_INVALID_ARG;
  if (!workspace || workspace_bytes < insite_gen_gram_workspace_bytes(n_patients, n_steps, n_groups, n_terms))
    return INSITE_E_WORKSPACE;
  if (n_steps >= 65536) return INSITE_E_UNSUPPORTED;  // grid.y = steps
  hipStream_t hs = reinterpret_cast<hipStream_t>(stream);
  const int NE = n_groups * lib.nEg;
  char* w = static_cast<char*>(workspace);
  double* dsc = reinterpret_cast<double*>(w);
  double* rec = reinterpret_cast<double*>(w + gen_d_bytes(n_patients, n_steps));
  double* part = reinterpret_cast<double*>(w + gen_d_bytes(n_patients, n_steps) + gen_rec_bytes(n_patients));
  const int min_rows = (fd_kind == INSITE_FD_SMOOTHED4 || fd_kind == INSITE_FD_ORDER4) ? 5 : 2;
  if (n_patients > 0 && n_steps > 0) {
    if (!x || !rows || (n_statics > 0 && !u)) return INSITE_E_INVALID_ARG;
    const XView xv{x, tm ? 1 : ldx, tm ? ldx : 1};
    const unsigned gx = (unsigned)((n_patients + kBlock - 1) / kBlock);
    gen_deriv_kernel<<<dim3(gx, (unsigned)n_steps), kBlock, 0, hs>>>(xv, rows, n_steps, n_patients, fd_kind, min_rows,
                                                                     1.0 / dt, dsc, n_patients);
    st = launch_status();
    if (st != INSITE_OK) return st;
    gen_moments_kernel<<<gx, kBlock, 0, hs>>>(xv, dsc, n_patients, step_in, tm ? 1 : ld_in, tm ? ld_in : 1, group,
                                              n_statics > 0 ? u : x, n_statics, rows, n_steps, n_patients, lib.D,
                                              n_inputs, min_rows, rec);
    st = launch_status();
    if (st != INSITE_OK) return st;
  }
  const int64_t chunk = (n_patients + kGenChunks - 1) / kGenChunks > 0 ? (n_patients + kGenChunks - 1) / kGenChunks : 1;
  gen_contract_kernel<<<dim3((unsigned)((NE + kBlock - 1) / kBlock), kGenChunks), kBlock, 0, hs>>>(
      rec, n_patients, lib, n_groups, chunk, 0, part);
  st = launch_status();
  if (st != INSITE_OK) return st;
  gen_finalize_kernel<<<(NE + kBlock - 1) / kBlock, kBlock, 0, hs>>>(part, kGenChunks, lib, n_groups, G_out, b_out);
  return launch_status();
}

size_t insite_gen_gram_segments_workspace_bytes(int64_t n_patients, int32_t n_arms, int32_t n_terms) {
  if (n_patients < 0 || n_arms < 1 || n_terms < 1) return 0;
  const size_t NE = (size_t)n_arms * ((size_t)n_terms * (n_terms + 1) / 2 + n_terms);
  return gen_rec_bytes(n_patients) + (size_t)kGenChunks * NE * sizeof(double);
}

int32_t insite_gen_gram_segments_f64(const double* x, int64_t ldx, const int8_t* arm, int64_t ld_arm, int32_t layout,
                                     int32_t n_steps, const int32_t* seq_len, const double* u, int32_t n_statics,
                                     int64_t n_patients, int32_t n_arms, const int8_t* exps, int32_t n_terms,
                                     int32_t fd_kind, double dt, double* G_out, double* b_out, void* workspace,
                                     size_t workspace_bytes, void* stream) {
  if (layout != INSITE_LAYOUT_PATIENT_MAJOR && layout != INSITE_LAYOUT_TIME_MAJOR) return INSITE_E_INVALID_ARG;
  if (n_patients < 0 || n_steps < 1 || n_arms < 1 || n_arms > kGenMaxNC || !(dt > 0.0) || !G_out || !b_out)
    return INSITE_E_INVALID_ARG;
  if (fd_kind != INSITE_FD_ORDER1 && fd_kind != INSITE_FD_SMOOTHED1) return INSITE_E_INVALID_ARG;
  GenLib lib;
  int32_t st = build_gen_lib(exps, n_terms, 0, n_statics, &lib);
  if (st != INSITE_OK) return st;
  const bool tm = layout == INSITE_LAYOUT_TIME_MAJOR;
  if (tm ? (ldx < n_patients || ld_arm < n_patients) : (ldx < n_steps || ld_arm < n_steps - 1))
    return INSITE_E_INVALID_ARG;
  if (!workspace || workspace_bytes < insite_gen_gram_segments_workspace_bytes(n_patients, n_arms, n_terms))
    return INSITE_E_WORKSPACE;
  hipStream_t hs = reinterpret_cast<hipStream_t>(stream);
  const int NE = n_arms * lib.nEg;
  double* rec = static_cast<double*>(workspace);
  double* part = reinterpret_cast<double*>(static_cast<char*>(workspace) + gen_rec_bytes(n_patients));
  if (n_patients > 0) {
    if (!x || !arm || !seq_len || (n_statics > 0 && !u)) return INSITE_E_INVALID_ARG;
    const XView xv{x, tm ? 1 : ldx, tm ? ldx : 1};
    const unsigned gx = (unsigned)((n_patients + kBlock - 1) / kBlock);
    gen_seg_moments_kernel<<<gx, kBlock, 0, hs>>>(xv, arm, tm ? 1 : ld_arm, tm ? ld_arm : 1, seq_len, n_steps,
                                                  n_statics > 0 ? u : x, n_statics, n_patients, lib.D, n_arms,
                                                  fd_kind == INSITE_FD_SMOOTHED1 ? 1 : 0, 1.0 / dt, rec);
    st = launch_status();
    if (st != INSITE_OK) return st;
  }
  const int64_t chunk = (n_patients + kGenChunks - 1) / kGenChunks > 0 ? (n_patients + kGenChunks - 1) / kGenChunks : 1;
  gen_contract_kernel<<<dim3((unsigned)((NE + kBlock - 1) / kBlock), kGenChunks), kBlock, 0, hs>>>(
      rec, n_patients, lib, n_arms, chunk, 1, part);
  st = launch_status();
  if (st != INSITE_OK) return st;
  gen_finalize_kernel<<<(NE + kBlock - 1) / kBlock, kBlock, 0, hs>>>(part, kGenChunks, lib, n_arms, G_out, b_out);
  return launch_status();
}

// batched STLSQ for F in (INSITE_MAX_TERMS, 64]: dispatched by insite_stlsq_f64 (insite_hip.hip)
int32_t insite_stlsq_wave64_f64(const double* G, const double* b, int64_t n_sys, int32_t n_terms, double threshold,
                                double alpha, int32_t max_iter, int32_t unbias, double* coef_out, int8_t* mask_out,
                                int32_t* iters_out, void* stream) {
  if (n_terms < 1 || n_terms > kGenMaxF || n_sys < 0 || max_iter < 1) return INSITE_E_INVALID_ARG;
  if (n_sys == 0) return INSITE_OK;
  if (!G || !b || !coef_out || n_sys > 65535) return INSITE_E_INVALID_ARG;
  StlsqParams sp{threshold, alpha, max_iter, unbias, 1};
  gen_stlsq_wave_kernel<<<(unsigned)n_sys, kWave, 0, reinterpret_cast<hipStream_t>(stream)>>>(
      G, b, n_terms, (int)n_sys, sp, coef_out, mask_out, iters_out);
  return launch_status();
}

// stage-evaluated rollout for libraries with state degree 2..4 (dispatched by insite_rollout_f64)
int32_t insite_rollout_poly_f64(const double* y0, const double* u, const int8_t* arm, int64_t ld_arm,
                                const double* coef, int64_t coef_row_stride, const int8_t* exps, int32_t n_terms,
                                int64_t n_rows, int32_t T, int32_t n_statics, int32_t n_arms, double dt, int32_t method,
                                int32_t substeps, double drop_below, double* y_out, int64_t ld_y, int32_t layout,
                                void* stream) {
  if (layout != INSITE_LAYOUT_PATIENT_MAJOR && layout != INSITE_LAYOUT_TIME_MAJOR) return INSITE_E_UNSUPPORTED;
  if (n_rows < 0 || T < 0 || substeps < 1 || n_arms < 1 || n_arms > INSITE_MAX_ARMS) return INSITE_E_INVALID_ARG;
  if (method != INSITE_METHOD_EULER && method != INSITE_METHOD_RK4) return INSITE_E_INVALID_ARG;
  GenLib lib;
  int32_t st = build_gen_lib(exps, n_terms, 0, n_statics, &lib);
  if (st != INSITE_OK) return st;
  const bool tm = layout == INSITE_LAYOUT_TIME_MAJOR;
  if (tm ? (ld_arm < n_rows || ld_y < n_rows) : (ld_arm < T || ld_y < T)) return INSITE_E_INVALID_ARG;
  if (n_rows == 0 || T == 0) return INSITE_OK;
  if (!y0 || !arm || !coef || !y_out || (n_statics > 0 && !u)) return INSITE_E_INVALID_ARG;
  GenRollArgs ra{y0, n_statics > 0 ? u : y0, arm, coef, y_out, tm ? 1 : ld_arm, tm ? ld_arm : 1, tm ? 1 : ld_y,
                 tm ? ld_y : 1, coef_row_stride, n_rows, T, substeps, n_arms, dt, drop_below};
  const unsigned grid = (unsigned)((n_rows + kBlock - 1) / kBlock);
  hipStream_t hs = reinterpret_cast<hipStream_t>(stream);
  if (method == INSITE_METHOD_EULER) gen_rollout_kernel<INSITE_METHOD_EULER><<<grid, kBlock, 0, hs>>>(ra, lib);
  else gen_rollout_kernel<INSITE_METHOD_RK4><<<grid, kBlock, 0, hs>>>(ra, lib);
  return launch_status();
}

}  // extern "C"
