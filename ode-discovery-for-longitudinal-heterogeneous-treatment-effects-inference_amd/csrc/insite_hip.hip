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
#include <type_traits>

#include <cmath>
#include <cstdint>
#include <atomic>
#include <cstring>

#include "insite_hip.h"
#include "insite_common.h"

namespace {

constexpr int kMaxEntries = 64;       // Gram + moment entries, one per lane
constexpr int kGramMaxBlocks = 1024;  // fixed cap -> deterministic reduction order
constexpr int kPsStride = 17;         // per-patient LDS scratch row (odd -> conflict-free)

// Profiling-only phase timestamps (built with -DINSITE_TIMING by tools/build_ablation.sh): lane 0
// of each wave stores s_memtime at phase boundaries into g_tstamp[wave][slot].
#ifdef INSITE_TIMING
constexpr int kTsWaves = 1 << 16, kTsSlots = 10;  // slots 8/9: s_memrealtime at entry / exit
__device__ unsigned long long g_tstamp[kTsWaves * kTsSlots];
#define INSITE_TSTAMP(wave, slot)                                                                   \
  do {                                                                                              \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();                                     \
    if ((threadIdx.x & 63) == 0 && (wave) < kTsWaves) g_tstamp[(int64_t)(wave) * kTsSlots + (slot)] = t_; \
  } while (0)
#define INSITE_TREAL(wave, slot)                                                                    \
  do {                                                                                              \
    const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                                 \
    if ((threadIdx.x & 63) == 0 && (wave) < kTsWaves) g_tstamp[(int64_t)(wave) * kTsSlots + (slot)] = t_; \
  } while (0)
// slot 7: where the wave runs -- HW_ID (gfx9 layout: CU 11:8, SH 12, SE 14:13) | XCC_ID << 32
#define INSITE_THWID(wave)                                                                                     \
  do {                                                                                                         \
    const unsigned long long h_ = (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4) |             \
                                  ((unsigned long long)__builtin_amdgcn_s_getreg((3 << 11) | 20) << 32);      \
    if ((threadIdx.x & 63) == 0 && (wave) < kTsWaves) g_tstamp[(int64_t)(wave) * kTsSlots + 7] = h_;         \
  } while (0)
#else
#define INSITE_THWID(wave) \
  do {                     \
  } while (0)
#define INSITE_TSTAMP(wave, slot) \
  do {                            \
  } while (0)
#define INSITE_TREAL(wave, slot) \
  do {                           \
  } while (0)
#endif

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
  // MFMA Gram plan: C[16 x 16] += P^T Q over patients, P[p][a*F+i] = [arm_p == a] m_i(u_p),
  // Q[p][c] = m_{qexp[c]}(u_p) * moment_{qmom[c]}(p); entry e of arm a = C[a*F + ei[e]][qcol[e]]
  int32_t mfma;
  int32_t nq;
  int32_t n_atoms;                             // distinct u-monomials of the columns
  int8_t atom_exp[16][INSITE_MAX_STATICS];     // exponents of atom a (each <= 2)
  int8_t col_atom[INSITE_MAX_TERMS];           // atom of column j
  int8_t qatom[16];                            // Q column c = atom[qatom] * moment[qmom]
  int8_t qmom[16];  // 0: row count, 1: sum xs, 2: sum xs^2, 3: sum xdot, 4: sum xdot*xs
  int8_t qcol[kMaxEntries];
  // the same exponents packed into aligned dwords for loops with a run-time (wave-uniform) column or atom
  // index: a dynamically indexed int8 field of the by-value kernel argument compiles to a VECTOR byte load
  // plus s_waitcnt vmcnt(0) per iteration (no scalar byte loads on gfx9), which drained the gram's load
  // queue per atom of every work item; dword fields become scalar loads.
  int32_t ucode[INSITE_MAX_TERMS];  // column j: eu[j][0] | eu[j][1] << 8 | eu[j][2] << 16 | ex[j] << 24
  int32_t acode[16];                // atom a: atom_exp[a][0] | [1] << 8 | [2] << 16
};

// prod_i u[i]^((code >> 8 i) & 0xff): the u-monomial of a packed column / atom code
__device__ __forceinline__ double monomial_code(int code, const double* u) {
  double m = 1.0;
#pragma unroll
  for (int i = 0; i < INSITE_MAX_STATICS; ++i) {
    const int e = (code >> (8 * i)) & 0xff;
    for (int k = 0; k < e; ++k) m *= u[i];
  }
  return m;
}
__device__ __forceinline__ double monomial(const LibDesc& lib, int j, const double* u) {
  return monomial_code(lib.ucode[j] & 0xffffff, u);
}
__device__ __forceinline__ int col_ex(const LibDesc& lib, int j) { return (lib.ucode[j] >> 24) & 0xff; }

// =============================================================================================
// Discovery: fused smoothing + FD + library + Gram
// =============================================================================================
#ifndef INSITE_GT
#define INSITE_GT 16
#endif
#ifndef INSITE_PF
#define INSITE_PF 1
#endif
constexpr int kGT = INSITE_GT;     // time tile in steps: a multiple of the register ring length (8)
constexpr int kGStride = kGT + 1;  // LDS row stride in doubles (odd -> lane-per-row reads conflict free)
// per-wave LDS slot: 64 rows of max(kGStride, 17) doubles -- also the MFMA contraction's staging rows
// (32 x 23) and the scalar path's 64 x kPsStride rows
constexpr int kGSlot = kGStride > 17 ? kGStride : 17;
constexpr int kGPF = INSITE_PF;    // tiles in flight (register prefetch depth, 1 or 2)
#ifndef INSITE_GRAM_SCPF
#define INSITE_GRAM_SCPF 1
#endif
#ifndef INSITE_TM_DEPTH
#define INSITE_TM_DEPTH 2
#endif
// Time-major register ring: tiles of kGT steps, kTmDepth - 1 in flight while one is consumed.  A
// wave's step loads are 512-B rows; with ~1.5 waves per SIMD at C2 sizes the bytes in flight per
// wave set the achieved bandwidth (Little's law), so the ring is deep.
constexpr int kTmDepth = INSITE_TM_DEPTH;

__device__ __forceinline__ void add_row(double xk, double dk, double& Sx, double& Sxx, double& Sd, double& Sdx) {
  Sx += xk;
  Sxx = fma(xk, xk, Sxx);
  Sd += dk;
  Sdx = fma(dk, xk, Sdx);
}

// Whole-trajectory moments for short smoothed trajectories (5 <= LL <= 7 rows), every stencil
// position resolved at compile time.
template <int LL>
__device__ void small_trajectory(const double* __restrict__ xrow, int64_t step, const GramW& w, double& Sx,
                                 double& Sxx, double& Sd, double& Sdx) {
  double xv[LL], xs[LL];
#pragma unroll
  for (int j = 0; j < LL; ++j) xv[j] = xrow[j * step];
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
    double d;
    if (k == 0) d = fd_pos0(xs[0], xs[1], xs[2], xs[3], xs[4]) * w.inv_dt;
    else if (k == 1) d = fd_pos1(xs[0], xs[1], xs[2], xs[3], xs[4]) * w.inv_dt;
    else if (k == LL - 2) d = fd_pos3(xs[LL - 5], xs[LL - 4], xs[LL - 3], xs[LL - 2], xs[LL - 1]) * w.inv_dt;
    else if (k == LL - 1) d = fd_pos4(xs[LL - 5], xs[LL - 4], xs[LL - 3], xs[LL - 2], xs[LL - 1]) * w.inv_dt;
    else d = fd_int(w, xs[k - 2], xs[k - 1], xs[k + 1], xs[k + 2]);
    add_row(xv[k], d, Sx, Sxx, Sd, Sdx);  // library on the raw sample (pysindy: x_dot only is smoothed)
  }
}


// Telescoped derivative moments.  With the antisymmetric interior stencil
// d_k = fd1 (v_{k+1} - v_{k-1}) + fd2 (v_{k+2} - v_{k-2}),  for rows k = a..b:
//   sum d_k     = [fd1 (v_{b+1} + v_b) + fd2 (v_{b+2} + v_{b+1} + v_b + v_{b-1})]  - [same at a-1 .. a-2]
//   sum d_k v_k = [fd1 v_b v_{b+1} + fd2 (v_{b-1} v_{b+1} + v_b v_{b+2})]             - [a-side mirror]
// so the interior body needs no per-row derivative work at all.
__device__ __forceinline__ void tele_hi(const GramW& w, double vm1, double v0, double v1, double v2, double& sd,
                                        double& sdx) {  // v_{b-1}, v_b, v_{b+1}, v_{b+2}
  sd = w.fd1 * (v1 + v0) + w.fd2 * ((v2 + v1) + (v0 + vm1));
  sdx = w.fd1 * (v0 * v1) + w.fd2 * (vm1 * v1 + v0 * v2);
}
__device__ __forceinline__ void tele_lo(const GramW& w, double vm2, double vm1, double v0, double v1, double& sd,
                                        double& sdx) {  // v_{a-2}, v_{a-1}, v_a, v_{a+1}
  sd = w.fd1 * (v0 + vm1) + w.fd2 * ((v1 + v0) + (vm1 + vm2));
  sdx = w.fd1 * (vm1 * v0) + w.fd2 * (vm2 * v0 + vm1 * v1);
}

// In-launch fixed-order reduction of the gram partials (the split-K hand-off of the MI355X HIP guide,
// §6 Guideline 16, write-through form): every block stores its compact partial (the n_arms * nE Gram
// entries, a * nE + e) write-through (sc1, agent-scope atomic stores), drains, and takes a ticket; the
// last of each group of kTailGroup blocks (block-index order) sums the group's partials into a group
// partial, published the same way; the last group reducer (agent-scope acquire, then plain loads) sums
// the group partials in group order and writes G (both triangles) and b.  The summation order is fixed
// by block and group index, never by arrival, so results are deterministic.  The group reductions of
// all but the last group overlap the other blocks' streaming; after the last block only one group
// (<= kTailGroup partials of <= kTailMaxEnt doubles) and <= 64 group partials remain, where a separate
// finalize launch read every block's full tile.  Counters cnt[0] (groups), cnt[1 + g]: the last arriver
// of each counter resets it (all its arrivals are in), so a call leaves them zero; the workspace header
// must be zero before its first use (insite_gram_workspace_bytes).  The launcher's alternative, a memset
// node per call (-DINSITE_GRAM_MEMSET), puts a ~20 us gap in the stream on ROCm 7.2 (profiles/).
#ifndef INSITE_TAIL_RELEASE_FENCE
#define INSITE_TAIL_RELEASE_FENCE 0
#endif
constexpr int kTailGroup = 16;
constexpr int kTailMaxGroups = 64;  // group partials summed by the last reducer (counters cnt[1 .. 64])
constexpr int kTailMaxEnt = INSITE_MAX_ARMS * (INSITE_MAX_TERMS * (INSITE_MAX_TERMS + 1) / 2 + INSITE_MAX_TERMS);
struct GramOut {
  double* G;
  double* b;
  int n_arms;
  // STLSQ fused into the tail (gram_kernel STF > 0): the last block solves the n_arms systems
  double* coef;
  int8_t* mask;
  int32_t* iters;
  StlsqParams sp;
  double* mom;  // MOM = 2: per-patient moments [N, 5]
};

template <int F>
__device__ int stlsq_solve(const double (&g)[F][F], const double (&rhs)[F], double thr, double alpha,
                           int max_iter, int unbias, double (&c)[F], unsigned& sup,
                           unsigned init = (1u << F) - 1u);

__device__ __forceinline__ void tail_store(double* p, double v) {  // sc1 (write-through) 8-byte store
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), __double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// The tail's last stage, shared by gram_tail and the deferred finalisation (deferred_finalize): red[0, n_ent)
// holds the reduced Gram entries; write G (both triangles) and b, and with STF > 0 solve the n_arms STLSQ fits.
template <int STF>
__device__ __forceinline__ void tail_finish(double* red, int n_ent, const LibDesc& lib, const GramOut& o) {
  const int64_t F = lib.F;
  double* dense = red + kTailMaxEnt + 8;  // STF: [a][F x F | F] copy in LDS for the fused STLSQ
  constexpr int kDense = STF * STF + STF;
  for (int idx = threadIdx.x; idx < n_ent; idx += kBlock) {
    const int a = idx / lib.nE, e = idx - a * lib.nE;
    const int i = lib.ei[e], k = lib.ek[e];
    const double v = red[idx];
    if (k >= 0) {
      o.G[(a * F + i) * F + k] = v;
      o.G[(a * F + k) * F + i] = v;
      if constexpr (STF > 0) {
        dense[a * kDense + i * STF + k] = v;
        dense[a * kDense + k * STF + i] = v;
      }
    } else {
      o.b[a * F + i] = v;
      if constexpr (STF > 0) dense[a * kDense + STF * STF + i] = v;
    }
  }
  if constexpr (STF > 0) {  // one thread per arm, register-resident STLSQ (reference sindy.py:190-192)
    __syncthreads();
    const int a = (int)threadIdx.x;
    if (a < o.n_arms) {
      const double* d = dense + a * kDense;
      double g[STF][STF], rhs[STF], c[STF];
#pragma unroll
      for (int i = 0; i < STF; ++i) {
        rhs[i] = d[STF * STF + i];
#pragma unroll
        for (int j = 0; j <= i; ++j) g[i][j] = d[i * STF + j];
      }
      unsigned sup = 0u;
      const int it = stlsq_solve<STF>(g, rhs, o.sp.thr, o.sp.alpha, o.sp.max_iter, o.sp.unbias, c, sup);
#pragma unroll
      for (int i = 0; i < STF; ++i) {
        o.coef[a * STF + i] = c[i];
        if (o.mask) o.mask[a * STF + i] = (int8_t)((sup >> i) & 1u);
      }
      if (o.iters) o.iters[a] = it;
    }
  }
}

template <int STF>
__device__ __forceinline__ void gram_tail(const int vblk, const int nblk, double* __restrict__ part, int n_ent,
                                          unsigned* __restrict__ cnt, const LibDesc& lib, const GramOut& o,
                                          double* red) {
  int* flag = reinterpret_cast<int*>(red + kTailMaxEnt);  // "I am last", through the kernel's LDS array
  // group size: kTailGroup blocks, or a multiple of it so that at most kTailMaxGroups groups remain (the
  // segment kernel's one-tile-per-wave grids reach 8192 blocks); the group sums run in block order either way
  const int tg = nblk <= kTailGroup * kTailMaxGroups
                     ? kTailGroup
                     : ((nblk + kTailMaxGroups - 1) / kTailMaxGroups + kTailGroup - 1) / kTailGroup * kTailGroup;
  const int ng = (nblk + tg - 1) / tg;
  const int g = vblk / tg;
  const int g0 = g * tg;
  const int gs = nblk - g0 < tg ? nblk - g0 : tg;
  double* gpart = part + (int64_t)nblk * n_ent;
#ifdef INSITE_TIMING  // the final reducer's tail phases -> g_tstamp wave 49152 (slot 0 entry, 1..6 phases, 8/9 real)
  unsigned long long tt[7] = {__builtin_amdgcn_s_memtime(), 0, 0, 0, 0, 0, 0};
  const unsigned long long tr0 = __builtin_amdgcn_s_memrealtime();
#define INSITE_TT(k) tt[k] = __builtin_amdgcn_s_memtime()
#else
#define INSITE_TT(k) \
  do {               \
  } while (0)
#endif
  auto publish = [&](unsigned* counter, unsigned arrivals) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
    __syncthreads();
    if (threadIdx.x == 0) {
      // No release fence before the ticket (A/B knob INSITE_TAIL_RELEASE_FENCE).  On gfx950 an agent-scope
      // release compiles to `buffer_wbl2 sc1; s_waitcnt vmcnt(0)`: a write-back of every dirty line in this
      // XCD's L2 -- in the fused step kernel the rollout role's y stores -- at every block's arrival, which
      // measured 0.0622 -> 0.0732 ms per C2 step (profiles/r03/).  What the fence would order is already
      // ordered: every partial is written by an agent-scope atomic store, which gfx950 issues write-through
      // (`global_store ... sc1`: it never sits dirty in the L2), each storing wave has drained its stores
      // (s_waitcnt vmcnt(0): completion is acknowledged from the device coherence point) before the
      // __syncthreads that precedes this ticket, the ticket is an agent-scope atomic performed at that point,
      // and the last arriver reads only after its acquire fence (buffer_inv sc1).
#if INSITE_TAIL_RELEASE_FENCE
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
#endif
      const unsigned t = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = t == arrivals - 1u;
      if (last) {
        __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // every arrival is in
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      *flag = last;
    }
    __syncthreads();
    return *flag != 0;
  };
  if (!publish(&cnt[1 + g], (unsigned)gs)) return;
  INSITE_TT(1);
  for (int q = threadIdx.x; q < n_ent; q += kBlock) {  // the group's partials, block-index order
    double acc = 0.0;
    for (int j0 = 0; j0 < gs; j0 += kTailGroup) {  // kTailGroup loads in flight per round
      double v[kTailGroup];
#pragma unroll
      for (int j = 0; j < kTailGroup; ++j) v[j] = part[(int64_t)(g0 + (j0 + j < gs ? j0 + j : 0)) * n_ent + q];
#pragma unroll
      for (int j = 0; j < kTailGroup; ++j) acc += j0 + j < gs ? v[j] : 0.0;  // 0 + v[0] = v[0]: the old order
    }
    tail_store(gpart + (int64_t)g * n_ent + q, acc);
  }
  INSITE_TT(2);
  if (!publish(&cnt[0], (unsigned)ng)) return;
  INSITE_TT(3);
  for (int q = threadIdx.x; q < n_ent; q += kBlock) {  // the group partials, group order (ng <= 64)
    double acc = 0.0;
#pragma unroll 16
    for (int j = 0; j < ng; ++j) acc += gpart[(int64_t)j * n_ent + q];
    red[q] = acc;
  }
  __syncthreads();
  INSITE_TT(4);
  tail_finish<STF>(red, n_ent, lib, o);
#ifdef INSITE_TIMING
  INSITE_TT(6);
  if (threadIdx.x == 0) {
    unsigned long long* d = g_tstamp + (int64_t)49152 * kTsSlots;
    for (int k = 0; k < 7; ++k) d[k] = tt[k];
    d[8] = tr0;
    d[9] = __builtin_amdgcn_s_memrealtime();
  }
#endif
#undef INSITE_TT
}
// Deferred finalisation (step_deferred_kernel): one block reduces the nblk block partials a PREVIOUS launch
// left in `part` and finishes them (G|b, STLSQ) with tail_finish.  Same association as gram_tail (each group of
// tg blocks summed in block order from 0, then the groups in order), so G|b are bitwise those of the in-launch
// tail over the same partials; the (group, entry) sums run on all the block's threads, kTailGroup loads in
// flight each.  The partials were written by the previous kernel on this stream: visible after its end.
template <int STF>
__device__ void deferred_finalize(const double* __restrict__ part, const int nblk, const int n_ent, const LibDesc& lib,
                                  const GramOut& o, double* red) {
  constexpr int kOff = kTailMaxEnt + 8 + INSITE_MAX_ARMS * (INSITE_MAX_TERMS * INSITE_MAX_TERMS + INSITE_MAX_TERMS);
  // groups of kTailGroup blocks as in gram_tail, coarser (a multiple of it) when their sums would not fit the LDS
  const int maxg = min(kTailMaxGroups, (kWavesPerBlock * kWave * kGSlot - kOff) / (n_ent > 0 ? n_ent : 1));
  const int tg = nblk <= kTailGroup * maxg ? kTailGroup
                                           : ((nblk + maxg - 1) / maxg + kTailGroup - 1) / kTailGroup * kTailGroup;
  const int ng = (nblk + tg - 1) / tg;
  double* gsum = red + kOff;  // [ng][n_ent] group sums, after tail_finish's scratch
  for (int pi = threadIdx.x; pi < ng * n_ent; pi += kBlock) {
    const int g = pi / n_ent, q = pi - g * n_ent;
    const int g0 = g * tg, gs = nblk - g0 < tg ? nblk - g0 : tg;
    double acc = 0.0;
    for (int j0 = 0; j0 < gs; j0 += kTailGroup) {
      double v[kTailGroup];
#pragma unroll
      for (int j = 0; j < kTailGroup; ++j) v[j] = part[(int64_t)(g0 + (j0 + j < gs ? j0 + j : 0)) * n_ent + q];
#pragma unroll
      for (int j = 0; j < kTailGroup; ++j) acc += j0 + j < gs ? v[j] : 0.0;
    }
    gsum[pi] = acc;
  }
  __syncthreads();
  for (int q = threadIdx.x; q < n_ent; q += kBlock) {
    double acc = 0.0;
    for (int g = 0; g < ng; ++g) acc += gsum[g * n_ent + q];
    red[q] = acc;
  }
  __syncthreads();
  tail_finish<STF>(red, n_ent, lib, o);
}
static_assert(kTailMaxEnt + 8 + INSITE_MAX_ARMS * (INSITE_MAX_TERMS * INSITE_MAX_TERMS + INSITE_MAX_TERMS) +
                      kTailMaxEnt <= kWavesPerBlock * kWave * kGSlot,
              "deferred_finalize holds at least one group's sums in the gram kernel's LDS array");

// ---- Dynamic gram tail (INSITE_DEF_DYN): the deferred step's gram waves stream a static share
// of the tiles as before (one contiguous range per wave, block partials), then CLAIM fixed pieces of the remaining
// tail tiles -- (tile, range of kGT-step groups), never crossing a tile -- from per-XCD heads, each piece's Gram
// contribution stored in a partial slot of its own, indexed by PIECE, not by wave.  The next launch's finaliser sums
// the block partials and then the piece partials in one fixed order (dyn_finalize), so G|b do not depend on which
// wave took which piece.  Claims are agent-scope fetch-adds on one 128-B line per XCD (a wave claims from the head
// of the XCD its block runs on -- blockIdx % 8 under the dispatcher's round robin; speed only, correctness does not
// depend on placement -- and moves on to the other heads when its own is exhausted); the next piece is claimed while
// the current one streams.  The last wave to finish claiming (a 64-bit done word: waves << 32 | pieces) stores the
// number of pieces processed into the slot record and resets the claim area, so every launch leaves it zero, and the
// finaliser flags a slot whose pieces do not add up (NaN, iters -3) instead of summing it.
struct DynGram {
  unsigned* claim;   // kXcds head lines + one done line (kClaimWords words each); zero between launches
  double* ppart;     // piece partials [P][n_ent] (after the block partials of the slot)
  unsigned* hdr;     // the slot header (record word kSlotRec + 4: pieces processed)
  int64_t tile0;     // tiles [0, tile0) static, [tile0, n_tiles) claimed
  int64_t P;         // pieces: (n_tiles - tile0) * ppt
  int32_t pg;        // kGT-step groups per piece
  int32_t ppt;       // pieces per tail tile
  int32_t waves;     // gram waves taking part (the done count)
};
constexpr int kClaimWords = 32;  // one 128-B line per head
constexpr int kDynRecDone = 116;  // slot-header words (after the slot record, kSlotRec = 112 .. 115): pieces processed
constexpr int kDynRecP = 117;     //   and pieces streamed (the finaliser checks they agree)
constexpr int kDynHeads = 8;
constexpr size_t kDynClaimBytes = (size_t)(kDynHeads + 1) * kClaimWords * sizeof(unsigned);

// The fixed-order finalisation of the dynamic gram's slot: rows = block partials then piece partials, [R][n_ent].
// 256 threads take (row group, entry pair): the rows are cut into NGR contiguous row groups, each summed in row order
// with 16-B loads and kDynUnroll of them in flight per thread (the slot is ~1 MB at C2's shape, so one block needs
// ~100 KB in flight to read it in ~15 us beside the streaming), then the NGR group sums in group order.
constexpr int kDynUnroll = 16;
template <int STF>
__device__ void dyn_finalize(const double* __restrict__ part, const int R, const int n_ent, const LibDesc& lib,
                             const GramOut& o, double* red) {
  constexpr int kOff = kTailMaxEnt + 8 + INSITE_MAX_ARMS * (INSITE_MAX_TERMS * INSITE_MAX_TERMS + INSITE_MAX_TERMS);
  const int npair = (n_ent + 1) / 2;
  const int ngr = kBlock / npair;  // >= 1 (n_ent <= kTailMaxEnt <= 2 * kBlock)
  double* gsum = red + kOff;       // [ngr][2 * npair]
  const int t = (int)threadIdx.x;
  if (t < ngr * npair) {
    const int gq = t / npair, pp = t - gq * npair;
    const int r0 = (int)((int64_t)gq * R / ngr), r1 = (int)((int64_t)(gq + 1) * R / ngr);
    double ax = 0.0, ay = 0.0;
    const bool odd_last = 2 * pp + 1 >= n_ent;  // (n_ent odd: the last pair's second entry does not exist)
    for (int r = r0; r < r1; r += kDynUnroll) {
      double vx[kDynUnroll], vy[kDynUnroll];
#pragma unroll
      for (int j = 0; j < kDynUnroll; ++j) {
        const int rr = r + j < r1 ? r + j : r0;
        const double* q = part + (int64_t)rr * n_ent + 2 * pp;
        if ((n_ent & 1) == 0) {
          const double2 v = *reinterpret_cast<const double2*>(q);
          vx[j] = v.x;
          vy[j] = v.y;
        } else {
          vx[j] = q[0];
          vy[j] = odd_last ? 0.0 : q[1];
        }
      }
#pragma unroll
      for (int j = 0; j < kDynUnroll; ++j) {
        ax += r + j < r1 ? vx[j] : 0.0;
        ay += r + j < r1 ? vy[j] : 0.0;
      }
    }
    gsum[gq * 2 * npair + 2 * pp] = ax;
    gsum[gq * 2 * npair + 2 * pp + 1] = ay;
  }
  __syncthreads();
  for (int q = t; q < n_ent; q += kBlock) {
    double acc = 0.0;
    for (int g = 0; g < ngr; ++g) acc += gsum[g * 2 * npair + q];
    red[q] = acc;
  }
  __syncthreads();
  tail_finish<STF>(red, n_ent, lib, o);
}
static_assert(kTailMaxEnt + 8 + INSITE_MAX_ARMS * (INSITE_MAX_TERMS * INSITE_MAX_TERMS + INSITE_MAX_TERMS) +
                      2 * kBlock + 64 <= kWavesPerBlock * kWave * kGSlot,
              "dyn_finalize's group sums fit the gram kernel's LDS array");
static_assert(kTailMaxEnt + 8 + INSITE_MAX_ARMS * (INSITE_MAX_TERMS * INSITE_MAX_TERMS + INSITE_MAX_TERMS) <=
                  kWavesPerBlock * kWave * kGSlot,
              "tail scratch fits the gram kernel's LDS array");

// Lane = patient.  Work item = (64-patient tile, time segment [s*seg, (s+1)*seg)).  Rows are
// staged [64 x kGT] through LDS (coalesced 16-B loads; the next tile in flight while the current
// one is consumed); each lane streams its row through 8-deep register rings (compile-time ring
// indices: no moves).  Per body row only xs (5 flops), sum xs and sum xs^2 are updated; the
// derivative moments of the body are telescoped to its boundary samples.  A segment starts with
// an 8-step (4 without smoothing) warm-up.  Edge rows: 4 head rows (segment 0) and 4 tail rows
// (the segment holding step L-1) per patient, 2 + 2 without smoothing.  Moments are additive over
// segments; each work item adds its A(u) M A(u)^T contribution, as a 16x16x64 f64 MFMA product
// when the library fits (lib.mfma), else one Gram entry per lane.
// TM (time-major x[k * ldx + p]): a lane loads its own patient's kGT samples of a tile directly
// (each wave instruction reads 64 consecutive doubles of one step); no LDS staging or wave sync.
// MOM = 1: per-patient moments mode (one time segment per patient): instead of the Gram contraction
// every lane writes its patient's moments {L, sum xs, sum xs^2, sum xdot, sum xdot xs} to
// partial[p * 5 ..] (insite_sindy_fit_per_patient_f64).  MOM = 2: both from the same pass -- the moments
// to out.mom and the Gram with its reduction (insite_gram_moments_f64: C4's global + per-patient fits
// read x once).
// Otherwise the block partials are reduced inside the launch (gram_tail) into G [A, F, F] and b [A, F].
// The body is a device function of a virtual block index / grid size (vblk, vgrid) and the block's LDS,
// so the fused step kernel (step_kernel) can run it on a subset of its blocks.
constexpr int kGramSmem = kWavesPerBlock * kWave * kGSlot;  // doubles of LDS per block
// Work item -> (64-patient tile, time segment).  0: tile-major (the segments of one tile are consecutive
// items); 1 (A/B knob): segment-major (consecutive items are adjacent tiles of one segment, so the waves
// resident together read neighbouring columns of the same steps).
#ifndef INSITE_GRAM_ORDER
#define INSITE_GRAM_ORDER 0
#endif
// cache policy of the gram's time-major x loads (A/B: 2 = non-temporal, x is read once per launch; measured slower
// on the C2 step, 0.0706-0.0709 vs 0.0685-0.0692 ms launches, profiles/r04/lnt/)
#ifndef INSITE_GRAM_LOAD_AUX
#define INSITE_GRAM_LOAD_AUX 0
#endif
__device__ __forceinline__ int64_t gram_item_tile(int64_t item, int n_seg, int64_t n_tiles) {
  return INSITE_GRAM_ORDER ? item % n_tiles : item / n_seg;
}
__device__ __forceinline__ int gram_item_seg(int64_t item, int n_seg, int64_t n_tiles) {
  return INSITE_GRAM_ORDER ? (int)(item / n_tiles) : (int)(item - (item / n_seg) * n_seg);
}
// The block's partial (fixed order: wave 0..3 per entry) -> compact partial[block][a * nE + e], write-through.
template <bool MFMA, int NARM>
__device__ __forceinline__ void gram_block_partial(const int vblk, double* __restrict__ smem, const LibDesc& lib,
                                                   const GramOut& out, double* __restrict__ partial, const dbl4& cacc,
                                                   const double (&acc)[NARM], const int wid, const int lane) {
  __syncthreads();
  double* red = smem;
  const int n_ent = out.n_arms * lib.nE;  // the Gram entries the tail needs (<= kTailMaxEnt)
  if constexpr (MFMA) {
    // canonical C[row][col], row = (lane >> 4) + 4 j, col = lane & 15
#pragma unroll
    for (int j = 0; j < 4; ++j) red[wid * 256 + ((lane >> 4) + 4 * j) * 16 + (lane & 15)] = cacc[j];
  } else {
#pragma unroll
    for (int a = 0; a < NARM; ++a) red[(wid * NARM + a) * kWave + lane] = acc[a];
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < n_ent; idx += kBlock) {
    const int a = idx / lib.nE, e = idx - a * lib.nE;
    const int q = MFMA ? (a * lib.F + lib.ei[e]) * 16 + lib.qcol[e] : a * kWave + e;
    constexpr int stride = MFMA ? 256 : NARM * kWave;
    double v = red[q];
#pragma unroll
    for (int ww = 1; ww < kWavesPerBlock; ++ww) v += red[ww * stride + q];
    tail_store(partial + (int64_t)vblk * n_ent + idx, v);
  }
}

template <int VEC, int NARM, bool SMOOTH, bool MFMA, bool TM, int MOM, int STF = 0, int DYN = 0>
__device__ __forceinline__ void gram_body(const int vblk, const int vgrid, double* __restrict__ smem,
            const double* __restrict__ x, int64_t ldx, int n_steps, const double* __restrict__ u,
            const int8_t* __restrict__ arm, const int32_t* __restrict__ rows, int64_t N, int seg, int n_seg,
            const GramW& w, const LibDesc& lib, double* __restrict__ partial, unsigned* __restrict__ cnt,
            const GramOut& out, const DynGram* __restrict__ dgp = nullptr) {
  static_assert(!DYN || (TM && MFMA && MOM == 0), "the claimed gram tail is the deferred step's (time-major, MFMA)");
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);  // wave-uniform (SGPR)
  double* xt = smem + wid * (kWave * kGSlot);
  constexpr int kMinMain = SMOOTH ? 8 : 5;  // shorter (5..7, smoothed) rows take small_trajectory
  constexpr int kWarm = SMOOTH ? 8 : 4;     // warm-up steps of a segment's first tile
  constexpr int kLag = SMOOTH ? 4 : 2;      // body row kd = t - kLag
  constexpr int LPR = kGT / VEC;            // lanes per row segment
  constexpr int RPI = kWave / LPR;          // rows per wave instruction
  constexpr int NLD = kWave / RPI;          // load instructions per tile
  static_assert(!TM || (VEC == 1 && NLD == kGT), "time-major tiles hold the lane's own kGT samples");
  INSITE_TSTAMP(blockIdx.x * kWavesPerBlock + wid, 0);
  INSITE_TREAL(blockIdx.x * kWavesPerBlock + wid, 8);
  INSITE_THWID(blockIdx.x * kWavesPerBlock + wid);

  // G-phase accumulators
  dbl4 cacc = {0.0, 0.0, 0.0, 0.0};  // MFMA path: C[(lane>>4) + 4j][lane & 15]
  double acc[NARM];                   // scalar path: entry `lane`, per arm
#pragma unroll
  for (int a = 0; a < NARM; ++a) acc[a] = 0.0;
  const int my_i = lane < lib.nE ? lib.ei[lane] : 0;
  const int my_k = lane < lib.nE ? lib.ek[lane] : 0;
  const int my_exi = lib.ex[my_i];
  const int my_exk = my_k >= 0 ? lib.ex[my_k] : 0;
  // MFMA operand roles of this lane: P row r = a*F + i (atom of column i, arm a), Q column r
  const int pr_r = lane & 15;
  const int pr_a = pr_r / lib.F, pr_i = pr_r - (pr_r / lib.F) * lib.F;
  const bool pr_ok = MFMA && pr_r < NARM * lib.F;
  const int pr_atom = pr_ok ? lib.col_atom[pr_i] : 0;
  const bool q_ok = MFMA && pr_r < lib.nq;
  const int q_atom = q_ok ? lib.qatom[pr_r] : 0;
  const int q_mom = q_ok ? lib.qmom[pr_r] : 0;
  const int cl = (lane % LPR) * VEC;

  const int64_t n_tiles = (N + kWave - 1) / kWave;
  // Work pieces (tile, owned steps [s0, sE)).  n_seg > 0: items (tile, segment) of `seg` steps, strided over the
  // waves.  n_seg == 0 (range mode): the (tile, kGT-step group) units, tile-major, cut into one equal contiguous
  // range per wave (as the rollout role cuts its work), a piece being the part of the range inside one tile --
  // every wave streams the same number of steps whatever the cohort size, where items leave the waves with
  // one item more than the others setting the end (C2 at 1,228 waves: 3,126 items = 2.55 per wave).
  const bool ranged = n_seg == 0;
  const int ng = (n_steps + kGT - 1) / kGT;
  const int64_t nW = (int64_t)vgrid * kWavesPerBlock;
  const int64_t wv = (int64_t)vblk * kWavesPerBlock + wid;
  const int64_t units = ranged ? n_tiles * ng : n_tiles * n_seg;
  // DYN: only the tiles [0, tile0) are cut into static ranges; the rest is claimed piece by piece
  const int64_t units_s = (DYN && ranged) ? dgp->tile0 * ng : units;
  const int64_t c_end = ranged ? (wv + 1) * units_s / nW : units;
  struct Piece {
    int64_t tile, next;
    int s0, sE;
  };
  auto piece_of = [&](int64_t c) -> Piece {
    Piece pc;
    if (ranged) {
      pc.tile = c / ng;
      const int g0 = (int)(c - pc.tile * ng);
      const int g1 = (int)min((int64_t)ng, (int64_t)g0 + (c_end - c));
      pc.s0 = g0 * kGT;
      pc.sE = g1 * kGT;
      pc.next = c + (g1 - g0);
    } else {
      pc.tile = gram_item_tile(c, n_seg, n_tiles);
      pc.s0 = gram_item_seg(c, n_seg, n_tiles) * seg;
      pc.sE = pc.s0 + seg;
      pc.next = c + nW;
    }
    return pc;
  };
  // time-major register ring, live across work items: a wave with several items requests the next item's
  // first tiles as soon as the current item's last tile is consumed, so they stream in under the current
  // item's tail rows and Gram contraction (per-item start-up latency hidden; C4: ~8 items per wave)
  typedef double TmTile[kGT];
  TmTile vr[TM ? kTmDepth : 1];
  bool prefetched = false;  // wave-uniform: vr holds the current item's first kTmDepth tiles already
  // The next piece's per-patient scalars (row count, arm, statics) are requested with its first tiles and BEFORE
  // them (INSITE_GRAM_SCPF): vmcnt is in order, so scalars loaded after the tiles at the piece start made the wave
  // wait for every tile in flight -- one drained prefetch ring per piece
  int sc_L = 0, sc_a = -1;
  double sc_u[INSITE_MAX_STATICS] = {0.0, 0.0, 0.0};
  auto sc_load = [&](int64_t pp) {
    const int64_t pcl = pp < N ? pp : N - 1;
    sc_L = rows[pcl];
    sc_a = arm[pcl];
#pragma unroll
    for (int t = 0; t < INSITE_MAX_STATICS; ++t) sc_u[t] = u[pcl * lib.U + (t < lib.U ? t : 0)];
  };
  // wave-uniform descriptor over steps [t0, min(t0 + kGT, lim)) based at column q0 (valid columns qv): steps
  // past lim and lanes past N (out-of-range offset) read as 0
  auto tm_load_for = [&](TmTile& v, int t0, int lim, int64_t q0, int qv, unsigned qoff) {
    const int nrow = lim - t0 < kGT ? lim - t0 : kGT;
    const int bytes = nrow > 0 ? (int)(((int64_t)(nrow - 1) * ldx + qv) * 8) : 0;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(x + (int64_t)(nrow > 0 ? t0 : 0) * ldx + q0), (short)0, bytes, 0x00020000);
#pragma unroll
    for (int i = 0; i < kGT; ++i)
      v[i] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, qoff + (unsigned)(i * ldx * 8), 0,
                                                                             INSITE_GRAM_LOAD_AUX));
  };
  // ---- DYN state: claims are fetch-adds by lane 0 on the head of kDynHeads it is on; the piece index is read
  // (readfirstlane) only at wave-uniform points ----
  int64_t dq = -1, dnext = -1;        // the claimed piece being processed / the next one (once read)
  bool dnext_ok = false, dinfl = false, dexh = !DYN || dgp->P <= 0;
  int dphase = 0, dh = (int)(blockIdx.x % kDynHeads), dtried = 0;
  unsigned dcl = 0u, dmine = 0u;
  auto dyn_issue = [&]() {
    if constexpr (DYN) {
      if (lane == 0) dcl = __hip_atomic_fetch_add(dgp->claim + dh * kClaimWords, 1u, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
      dinfl = true;
    }
  };
  auto dyn_read = [&]() -> int64_t {  // the in-flight claim's piece, moving on to the other heads when exhausted
    if constexpr (DYN) {
      for (;;) {
        const int64_t idx = (int64_t)__builtin_amdgcn_readfirstlane(dcl);
        const int64_t lo = dh * dgp->P / kDynHeads, hi = (dh + 1) * dgp->P / kDynHeads;
        dinfl = false;
        if (lo + idx < hi) return lo + idx;
        if (++dtried >= kDynHeads) {
          dexh = true;
          return -1;
        }
        dh = (dh + 1) % kDynHeads;
        dyn_issue();
      }
    }
    return -1;
  };
  auto dyn_piece = [&](int64_t q) -> Piece {
    Piece pc;
    const int64_t tt = q / dgp->ppt;
    const int j = (int)(q - tt * dgp->ppt);
    pc.tile = dgp->tile0 + tt;
    pc.s0 = j * dgp->pg * kGT;
    pc.sE = min(ng, (j + 1) * dgp->pg) * kGT;
    pc.next = 0;
    return pc;
  };
  int64_t cur = ranged ? wv * units_s / nW : wv;
  for (;;) {
    Piece pc;
    if (cur < c_end) {
      pc = piece_of(cur);
      cur = pc.next;
      if constexpr (DYN)  // the last static piece: the first claim in flight while it streams
        if (!(cur < c_end) && !dexh) dyn_issue();
    } else {
      if constexpr (!DYN) {
        break;
      } else {
        if (dphase == 0) {  // every static range done: this block's partial (a block barrier), then claimed pieces
          gram_block_partial<MFMA, NARM>(vblk, smem, lib, out, partial, cacc, acc, wid, lane);
          __syncthreads();  // (the block's LDS is the waves' staging area again from here)
          cacc = {0.0, 0.0, 0.0, 0.0};
          dphase = 1;
        } else {  // the previous claimed piece's contribution -> its own slot (wave-local, no barrier)
          wave_lds_sync();
#pragma unroll
          for (int j = 0; j < 4; ++j) xt[((lane >> 4) + 4 * j) * 16 + (lane & 15)] = cacc[j];
          wave_lds_sync();
          const int n_ent = out.n_arms * lib.nE;
          for (int idx = lane; idx < n_ent; idx += kWave) {
            const int a = idx / lib.nE, e = idx - a * lib.nE;
            dgp->ppart[dq * n_ent + idx] = xt[(a * lib.F + lib.ei[e]) * 16 + lib.qcol[e]];
          }
          wave_lds_sync();
          cacc = {0.0, 0.0, 0.0, 0.0};
        }
        if (!dnext_ok) {
          if (!dinfl && !dexh) dyn_issue();
          dnext = dinfl ? dyn_read() : -1;
        }
        dnext_ok = false;
        dq = dnext;
        if (dq < 0) break;
        ++dmine;
        pc = dyn_piece(dq);
        if (!dexh) dyn_issue();  // the next claim in flight while this piece streams
      }
    }
    const int64_t tile = pc.tile;
    const int64_t p0 = tile * kWave;
    const int64_t p = p0 + lane;
    // time-major: the first kTmDepth tiles are requested before the per-patient scalars (their
    // range is clipped at the stored steps, not at this wave's longest row, which is not known yet)
    const int s0 = pc.s0;       // first step owned by this piece
    const bool first = s0 == 0;  // the piece holding the head rows (and the row count) of its tile
    const int tb = first ? 0 : s0 - kWarm;
    const int tm_valid = (int)(N - p0 < kWave ? N - p0 : kWave);
    const unsigned tm_off = p < N ? (unsigned)lane * 8u : kOOB;
    auto tm_load = [&](TmTile& v, int t0, int lim) { tm_load_for(v, t0, lim, p0, tm_valid, tm_off); };
    if (!(TM && INSITE_GRAM_SCPF && prefetched)) sc_load(p);  // (before the first tiles)
#ifndef INSITE_GRAM_LATE_ISSUE
    if constexpr (TM) {
      const int s1p = min(pc.sE, n_steps);
      if (!prefetched) {
#pragma unroll
        for (int d = 0; d < kTmDepth; ++d)
          if (tb + d * kGT < s1p) tm_load(vr[d], tb + d * kGT, s1p);
      }
    }
#endif
    prefetched = false;
    int L = 0;
    int arm_p = -1;
    double uu[INSITE_MAX_STATICS] = {0.0, 0.0, 0.0};
    {  // per-patient scalars, issued together and unconditionally (clamped index; sc_load)
      const int Lr = sc_L;
      const int ar = sc_a;
#pragma unroll
      for (int t = 0; t < INSITE_MAX_STATICS; ++t) uu[t] = (p < N && t < lib.U) ? sc_u[t] : 0.0;
      if (p < N) {
        L = Lr;
        arm_p = ar;
        if (L > n_steps) L = n_steps;  // stored steps (host: n_steps <= ldx when patient-major)
        if (L < 5) L = 0;  // too short for the 5-point stencils: contributes nothing
      }
    }
    const int Lm = L >= kMinMain ? L : 0;  // length on the streaming path
    const int Lmax = wave_max_i(Lm);
    const int s1 = min(pc.sE, Lmax);         // one past the last step processed
    INSITE_TSTAMP(blockIdx.x * kWavesPerBlock + wid, 1);
    const int e = min(Lm, pc.sE);            // per-lane end of owned steps
    const int Lmin = wave_min_i(e);
    const int bstart = max(2 * kLag, s0);    // first body step of the segment
    const bool has_body = e > bstart;        // at least one body row owned
    double Sx = 0.0, Sxx = 0.0, Sd = 0.0, Sdx = 0.0;

    if (s0 < Lmax) {
      typedef double TileRegs[NLD][VEC];
      TileRegs vA, vB;  // two tiles in flight (register prefetch, depth 2)
      // Loads are issued unconditionally from a clamped (always valid) address and masked after
      // the fact: exec-masked loads would make the compiler drain vmcnt(0) at every tile.
      auto load_tile = [&](TileRegs& v, int t0) {
        const int col = t0 + cl;
        const bool col_ok = col < s1;
        const int colc = col_ok ? col : 0;
#pragma unroll
        for (int it = 0; it < NLD; ++it) {
          const int64_t pr = p0 + it * RPI + lane / LPR;
          const bool ok = col_ok && pr < N;
          const double* src = x + (pr < N ? pr : N - 1) * ldx + colc;
          if constexpr (VEC == 2) {
            const double2 q = *reinterpret_cast<const double2*>(src);
            v[it][0] = ok ? q.x : 0.0;
            v[it][1] = ok ? q.y : 0.0;
          } else {
            const double q = *src;
            v[it][0] = ok ? q : 0.0;
          }
        }
      };
      auto store_tile = [&](const TileRegs& v) {
        if constexpr (TM) return;
        wave_lds_sync();  // every lane finished reading the previous tile
#pragma unroll
        for (int it = 0; it < NLD; ++it) {
          const int r = it * RPI + lane / LPR;
#pragma unroll
          for (int q = 0; q < VEC; ++q) xt[r * kGStride + cl + q] = v[it][q];
        }
        wave_lds_sync();
      };

      double xr[8], sr[8];  // rings: xr[i & 7] = x[tb + i];  sr[k & 7] = xs[tb + k]
#pragma unroll
      for (int j = 0; j < 8; ++j) xr[j] = sr[j] = 0.0;
      double loSd = 0.0, loSdx = 0.0;  // telescoped a-side terms
      // b-side / tail samples x[e-8 .. e-1] (x[e-5 .. e-1] unsmoothed), loaded during the last tile
      const bool tail = Lm > 0 && e == Lm && Lm - 1 >= s0;  // this segment holds step L-1
      const bool need_end = has_body || tail;
      constexpr int NQ = SMOOTH ? 8 : 5;
      double qe[NQ];
      bool tail_issued = false;
      auto issue_tail = [&]() {
        if (tail_issued) return;
        tail_issued = true;
        // valid either way: e >= NQ when need_end, and the patient-major ldx >= L >= NQ
        const int64_t pc = p < N ? p : N - 1;
        const double* xe = TM ? x + (need_end ? (int64_t)(e - NQ) * ldx + pc : pc)
                              : x + (need_end ? p * ldx + (e - NQ) : 0);
        const int64_t st = TM ? (need_end ? ldx : 0) : 1;
#pragma unroll
        for (int j = 0; j < NQ; ++j) {
          const double q = xe[j * st];
          qe[j] = need_end ? q : 0.0;
        }
      };

      // ---- first tile: steps [tb, tb+16): warm-up, a-side terms, head rows, body ----
      // sample i of the tile being consumed: LDS (patient-major) or the lane's own registers
      auto sample = [&](const auto& v, int i) -> double {
        if constexpr (TM) return v[i];
        else return xt[lane * kGStride + i];
      };
      if constexpr (TM) {
#ifdef INSITE_GRAM_LATE_ISSUE
#pragma unroll
        for (int d = 0; d < kTmDepth; ++d)
          if (tb + d * kGT < s1) tm_load(vr[d], tb + d * kGT, s1);
#endif
        if (!(tb + kTmDepth * kGT < s1)) issue_tail();  // every remaining tile already in flight
      } else {
        load_tile(vA, tb);
        store_tile(vA);
        if (tb + kGT < s1) load_tile(vA, tb + kGT);
        if constexpr (kGPF == 2) {
          if (tb + 2 * kGT < s1) load_tile(vB, tb + 2 * kGT);
          else issue_tail();
        } else {
          if (tb + kGT >= s1) issue_tail();
        }
      }
      {
        const bool masked = tb + kGT > Lmin;
#pragma unroll
        for (int i = 0; i < kGT; ++i) {
          if constexpr (TM) xr[i & 7] = sample(vr[0], i);
          else xr[i & 7] = sample(vA, i);
          const int t = tb + i;
          if constexpr (SMOOTH) {
            if (i >= 4) sr[(i - 2) & 7] = sg_int(w, xr[(i - 4) & 7], xr[(i - 3) & 7], xr[(i - 2) & 7], xr[(i - 1) & 7], xr[i & 7]);
            if (i == 7) {
              if (first) {  // head rows kd = 0..3 from x[0..7], xs[2..5]
                const double xs0 = sg_pos0(xr[0], xr[1], xr[2], xr[3], xr[4]);
                const double xs1 = sg_pos1(xr[0], xr[1], xr[2], xr[3], xr[4]);
                const double d0 = fd_pos0(xs0, xs1, sr[2], sr[3], sr[4]) * w.inv_dt;
                const double d1 = fd_pos1(xs0, xs1, sr[2], sr[3], sr[4]) * w.inv_dt;
                const double d2 = fd_int(w, xs0, xs1, sr[3], sr[4]);
                const double d3 = fd_int(w, xs1, sr[2], sr[4], sr[5]);
                const bool on = Lm > 0;
                add_row(on ? xr[0] : 0.0, on ? d0 : 0.0, Sx, Sxx, Sd, Sdx);
                add_row(on ? xr[1] : 0.0, on ? d1 : 0.0, Sx, Sxx, Sd, Sdx);
                add_row(on ? xr[2] : 0.0, on ? d2 : 0.0, Sx, Sxx, Sd, Sdx);
                add_row(on ? xr[3] : 0.0, on ? d3 : 0.0, Sx, Sxx, Sd, Sdx);
              }
            }
            if (i >= 8) {  // body row kd = t - 4: raw x[kd], x_dot from xs[kd-2 .. kd+2]
              double xk = xr[(i - 4) & 7];
              double dk = fd_int(w, sr[(i - 6) & 7], sr[(i - 5) & 7], sr[(i - 3) & 7], sr[(i - 2) & 7]);
              if (masked) {
                xk = (t < e) ? xk : 0.0;
                dk = (t < e) ? dk : 0.0;
              }
              add_row(xk, dk, Sx, Sxx, Sd, Sdx);
            }
          } else {
            if (i == 3) tele_lo(w, xr[0], xr[1], xr[2], xr[3], loSd, loSdx);  // x[a-2..a+1], a = tb + 2
            if (i == 4 && first) {  // head rows kd = 0, 1 from x[0..4]
              const double d0 = fd_pos0(xr[0], xr[1], xr[2], xr[3], xr[4]) * w.inv_dt;
              const double d1 = fd_pos1(xr[0], xr[1], xr[2], xr[3], xr[4]) * w.inv_dt;
              const bool on = Lm > 0;
              add_row(on ? xr[0] : 0.0, on ? d0 : 0.0, Sx, Sxx, Sd, Sdx);
              add_row(on ? xr[1] : 0.0, on ? d1 : 0.0, Sx, Sxx, Sd, Sdx);
            }
            if (i >= 4) {  // body row kd = t - 2
              double xk = xr[(i - 2) & 7];
              if (masked) xk = (t < e) ? xk : 0.0;
              Sx += xk;
              Sxx = fma(xk, xk, Sxx);
            }
          }
        }
      }
      INSITE_TSTAMP(blockIdx.x * kWavesPerBlock + wid, 2);
      // ---- remaining tiles of the segment (buffers alternate A, B; two tiles in flight) ----
      auto consume = [&](int t0, const auto& v) {
        if (t0 + kGT <= Lmin) {
#ifdef INSITE_ABLATE_GRAM_NOCOMPUTE  // profiling only: stream the samples, one add per step
#pragma unroll
          for (int i = 0; i < kGT; ++i) Sx += sample(v, i);
          return;
#endif
#pragma unroll
          for (int i = 0; i < kGT; ++i) {
            xr[i & 7] = sample(v, i);
            if constexpr (SMOOTH) {
              sr[(i - 2) & 7] = sg_int(w, xr[(i - 4) & 7], xr[(i - 3) & 7], xr[(i - 2) & 7], xr[(i - 1) & 7], xr[i & 7]);
              add_row(xr[(i - 4) & 7], fd_int(w, sr[(i - 6) & 7], sr[(i - 5) & 7], sr[(i - 3) & 7], sr[(i - 2) & 7]),
                      Sx, Sxx, Sd, Sdx);
            } else {
              const double xk = xr[(i - 2) & 7];
              Sx += xk;
              Sxx = fma(xk, xk, Sxx);
            }
          }
        } else {
#pragma unroll
          for (int i = 0; i < kGT; ++i) {
            if (t0 + i < s1) {
              xr[i & 7] = sample(v, i);
              const bool own = t0 + i < e;
              if constexpr (SMOOTH) {
                sr[(i - 2) & 7] = sg_int(w, xr[(i - 4) & 7], xr[(i - 3) & 7], xr[(i - 2) & 7], xr[(i - 1) & 7], xr[i & 7]);
                const double dk = fd_int(w, sr[(i - 6) & 7], sr[(i - 5) & 7], sr[(i - 3) & 7], sr[(i - 2) & 7]);
                add_row(own ? xr[(i - 4) & 7] : 0.0, own ? dk : 0.0, Sx, Sxx, Sd, Sdx);
              } else {
                const double xk = own ? xr[(i - 2) & 7] : 0.0;
                Sx += xk;
                Sxx = fma(xk, xk, Sxx);
              }
            }
          }
        }
      };
      if constexpr (TM) {
        // ring slot d holds tile tb + d * kGT (mod kTmDepth); each slot is refilled with the tile
        // kTmDepth ahead right after it is consumed (compile-time slot indices: no moves)
        if (tb + kTmDepth * kGT < s1) tm_load(vr[0], tb + kTmDepth * kGT, s1);
        else issue_tail();
        for (int t0 = tb + kGT; t0 < s1;) {
#pragma unroll
          for (int d = 1; d <= kTmDepth; ++d) {
            if (t0 < s1) {  // uniform
              consume(t0, vr[d % kTmDepth]);
              if (t0 + kTmDepth * kGT < s1) tm_load(vr[d % kTmDepth], t0 + kTmDepth * kGT, s1);
              else issue_tail();
              t0 += kGT;
            }
          }
        }
#ifndef INSITE_GRAM_NO_XPREFETCH
        {  // every tile of this item consumed: request the wave's next item's first tiles
          bool have = cur < c_end;  // uniform
          Piece np;
          if (have) {
            np = piece_of(cur);
          } else if constexpr (DYN) {
            if (dinfl) {  // the claim issued when this piece started: read it here, where only the tail loads are left
              dnext = dyn_read();
              dnext_ok = true;
              have = dnext >= 0;
              if (have) np = dyn_piece(dnext);
            }
          }
          if (have) {
            const int64_t np0 = np.tile * kWave;
            const int ntb = np.s0 == 0 ? 0 : np.s0 - kWarm;
            const int ns1p = min(np.sE, n_steps);
            const int nvalid = (int)(N - np0 < kWave ? N - np0 : kWave);
            const unsigned noff = np0 + lane < N ? (unsigned)lane * 8u : kOOB;
            if (INSITE_GRAM_SCPF) sc_load(np0 + lane);
#pragma unroll
            for (int d = 0; d < kTmDepth; ++d)
              if (ntb + d * kGT < ns1p) tm_load_for(vr[d], ntb + d * kGT, ns1p, np0, nvalid, noff);
            prefetched = true;
          }
        }
#endif
      } else if constexpr (kGPF == 2) {
        for (int t0 = tb + kGT; t0 < s1;) {
          store_tile(vA);
          if (t0 + 2 * kGT < s1) load_tile(vA, t0 + 2 * kGT);
          else issue_tail();
          consume(t0, vA);
          t0 += kGT;
          if (t0 >= s1) break;
          store_tile(vB);
          if (t0 + 2 * kGT < s1) load_tile(vB, t0 + 2 * kGT);
          else issue_tail();
          consume(t0, vB);
          t0 += kGT;
        }
      } else {
        for (int t0 = tb + kGT; t0 < s1; t0 += kGT) {
          store_tile(vA);
          if (t0 + kGT < s1) load_tile(vA, t0 + kGT);
          else issue_tail();
          consume(t0, vA);
        }
      }
      INSITE_TSTAMP(blockIdx.x * kWavesPerBlock + wid, 3);
      // ---- b-side telescoped terms and tail rows from the prefetched end samples ----
      issue_tail();
      if (need_end) {
        if constexpr (SMOOTH) {
          const double* q = qe;  // x[e-8 .. e-1]
          const double a0 = sg_int(w, q[0], q[1], q[2], q[3], q[4]);  // xs[e-6]
          const double a1 = sg_int(w, q[1], q[2], q[3], q[4], q[5]);  // xs[e-5]
          const double a2 = sg_int(w, q[2], q[3], q[4], q[5], q[6]);  // xs[e-4]
          const double a3 = sg_int(w, q[3], q[4], q[5], q[6], q[7]);  // xs[e-3]
          if (tail) {  // rows L-4 .. L-1: raw x[L-4 .. L-1] = q[4 .. 7]
            const double a4 = sg_pos3(q[3], q[4], q[5], q[6], q[7]);  // xs[L-2]
            const double a5 = sg_pos4(q[3], q[4], q[5], q[6], q[7]);  // xs[L-1]
            add_row(q[4], fd_int(w, a0, a1, a3, a4), Sx, Sxx, Sd, Sdx);
            add_row(q[5], fd_int(w, a1, a2, a4, a5), Sx, Sxx, Sd, Sdx);
            add_row(q[6], fd_pos3(a1, a2, a3, a4, a5) * w.inv_dt, Sx, Sxx, Sd, Sdx);
            add_row(q[7], fd_pos4(a1, a2, a3, a4, a5) * w.inv_dt, Sx, Sxx, Sd, Sdx);
          }
        } else {
          const double* q = qe;  // x[e-5 .. e-1]
          if (has_body) {  // body rows a..b, b = e - 3: x[b-1..b+2] = x[e-4 .. e-1]
            double hiSd, hiSdx;
            tele_hi(w, q[1], q[2], q[3], q[4], hiSd, hiSdx);
            Sd += hiSd - loSd;
            Sdx += hiSdx - loSdx;
          }
          if (tail) {
            add_row(q[3], fd_pos3(q[0], q[1], q[2], q[3], q[4]) * w.inv_dt, Sx, Sxx, Sd, Sdx);
            add_row(q[4], fd_pos4(q[0], q[1], q[2], q[3], q[4]) * w.inv_dt, Sx, Sxx, Sd, Sdx);
          }
        }
      }
    }
    if constexpr (SMOOTH) {
      if (first && L > 0 && L < kMinMain) {
        const double* xrow = TM ? x + p : x + p * ldx;
        const int64_t st = TM ? ldx : 1;
        if (L == 5) small_trajectory<5>(xrow, st, w, Sx, Sxx, Sd, Sdx);
        else if (L == 6) small_trajectory<6>(xrow, st, w, Sx, Sxx, Sd, Sdx);
        else small_trajectory<7>(xrow, st, w, Sx, Sxx, Sd, Sdx);
      }
    }
    if (s0 >= Lmax && !(SMOOTH && first)) continue;  // nothing owned by this work piece (uniform)
    if constexpr (MOM != 0) {  // 1: moments only (partial = the [N, 5] moments); 2: moments to out.mom + the Gram
      if (p < N) {
        double* mrow = (MOM == 1 ? partial : out.mom) + p * 5;
        mrow[0] = (double)L;
        mrow[1] = Sx;
        mrow[2] = Sxx;
        mrow[3] = Sd;
        mrow[4] = Sdx;
      }
      if constexpr (MOM == 1) continue;
    }
#ifdef INSITE_ABLATE_NOGPHASE
    acc[0] += Sx + Sxx + Sd + Sdx;
    continue;
#endif

    INSITE_TSTAMP(blockIdx.x * kWavesPerBlock + wid, 4);
    // ---- per-patient Gram block A(u) M A(u)^T ----
    const double M0 = first ? (double)L : 0.0;  // row count, counted once per patient
    const int my_arm = (L > 0) ? arm_p : -1;
    double* ps = xt;  // reuse the x tile
    if constexpr (MFMA) {
      // producer row per patient: atoms (u-monomials) | 5 moments | arm; consumer lanes gather
      // their P (arm-masked atom of column i) and Q (atom * moment) operands by per-lane index.
      constexpr int kRS = 23;  // row stride (odd); 32 patients per half fit the x tile
      for (int h = 0; h < 2; ++h) {
        wave_lds_sync();
        if ((lane >> 5) == h) {
          double* row = ps + (lane & 31) * kRS;
          for (int a = 0; a < lib.n_atoms; ++a) {  // uniform loop; exponents <= 2 (scalar loads of acode)
            const int c = lib.acode[a];
            const int e0 = c & 0xff, e1 = (c >> 8) & 0xff, e2 = (c >> 16) & 0xff;
            double m = 1.0;
            if (e0 >= 1) m *= uu[0];
            if (e0 >= 2) m *= uu[0];
            if (e1 >= 1) m *= uu[1];
            if (e1 >= 2) m *= uu[1];
            if (e2 >= 1) m *= uu[2];
            if (e2 >= 2) m *= uu[2];
            row[a] = m;
          }
          row[16] = M0;
          row[17] = Sx;
          row[18] = Sxx;
          row[19] = Sd;
          row[20] = Sdx;
          row[21] = (double)my_arm;
        }
        wave_lds_sync();
#pragma unroll
        for (int st = 0; st < 8; ++st) {  // K = 4 patients per MFMA, 8 steps per half
          const double* row = ps + (4 * st + (lane >> 4)) * kRS;
          const double av = (pr_ok && (int)row[21] == pr_a) ? row[pr_atom] : 0.0;
          const double bv = q_ok ? row[q_atom] * row[16 + q_mom] : 0.0;
          cacc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, cacc, 0, 0, 0);
        }
      }
      wave_lds_sync();
    } else {
      wave_lds_sync();
      for (int j = 0; j < lib.F; ++j) ps[lane * kPsStride + j] = monomial(lib, j, uu);
      ps[lane * kPsStride + 9] = M0;    // moment x^0
      ps[lane * kPsStride + 10] = Sx;   // moment x^1
      ps[lane * kPsStride + 11] = Sxx;  // moment x^2
      ps[lane * kPsStride + 12] = Sd;   // moment xdot * x^0
      ps[lane * kPsStride + 13] = Sdx;  // moment xdot * x^1
      ps[lane * kPsStride + 14] = (double)my_arm;
      wave_lds_sync();
      if (lane < lib.nE) {
        const int moff = my_k >= 0 ? 9 + my_exi + my_exk : 12 + my_exi;
        for (int q = 0; q < kWave; ++q) {
          const double* row = ps + q * kPsStride;
          double wq = row[my_i] * row[moff];
          if (my_k >= 0) wq *= row[my_k];
          const int a = (int)row[14];
#pragma unroll
          for (int aa = 0; aa < NARM; ++aa) acc[aa] += (a == aa) ? wq : 0.0;
        }
      }
      wave_lds_sync();
    }
  }

  INSITE_TSTAMP(blockIdx.x * kWavesPerBlock + wid, 5);
  // ---- block reduction (fixed order) -> compact partial[block][a * nE + e] -> gram_tail ----
  if constexpr (MOM == 1) return;
  if constexpr (DYN) {  // (the block partial was taken at the static -> claimed transition; dq < 0: all heads dry)
    if (lane == 0) {
      unsigned long long* dw = reinterpret_cast<unsigned long long*>(dgp->claim + kDynHeads * kClaimWords);
      const unsigned long long old = __hip_atomic_fetch_add(dw, (1ull << 32) | (unsigned long long)dmine,
                                                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if ((unsigned)(old >> 32) == (unsigned)dgp->waves - 1u) {  // the last wave: every claim has returned
        __hip_atomic_store(dgp->hdr + kDynRecDone, (unsigned)old + dmine, __ATOMIC_RELAXED,  // pieces processed,
                           __HIP_MEMORY_SCOPE_AGENT);                                // for the finaliser's check
#pragma unroll
        for (int h = 0; h < kDynHeads; ++h)
          __hip_atomic_store(dgp->claim + h * kClaimWords, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(dw, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    return;
  }
  gram_block_partial<MFMA, NARM>(vblk, smem, lib, out, partial, cacc, acc, wid, lane);
  INSITE_TSTAMP(blockIdx.x * kWavesPerBlock + wid, 6);
  if (cnt) gram_tail<STF>(vblk, vgrid, partial, out.n_arms * lib.nE, cnt, lib, out, smem);  // null: the deferred step's
  INSITE_TREAL(blockIdx.x * kWavesPerBlock + wid, 9);
}

#ifndef INSITE_GRAM_WPE
#define INSITE_GRAM_WPE 2  // waves per SIMD the gram's register budget is sized for (2: <= 256 VGPR+AGPR)
#endif
#ifndef INSITE_MOM_WPE
#define INSITE_MOM_WPE 2  // the per-patient-moments instance (no contraction phase)
#endif
template <int VEC, int NARM, bool SMOOTH, bool MFMA, bool TM, int MOM, int STF = 0>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(MOM == 1 ? INSITE_MOM_WPE : INSITE_GRAM_WPE)))
gram_kernel(const double* __restrict__ x, int64_t ldx, int n_steps, const double* __restrict__ u,
            const int8_t* __restrict__ arm, const int32_t* __restrict__ rows, int64_t N, int seg, int n_seg,
            GramW w, LibDesc lib, double* __restrict__ partial, unsigned* __restrict__ cnt, GramOut out) {
  __shared__ double smem[kGramSmem];
  gram_body<VEC, NARM, SMOOTH, MFMA, TM, MOM, STF>((int)blockIdx.x, (int)gridDim.x, smem, x, ldx, n_steps, u, arm, rows,
                                                  N, seg, n_seg, w, lib, partial, cnt, out);
}

// =============================================================================================
// STLSQ on Gram systems (pkpd/utils.py:213-327 semantics)
// =============================================================================================
// Solve (G_SS + alpha I) c_S = b_S for the support mask `m` with the inactive rows/columns
// replaced by identity rows: the Cholesky factor stays block diagonal, so the active block
// performs exactly the operations of the reduced solve (one reciprocal per pivot).  Only the lower
// triangle of g is read.  Returns false if the active block is not positive definite.
template <int F>
__device__ bool masked_cholesky_solve(const double (&g)[F][F], const double (&rhs)[F], unsigned m,
                                      double alpha, double (&c)[F]) {
  double l[F][F], rd[F];
  bool ok = true;
#pragma unroll
  for (int i = 0; i < F; ++i) {
    const bool ai = (m >> i) & 1u;
#pragma unroll
    for (int j = 0; j <= i; ++j) {
      const bool act = ai && ((m >> j) & 1u);
      double a = act ? g[i][j] : 0.0;
      if (i == j) a = ai ? a + alpha : 1.0;
#pragma unroll
      for (int q = 0; q < j; ++q) a = fma(-l[i][q], l[j][q], a);
      if (i == j) {
        if (!(a > 0.0)) {
          ok = false;
          a = 1e-300;
        }
        // 1/sqrt(a) from v_rsq_f64 + two Newton steps (no IEEE sqrt/div sequences on the
        // factorisation's critical path); l_ii = a / sqrt(a)
        double r = __builtin_amdgcn_rsq(a);
        r = r * fma(-0.5 * a * r, r, 1.5);
        r = r * fma(-0.5 * a * r, r, 1.5);
        l[i][i] = a * r;
        rd[i] = r;
      } else {
        l[i][j] = a * rd[j];
      }
    }
  }
  double z[F];
#pragma unroll
  for (int i = 0; i < F; ++i) {
    double s = ((m >> i) & 1u) ? rhs[i] : 0.0;
#pragma unroll
    for (int q = 0; q < i; ++q) s = fma(-l[i][q], z[q], s);
    z[i] = s * rd[i];
  }
#pragma unroll
  for (int i = F - 1; i >= 0; --i) {
    double s = z[i];
#pragma unroll
    for (int q = i + 1; q < F; ++q) s = fma(-l[q][i], c[q], s);
    c[i] = ((m >> i) & 1u) ? s * rd[i] : 0.0;
  }
  return ok;
}

// One STLSQ fit: all-ones initial support (pysindy BaseOptimizer), ridge on the active set,
// zero |c| < thr, stop when nothing was removed or the pattern repeats, then ind = |c| > 1e-14
// and the unbias solve.  Returns the iteration count, -1 if a solve was not positive definite.
template <int F>
__device__ int stlsq_solve(const double (&g)[F][F], const double (&rhs)[F], double thr, double alpha,
                           int max_iter, int unbias, double (&c)[F], unsigned& sup, unsigned init) {
  // init: initial support (all ones = pysindy BaseOptimizer; a global model's support =
  // LSQIntialMask, pkpd/utils.py:250-253).  The stop rule compares the support size with the
  // initial one (:308) and the pattern with the previous iterate (history_[0] = full lstsq guess).
  const unsigned all = (1u << F) - 1u;
  unsigned ind = init, prev = all;
  bool ok = true;
  int it = 0;
#pragma unroll
  for (int i = 0; i < F; ++i) c[i] = 0.0;
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
    if (ind == init || pattern == prev) break;
    prev = pattern;
  }
  sup = 0u;
#pragma unroll
  for (int i = 0; i < F; ++i)
    if (fabs(c[i]) > 1e-14) sup |= 1u << i;
  if (unbias && sup) {
    // pysindy's unbias is an unregularised lstsq on the support, i.e. its MINIMUM-NORM solution when the
    // support holds exactly duplicated columns (a static that is the same for every patient, e.g. EQ_5_A/B's
    // single patient type u0 == 1: columns {1, u0} and {x0, x0 u0} coincide, G singular).  Column k equals
    // an earlier active column i iff ||theta_i - theta_k||^2 = G_ii + G_kk - 2 G_ik = 0 with b_i = b_k:
    // solve on one representative per group, then split its coefficient equally (the minimum-norm split).
    int rep[F];
    unsigned solve = sup;
#pragma unroll
    for (int k = 0; k < F; ++k) {
      rep[k] = k;
#pragma unroll
      for (int i = 0; i < k; ++i)
        if (rep[k] == k && rep[i] == i && ((sup >> i) & 1u) && ((sup >> k) & 1u) && g[i][i] == g[k][k] &&
            g[k][i] == g[i][i] && rhs[i] == rhs[k])
          rep[k] = i;
      if (rep[k] != k) solve &= ~(1u << k);
    }
    ok &= masked_cholesky_solve<F>(g, rhs, solve, 0.0, c);
    if (solve != sup) {
#pragma unroll
      for (int i = 0; i < F; ++i) {
        int cnt = 0;
#pragma unroll
        for (int k = 0; k < F; ++k) cnt += (((sup >> k) & 1u) && rep[k] == i) ? 1 : 0;
        if (cnt > 1) c[i] /= (double)cnt;
      }
#pragma unroll
      for (int k = 0; k < F; ++k)
#pragma unroll
        for (int i = 0; i < k; ++i)
          if (rep[k] == i) c[k] = c[i];
    }
  }
  return ok ? it : -1;
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
#pragma unroll
    for (int j = 0; j <= i; ++j) g[i][j] = G[(s * F + i) * F + j];
  }
  unsigned sup = 0u;
  const int it = stlsq_solve<F>(g, rhs, thr, alpha, max_iter, unbias, c, sup);
#pragma unroll
  for (int i = 0; i < F; ++i) {
    coef[s * F + i] = c[i];
    if (mask) mask[s * F + i] = (int8_t)((sup >> i) & 1u);
  }
  if (iters) iters[s] = it;
}



// =============================================================================================
// Treatment-segment discovery (cancer_sim / EQ_5)
// =============================================================================================
// Reference: process_sindy_training_data (pkpd/utils.py:433-462, 607-637) cuts a patient's samples
// x[0..L] at every change of the per-step treatment into segments that share their boundary sample
// (the last one ends at x[L]); the four per-arm SINDy fits (sindy.py:193-216) differentiate each
// segment with FiniteDifference(order=1) — forward difference, backward at the segment's last
// sample — or SmoothedFiniteDifference(savgol window 2, polyorder 1).  Streaming form, lane =
// patient, one pass over the samples j < L of each lane:
//   sample j (own segment, arm a_j): library input xo_j, derivative d_j = (xs_{j+1} - xo_j) / dt;
//   if sample j+1 ends that segment (j+1 = L or a_{j+1} != a_j) it is added to the same arm as its
//   last sample: input x_{j+1}, derivative d_j (the backward difference at a segment end equals the
//   forward difference of the sample before it).
// So per step the lane adds (n, sx, sxx, n d, d sx), n = 1 + end, to arm a_j: one select per arm.
// Smoothed: inside a segment xs_i = (x_i + x_{i+1}) / 2 except at its first and last sample (raw);
// the derivative uses xs, the library the raw samples (pysindy smooths only for x_dot).
// Per 64-patient tile the per-(patient, arm) moments are contracted to Gram entries (one entry per
// lane, patients staged through LDS in two halves); the block partials go through the in-launch tail of
// gram_kernel (gram_tail: fixed-order group sums, G / b and the per-arm STLSQ in the last block).
#ifndef INSITE_SEG_KC
#define INSITE_SEG_KC 4
#endif
#ifndef INSITE_SEG_PF
#define INSITE_SEG_PF 1
#endif
constexpr int kSegMaxBlocks = 8192;  // partials: kSegMaxBlocks x NARM x 64 doubles (16 MB)
constexpr int kSegKC = INSITE_SEG_KC;  // steps per register chunk (loads issued ahead of the arithmetic)
constexpr bool kSegPF = INSITE_SEG_PF != 0;  // double-buffered chunks (next chunk in flight)
constexpr int kSegMono = INSITE_MAX_TERMS;
constexpr int kSegRS = kSegMono + 5 * INSITE_MAX_ARMS;  // LDS row: F monomials | NARM x 5 moments (29, odd)

#ifndef INSITE_SEG_WPE
#define INSITE_SEG_WPE 4  // waves per SIMD the register budget is sized for (4: <= 128 VGPRs)
#endif
#ifndef INSITE_SEG_RANGED
#define INSITE_SEG_RANGED 1
#endif
template <int NARM, bool SMOOTH1, int STF>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(INSITE_SEG_WPE)))
gram_seg_kernel(const double* __restrict__ x, int64_t xsp, int64_t xsk, const int8_t* __restrict__ arm, int64_t asp,
                int64_t ask, const int32_t* __restrict__ seq_len, int n_steps, const double* __restrict__ u, int64_t N,
                double inv_dt, LibDesc lib, double* __restrict__ partial, unsigned* __restrict__ cnt, GramOut out) {
  __shared__ double smem[kWavesPerBlock * 32 * kSegRS];
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  double* ps = smem + wid * (32 * kSegRS);
  double acc[NARM];
#pragma unroll
  for (int a = 0; a < NARM; ++a) acc[a] = 0.0;
  // contraction roles: lane = entry e + nE * g; the ng = 64 / nE lane groups split each half-tile's
  // 32 patients (group g takes q = g, g + ng, ...), so small libraries keep every lane busy
  const int ng = lib.nE <= kWave ? kWave / lib.nE : 1;
  const int my_g = lane / lib.nE;
  const int my_e = lane - my_g * lib.nE;
  const bool ent = my_g < ng;
  const int my_i = ent ? lib.ei[my_e] : 0;
  const int my_k = ent ? lib.ek[my_e] : -1;
  const int moff = kSegMono + (my_k >= 0 ? lib.ex[my_i] + lib.ex[my_k] : 3 + lib.ex[my_i]);

  const int64_t n_tiles = (N + kWave - 1) / kWave;
  // Work pieces (tile, steps [kbeg, kend)).  INSITE_SEG_RANGED (default): the (tile, kSegKC-step chunk) units,
  // tile-major, cut into one equal contiguous range per wave of a resident grid, a piece being the part of a
  // range inside one tile (it starts from sample kbeg with the segment state of that step: the arms of samples
  // kbeg - 1 and kbeg); moments are additive over a patient's pieces, so each piece is contracted on its own.
  // Otherwise one whole tile per wave (round 2; grid = one wave per tile).
  const int ngc = n_steps > 1 ? (n_steps - 1 + kSegKC - 1) / kSegKC : 1;
  const int64_t nW = (int64_t)gridDim.x * kWavesPerBlock, wv = (int64_t)blockIdx.x * kWavesPerBlock + wid;
  const int64_t c_end = INSITE_SEG_RANGED ? (wv + 1) * (n_tiles * ngc) / nW : n_tiles;
  for (int64_t cur = INSITE_SEG_RANGED ? wv * (n_tiles * ngc) / nW : wv; cur < c_end;) {
    int64_t tile;
    int kbeg, kend;
    if (INSITE_SEG_RANGED) {
      tile = cur / ngc;
      const int g0 = (int)(cur - tile * ngc);
      const int g1 = (int)min((int64_t)ngc, (int64_t)g0 + (c_end - cur));
      kbeg = g0 * kSegKC;
      kend = g1 * kSegKC;
      cur += g1 - g0;
    } else {
      tile = cur;
      kbeg = 0;
      kend = n_steps;
      cur += nW;
    }
    const int64_t p = tile * kWave + lane;
    const bool valid = p < N;
    int L = valid ? seq_len[p] : 0;
    if (L > n_steps - 1) L = n_steps - 1;
    if (L < 0) L = 0;
    const int Lw = min(wave_max_i(L), kend);  // one past the last step this piece processes
    double mo[NARM][5];
#pragma unroll
    for (int a = 0; a < NARM; ++a)
#pragma unroll
      for (int j = 0; j < 5; ++j) mo[a][j] = 0.0;
    // Per chunk the wave reads samples k0+1 .. k0+KC (+1) and arms k0+1 .. k0+KC through buffer
    // descriptors based at the wave's first patient (wave-uniform base, 32-bit per-lane offsets), every
    // load issued unconditionally: lanes past N read through an offset the hardware drops, steps past
    // the stored range read 0, and samples past the lane's own L are masked after the load (exec-masked
    // loads would serialise: one vmcnt(0) per load).
    const int64_t p0 = tile * kWave;
    const int nvalid = (int)(N - p0 < kWave ? N - p0 : kWave);
    const unsigned xvo = valid ? (unsigned)((int64_t)lane * xsp * 8) : kOOB;
    const unsigned avo = valid ? (unsigned)((int64_t)lane * asp) : kOOB;
    auto x_rsrc = [&](int kb) {  // samples kb .. kb + KC of the wave's patients
      int rows = n_steps - kb;
      if (rows > kSegKC + 1) rows = kSegKC + 1;
      const int bytes = rows > 0 ? (int)(((int64_t)(nvalid - 1) * xsp + (int64_t)(rows - 1) * xsk + 1) * 8) : 0;
      return __builtin_amdgcn_make_buffer_rsrc((void*)(x + p0 * xsp + (int64_t)(rows > 0 ? kb : 0) * xsk), (short)0,
                                               bytes, 0x00020000);
    };
    auto a_rsrc = [&](int kb) {  // arms kb .. kb + KC - 1 (stored steps < n_steps - 1)
      int rows = n_steps - 1 - kb;
      if (rows > kSegKC) rows = kSegKC;
      const int bytes = rows > 0 ? (int)((int64_t)(nvalid - 1) * asp + (int64_t)(rows - 1) * ask + 1) : 0;
      return __builtin_amdgcn_make_buffer_rsrc((void*)(arm + p0 * asp + (int64_t)(rows > 0 ? kb : 0) * ask), (short)0,
                                               bytes, 0x00020000);
    };
    const unsigned xstep = (unsigned)(xsk * 8), astep = (unsigned)ask;
    if (kbeg < Lw) {
      double xj;
      int aj;
      int aprev = -1;  // arm of sample j-1 (SMOOTH1: segment-start test)
      {
        const __amdgpu_buffer_rsrc_t rx = x_rsrc(kbeg), ra = a_rsrc(kbeg);
        const double x0 = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rx, xvo, 0, 0));
        xj = kbeg <= L ? x0 : 0.0;  // past the lane's samples (padding may be NaN): zero, as the chunk masks do
        const int a0 = (int)(int8_t)__builtin_amdgcn_raw_buffer_load_b8(ra, avo, 0, 0);
        aj = kbeg < L ? a0 : -1;
        if (SMOOTH1 && kbeg > 0) {  // uniform
          const int am = (int)(int8_t)__builtin_amdgcn_raw_buffer_load_b8(a_rsrc(kbeg - 1), avo, 0, 0);
          aprev = kbeg - 1 < L ? am : -1;
        }
      }
      constexpr int NX = kSegKC + (SMOOTH1 ? 1 : 0);
      // raw chunk registers; the masks (k <= L, k < L) are applied at the use, so a prefetched chunk
      // is not waited for when it is issued
      auto load = [&](double (&xr)[NX], int (&ar)[kSegKC], int k0) {
        const __amdgpu_buffer_rsrc_t rx = x_rsrc(k0 + 1), ra = a_rsrc(k0 + 1);
#pragma unroll
        for (int j = 0; j < NX; ++j)
          xr[j] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rx, xvo + j * xstep, 0, 0));
#pragma unroll
        for (int j = 0; j < kSegKC; ++j)
          ar[j] = (int)(int8_t)__builtin_amdgcn_raw_buffer_load_b8(ra, avo + j * astep, 0, 0);
      };
      auto process = [&](const double (&xr)[NX], const int (&ar)[kSegKC], int k0) {
#pragma unroll
        for (int j = 0; j < kSegKC; ++j) {
          const double x1 = (k0 + 1 + j <= L) ? xr[j] : 0.0;
          const int a1 = (k0 + 1 + j < L) ? ar[j] : -1;
          const bool endf = a1 != aj;  // sample j+1 closes j's segment (also at j+1 = L)
          const double xo = xj;  // library input: the raw sample (the smoothing feeds x_dot only)
          double xso, xs1;
          if constexpr (SMOOTH1) {
            const double x2 = (k0 + 2 + j <= L) ? xr[j + 1] : 0.0;
            xso = (aj != aprev) ? xj : 0.5 * (xj + x1);
            xs1 = endf ? x1 : 0.5 * (x1 + x2);
          } else {
            xso = xj;
            xs1 = x1;
          }
          const double d = (xs1 - xso) * inv_dt;
          const double xc = endf ? x1 : 0.0;
          const double n = endf ? 2.0 : 1.0;
          const double sx = xo + xc;
          const double sxx = fma(xo, xo, xc * xc);
          const double sd = d * n;
          const double sdx = d * sx;
#pragma unroll
          for (int a = 0; a < NARM; ++a) {
            const double w = (aj == a) ? 1.0 : 0.0;  // aj = -1 past the lane's own samples
            mo[a][0] = fma(w, n, mo[a][0]);
            mo[a][1] = fma(w, sx, mo[a][1]);
            mo[a][2] = fma(w, sxx, mo[a][2]);
            mo[a][3] = fma(w, sd, mo[a][3]);
            mo[a][4] = fma(w, sdx, mo[a][4]);
          }
          aprev = aj;
          aj = a1;
          xj = x1;
        }
      };
      double xA[NX], xB[NX];
      int aA[kSegKC], aB[kSegKC];
      if constexpr (kSegPF) {
        // two chunks in flight: chunk c + 1 is requested before chunk c is consumed (buffers alternate)
        load(xA, aA, kbeg);
        for (int k0 = kbeg; k0 < Lw;) {
          if (k0 + kSegKC < Lw) load(xB, aB, k0 + kSegKC);
          process(xA, aA, k0);
          k0 += kSegKC;
          if (k0 >= Lw) break;
          if (k0 + kSegKC < Lw) load(xA, aA, k0 + kSegKC);
          process(xB, aB, k0);
          k0 += kSegKC;
        }
      } else {
        for (int k0 = kbeg; k0 < Lw; k0 += kSegKC) {
          load(xA, aA, k0);
          process(xA, aA, k0);
        }
      }
    }
    // ---- per-(patient, arm) Gram blocks A(u) M_a A(u)^T, one entry per lane ----
    double uu[INSITE_MAX_STATICS];
#pragma unroll
    for (int t = 0; t < INSITE_MAX_STATICS; ++t) uu[t] = (valid && t < lib.U) ? u[p * lib.U + t] : 0.0;
    for (int h = 0; h < 2; ++h) {
      wave_lds_sync();
      if ((lane >> 5) == h) {
        double* row = ps + (lane & 31) * kSegRS;
        for (int j = 0; j < lib.F; ++j) row[j] = valid ? monomial(lib, j, uu) : 0.0;
#pragma unroll
        for (int a = 0; a < NARM; ++a)
#pragma unroll
          for (int j = 0; j < 5; ++j) row[kSegMono + 5 * a + j] = mo[a][j];
      }
      wave_lds_sync();
      if (ent) {
#pragma unroll 2
        for (int q = my_g; q < 32; q += ng) {
          const double* row = ps + q * kSegRS;
          const double wq = row[my_i] * (my_k >= 0 ? row[my_k] : 1.0);
#pragma unroll
          for (int a = 0; a < NARM; ++a) acc[a] = fma(wq, row[moff + 5 * a], acc[a]);
        }
      }
    }
    wave_lds_sync();
  }
  // ---- block reduction (fixed order) -> compact partial[block][a * nE + e] -> in-launch tail ----
  // (gram_tail: group partials, then G / b and, STF > 0, the per-arm STLSQ fits in the last arriving block;
  // replaces round 2's separate discovery_finalize launch)
  __syncthreads();
  double* red = smem;
#pragma unroll
  for (int a = 0; a < NARM; ++a) red[(wid * NARM + a) * kWave + lane] = acc[a];
  __syncthreads();
  const int n_ent = out.n_arms * lib.nE;
  for (int idx = threadIdx.x; idx < n_ent; idx += kBlock) {  // entry: fixed-order sum over waves and lane groups
    const int a = idx / lib.nE, e = idx - a * lib.nE;
    double sum = 0.0;
    for (int ww = 0; ww < kWavesPerBlock; ++ww)
      for (int g = 0; g < ng; ++g) sum += red[(ww * NARM + a) * kWave + g * lib.nE + e];
    tail_store(partial + (int64_t)blockIdx.x * n_ent + idx, sum);
  }
  gram_tail<STF>((int)blockIdx.x, (int)gridDim.x, partial, n_ent, cnt, lib, out, smem);
}

// Per-patient refit (LSQIntialMask per patient, pkpd_simulation.py:791-800):
// thread = patient.  Its Gram G_p = A(u) M A(u)^T and moments b_p come from the five moments the
// MOM pass wrote; STLSQ starts from the support of the global model of the patient's arm.  The
// unbias is the minimum-norm least-squares solution (what lstsq returns): with one patient the
// statics are constant, so Theta_p = [m_j(u) x^{e_j}] has rank <= 2 and the fitted RHS is
// alpha + beta x; (alpha, beta) solve the 1x1 / 2x2 moment system of the support's exponent
// groups and c_j = m_j * alpha / sum m_k^2 (e_j = 0), m_j * beta / sum m_k^2 (e_j = 1).  If
// sum |c| > 10 the reference refits without unbias (:795-798): the last ridge iterate is kept.
// Other arms keep the global coefficients; patients with < 5 rows keep the global model.
#ifndef INSITE_PP_WPE
#define INSITE_PP_WPE 2  // waves per SIMD the per-patient fit's register budget is sized for
#endif
// The ridge iterations of that STLSQ in closed form.  On the support S the system is
// (G_SS + alpha I) c = b_S with G = V W V^T, b = V s: V [j, e] = m_j [e_j == e] (two disjoint column
// groups, state exponent 0 / 1), W = [[M0, M1], [M1, M2]], s = (Sd, Sdx).  Its unique solution (alpha > 0)
// lies in span(V): c = V z with (W N + alpha I) z = s, N = V^T V = diag(n0, n1), n_e = sum_{j in S, e_j = e}
// m_j^2 -- a 2 x 2 solve per iteration instead of a 7 x 7 Cholesky (and ~20 registers instead of ~180), so
// the fit fits in the rollout's prologue (rollout_bits_range PR = 2).  Mathematically the masked solve of
// stlsq_solve (its rounding differs at the last bits).  Stop rules, support and iteration count are
// stlsq_solve's with init = the global support.  Returns the iteration count, or -3 if alpha <= 0 (the
// caller then runs stlsq_solve, whose Cholesky reports a singular ridge system).
__device__ __forceinline__ int refit_rank2(const double (&m)[INSITE_MAX_TERMS], const int (&e)[INSITE_MAX_TERMS], int F,
                                           const double (&M)[3], double Sd, double Sdx, double thr, double alpha,
                                           int max_iter, unsigned init, double (&c)[INSITE_MAX_TERMS], unsigned& sup) {
  if (!(alpha > 0.0)) return -3;
  const unsigned all = (1u << F) - 1u;
  unsigned ind = init, prev = all;
  int it = 0;
#pragma unroll
  for (int j = 0; j < INSITE_MAX_TERMS; ++j) c[j] = 0.0;
  for (int k = 0; k < max_iter; ++k) {
    it = k + 1;
    if (ind == 0u) {
#pragma unroll
      for (int j = 0; j < INSITE_MAX_TERMS; ++j) c[j] = 0.0;
      break;
    }
    double n0 = 0.0, n1 = 0.0;
#pragma unroll
    for (int j = 0; j < INSITE_MAX_TERMS; ++j) {
      const double q = ((ind >> j) & 1u) ? m[j] * m[j] : 0.0;
      if (e[j]) n1 += q;
      else n0 += q;
    }
    const double a11 = fma(M[0], n0, alpha), a12 = M[1] * n1, a21 = M[1] * n0, a22 = fma(M[2], n1, alpha);
    const double det = a11 * a22 - a12 * a21;
    const double z0 = (Sd * a22 - a12 * Sdx) / det, z1 = (a11 * Sdx - a21 * Sd) / det;
    unsigned big = 0u;
#pragma unroll
    for (int j = 0; j < INSITE_MAX_TERMS; ++j) {
      double cj = ((ind >> j) & 1u) ? m[j] * (e[j] ? z1 : z0) : 0.0;
      if (fabs(cj) >= thr) big |= 1u << j;
      else cj = 0.0;
      c[j] = cj;
    }
    ind = big;
    unsigned pattern = 0u;
#pragma unroll
    for (int j = 0; j < INSITE_MAX_TERMS; ++j)
      if (c[j] != 0.0) pattern |= 1u << j;
    if (ind == init || pattern == prev) break;
    prev = pattern;
  }
  sup = 0u;
#pragma unroll
  for (int j = 0; j < INSITE_MAX_TERMS; ++j)
    if (fabs(c[j]) > 1e-14) sup |= 1u << j;
  return it;
}

// The per-patient unbias (minimum-norm lstsq on the support, closed form -- see patient_fit_kernel) and the
// reference's sum |c| > 10 fallback; c holds the last ridge iterate on entry.
__device__ __forceinline__ void refit_unbias(const double (&m)[INSITE_MAX_TERMS], const int (&e)[INSITE_MAX_TERMS],
                                             const double (&M)[3], double Sd, double Sdx, unsigned sup,
                                             double (&c)[INSITE_MAX_TERMS]) {
  double n0 = 0.0, n1 = 0.0;
#pragma unroll
  for (int j = 0; j < INSITE_MAX_TERMS; ++j)
    if ((sup >> j) & 1u) {
      if (e[j]) n1 += m[j] * m[j];
      else n0 += m[j] * m[j];
    }
  const bool h0 = n0 > 0.0, h1 = n1 > 0.0;
  double al = 0.0, be = 0.0, cu[INSITE_MAX_TERMS];
  bool rank1 = false;
  if (h0 && h1) {
    const double det = M[0] * M[2] - M[1] * M[1];
    if (det > 1e-13 * M[0] * M[2]) {
      al = (Sd * M[2] - M[1] * Sdx) / det;
      be = (M[0] * Sdx - M[1] * Sd) / det;
    } else {
      rank1 = true;  // x constant: every support column ~ m_j x0^{e_j}
    }
  } else if (h0) {
    al = Sd / M[0];
  } else if (h1 && M[2] > 0.0) {
    be = Sdx / M[2];
  }
  double s1 = 0.0;
  if (rank1) {
    const double x0 = M[1] / M[0];
    double vv = 0.0;
#pragma unroll
    for (int j = 0; j < INSITE_MAX_TERMS; ++j)
      if ((sup >> j) & 1u) vv += (m[j] * (e[j] ? x0 : 1.0)) * (m[j] * (e[j] ? x0 : 1.0));
    const double tq = vv > 0.0 ? Sd / (M[0] * vv) : 0.0;
#pragma unroll
    for (int j = 0; j < INSITE_MAX_TERMS; ++j) {
      cu[j] = ((sup >> j) & 1u) ? m[j] * (e[j] ? x0 : 1.0) * tq : 0.0;
      s1 += fabs(cu[j]);
    }
  } else {
#pragma unroll
    for (int j = 0; j < INSITE_MAX_TERMS; ++j) {
      cu[j] = ((sup >> j) & 1u) ? (e[j] ? (h1 ? m[j] * be / n1 : 0.0) : (h0 ? m[j] * al / n0 : 0.0)) : 0.0;
      s1 += fabs(cu[j]);
    }
  }
  if (s1 <= 10.0) {
#pragma unroll
    for (int j = 0; j < INSITE_MAX_TERMS; ++j) c[j] = cu[j];
  }
}

// One patient's refit from its five moments (the patient_fit_kernel semantics): c[] = the refitted row of
// arm a (global coefficients outside the refit), returns the STLSQ iteration count (0: < 5 rows, the global
// model kept; -1: a non-positive-definite ridge system).
template <int F, bool FALLBACK = true>
__device__ __forceinline__ int patient_refit(const LibDesc& lib, const double* uu, const double (&M)[3], double Sd,
                                             double Sdx, int L, const double* gca, const StlsqParams& sp,
                                             double (&c)[INSITE_MAX_TERMS], unsigned& init_out) {
  const int Fr = lib.F;  // == F in patient_fit_kernel; the fold (F = INSITE_MAX_TERMS) runs any library
  unsigned init = 0u;
#pragma unroll
  for (int j = 0; j < INSITE_MAX_TERMS; ++j) {
    c[j] = j < Fr ? gca[j] : 0.0;
    if (j < Fr && fabs(c[j]) > 1e-14) init |= 1u << j;
  }
  init_out = init;
  if (L < 5) return 0;
  double m[INSITE_MAX_TERMS];
  int e[INSITE_MAX_TERMS];
#pragma unroll
  for (int j = 0; j < INSITE_MAX_TERMS; ++j) {
    m[j] = j < Fr ? monomial(lib, j, uu) : 0.0;
    e[j] = j < Fr ? col_ex(lib, j) : 0;
  }
  unsigned sup = 0u;
  int it = refit_rank2(m, e, Fr, M, Sd, Sdx, sp.thr, sp.alpha, sp.max_iter, init, c, sup);
  if constexpr (!FALLBACK) {
    if (it == -3) return -3;  // the caller guarantees alpha > 0
  } else if (it == -3) {  // alpha <= 0: the generic masked-Cholesky STLSQ
    double g[F][F], rhs[F], cf[F];
#pragma unroll
    for (int i = 0; i < F; ++i) {
      rhs[i] = m[i] * (e[i] ? Sdx : Sd);
#pragma unroll
      for (int j = 0; j <= i; ++j) g[i][j] = m[i] * m[j] * M[e[i] + e[j]];
    }
    it = stlsq_solve<F>(g, rhs, sp.thr, sp.alpha, sp.max_iter, 0, cf, sup, init);
#pragma unroll
    for (int j = 0; j < INSITE_MAX_TERMS; ++j) c[j] = j < F ? cf[j] : 0.0;
  }
  if (sp.unbias && sup) refit_unbias(m, e, M, Sd, Sdx, sup, c);
  return it;
}

// CHOL: the masked-Cholesky STLSQ (alpha <= 0, where the closed form does not apply; also the round-2 path);
// otherwise the closed-form refit, without the Cholesky code's registers
template <int F, bool CHOL>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(INSITE_PP_WPE)))
patient_fit_kernel(const double* __restrict__ mom, const double* __restrict__ u, const int8_t* __restrict__ arm,
                   const int32_t* __restrict__ rows, int64_t N, int n_steps, int n_arms, LibDesc lib,
                   const double* __restrict__ gcoef, StlsqParams sp, double* __restrict__ coef,
                   int8_t* __restrict__ mask, int32_t* __restrict__ iters) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= N) return;
  const int a = arm[p];
  int L = rows[p];
  if (L > n_steps) L = n_steps;
  for (int aa = 0; aa < n_arms; ++aa)
#pragma unroll
    for (int j = 0; j < F; ++j) coef[(p * n_arms + aa) * F + j] = gcoef[aa * F + j];
  if (a < 0 || a >= n_arms) {
    if (iters) iters[p] = -2;
    return;
  }
  if constexpr (!CHOL) {
  double uu[INSITE_MAX_STATICS];
#pragma unroll
  for (int t = 0; t < INSITE_MAX_STATICS; ++t) uu[t] = t < lib.U ? u[p * lib.U + t] : 0.0;
  const double M[3] = {mom[p * 5 + 0], mom[p * 5 + 1], mom[p * 5 + 2]};
  double c[INSITE_MAX_TERMS];
  unsigned init = 0u;
  const int it = patient_refit<F, false>(lib, uu, M, mom[p * 5 + 3], mom[p * 5 + 4], L, gcoef + a * F, sp, c, init);
  unsigned fin = 0u;
#pragma unroll
  for (int j = 0; j < F; ++j) {
    coef[(p * n_arms + a) * F + j] = c[j];
    if (fabs(c[j]) > 1e-14) fin |= 1u << j;
  }
  if (L < 5) fin = init;
  if (mask) {
#pragma unroll
    for (int j = 0; j < F; ++j) mask[p * F + j] = (int8_t)((fin >> j) & 1u);
  }
  if (iters) iters[p] = it;
  } else {
  unsigned init = 0u;
#pragma unroll
  for (int j = 0; j < F; ++j)
    if (fabs(gcoef[a * F + j]) > 1e-14) init |= 1u << j;
  if (L < 5) {
    if (mask) {
#pragma unroll
      for (int j = 0; j < F; ++j) mask[p * F + j] = (int8_t)((init >> j) & 1u);
    }
    if (iters) iters[p] = 0;
    return;
  }
  double uu[INSITE_MAX_STATICS];
#pragma unroll
  for (int t = 0; t < INSITE_MAX_STATICS; ++t) uu[t] = t < lib.U ? u[p * lib.U + t] : 0.0;
  const double M[3] = {mom[p * 5 + 0], mom[p * 5 + 1], mom[p * 5 + 2]};
  const double Sd = mom[p * 5 + 3], Sdx = mom[p * 5 + 4];
  double m[F], g[F][F], rhs[F], c[F];
  int e[F];
#pragma unroll
  for (int j = 0; j < F; ++j) {
    m[j] = monomial(lib, j, uu);
    e[j] = col_ex(lib, j);
  }
#pragma unroll
  for (int i = 0; i < F; ++i) {
    rhs[i] = m[i] * (e[i] ? Sdx : Sd);
#pragma unroll
    for (int j = 0; j <= i; ++j) g[i][j] = m[i] * m[j] * M[e[i] + e[j]];
  }
  unsigned sup = 0u;
  int it = stlsq_solve<F>(g, rhs, sp.thr, sp.alpha, sp.max_iter, 0, c, sup, init);
  if (sp.unbias && sup) {
    double n0 = 0.0, n1 = 0.0;
#pragma unroll
    for (int j = 0; j < F; ++j)
      if ((sup >> j) & 1u) {
        if (e[j]) n1 += m[j] * m[j];
        else n0 += m[j] * m[j];
      }
    const bool h0 = n0 > 0.0, h1 = n1 > 0.0;
    double al = 0.0, be = 0.0, cu[F];
    bool rank1 = false;
    if (h0 && h1) {
      const double det = M[0] * M[2] - M[1] * M[1];
      if (det > 1e-13 * M[0] * M[2]) {
        al = (Sd * M[2] - M[1] * Sdx) / det;
        be = (M[0] * Sdx - M[1] * Sd) / det;
      } else {
        rank1 = true;  // x constant: every support column ~ m_j x0^{e_j}
      }
    } else if (h0) {
      al = Sd / M[0];
    } else if (h1 && M[2] > 0.0) {
      be = Sdx / M[2];
    }
    double s1 = 0.0;
    if (rank1) {
      const double x0 = M[1] / M[0];
      double vv = 0.0;
#pragma unroll
      for (int j = 0; j < F; ++j)
        if ((sup >> j) & 1u) vv += (m[j] * (e[j] ? x0 : 1.0)) * (m[j] * (e[j] ? x0 : 1.0));
      const double tq = vv > 0.0 ? Sd / (M[0] * vv) : 0.0;
#pragma unroll
      for (int j = 0; j < F; ++j) {
        cu[j] = ((sup >> j) & 1u) ? m[j] * (e[j] ? x0 : 1.0) * tq : 0.0;
        s1 += fabs(cu[j]);
      }
    } else {
#pragma unroll
      for (int j = 0; j < F; ++j) {
        cu[j] = ((sup >> j) & 1u) ? (e[j] ? (h1 ? m[j] * be / n1 : 0.0) : (h0 ? m[j] * al / n0 : 0.0)) : 0.0;
        s1 += fabs(cu[j]);
      }
    }
    if (s1 <= 10.0) {
#pragma unroll
      for (int j = 0; j < F; ++j) c[j] = cu[j];
    }
  }
  unsigned fin = 0u;
#pragma unroll
  for (int j = 0; j < F; ++j) {
    coef[(p * n_arms + a) * F + j] = c[j];
    if (fabs(c[j]) > 1e-14) fin |= 1u << j;
  }
  if (mask) {
#pragma unroll
    for (int j = 0; j < F; ++j) mask[p * F + j] = (int8_t)((fin >> j) & 1u);
  }
  if (iters) iters[p] = it;
  }
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

// The per-patient refit folded into a rollout prologue (rollout_bits_range PR = 2; C4): the factual arm's
// row is refitted from the patient's moments (patient_refit, closed-form ridge), the other arms keep the
// global model; optional per-patient outputs as insite_fit_per_patient_moments_f64.
struct RefitArgs {
  const double* mom;      // [N, 5]
  const int8_t* farm;     // [N] factual arm
  const int32_t* rows;    // [N] regression rows
  const double* gcoef;    // [A, F] global model
  double* coef_out;       // [N, A, F] or null
  int8_t* mask_out;       // [N, F] or null
  int32_t* iters_out;     // [N] or null
  StlsqParams sp;
  int32_t n_steps;
};


// Per-patient affine rates of every arm, f_a(y) = alpha_a + beta_a y: columns with x-exponent 0 feed alpha,
// exponent 1 beta (terms with |c| <= drop dropped, sindy.py:388).  The lane's A x F coefficients are loaded
// first, every load from a clamped (valid) index so all of them are in flight at once -- a loop over the
// run-time F with the load inside issued one load and one wait per term (a per-patient-coefficient row at
// C4 sizes: 14 dependent HBM round trips before the first step); the column codes are dword scalar loads.
// Accumulation order (j ascending per arm) is that of the reference's term sum.
template <int NARM>
__device__ __forceinline__ void affine_rates_regs(const LibDesc& lib, const double (&cv)[NARM][INSITE_MAX_TERMS], int A,
                                                  double drop, const double* uu, double* alpha, double* beta);
template <int NARM>
__device__ __forceinline__ void load_coef_rows(const LibDesc& lib, const double* cbase, int A,
                                               double (&cv)[NARM][INSITE_MAX_TERMS]) {
#pragma unroll
  for (int a = 0; a < NARM; ++a)
#pragma unroll
    for (int j = 0; j < INSITE_MAX_TERMS; ++j) {
      const int aa = a < A ? a : 0, jj = j < lib.F ? j : 0;
      cv[a][j] = cbase[aa * lib.F + jj];
    }
}
template <int NARM>
__device__ __forceinline__ void affine_rates(const LibDesc& lib, const double* cbase, int A, double drop,
                                             const double* uu, double* alpha, double* beta) {
  double cv[NARM][INSITE_MAX_TERMS];
  load_coef_rows<NARM>(lib, cbase, A, cv);
  affine_rates_regs<NARM>(lib, cv, A, drop, uu, alpha, beta);
}
template <int NARM>
__device__ __forceinline__ void affine_rates_regs(const LibDesc& lib, const double (&cv)[NARM][INSITE_MAX_TERMS], int A,
                                                  double drop, const double* uu, double* alpha, double* beta) {
#pragma unroll
  for (int a = 0; a < NARM; ++a) alpha[a] = beta[a] = 0.0;
#pragma unroll
  for (int j = 0; j < INSITE_MAX_TERMS; ++j) {
    if (j < lib.F) {
      const int code = lib.ucode[j];
      const double m = monomial_code(code & 0xffffff, uu);
      const bool lin = (code >> 24) != 0;
#pragma unroll
      for (int a = 0; a < NARM; ++a) {
        if (a < A) {
          const double c = cv[a][j];
          const double v = fabs(c) > drop ? c * m : 0.0;
          if (lin) beta[a] += v;
          else alpha[a] += v;
        }
      }
    }
  }
}

// Interval propagator.  Every library of this ABI is affine in the state (INSITE_MAX_STATE_DEGREE
// 1), so per arm the RHS is f(y) = al + be * y with al, be fixed per patient, and one observation
// interval of either integrator is an affine map y <- A y + B whose coefficients are loop
// invariants (the stage arithmetic of the reference scan, hoisted out of the time loop):
//   Euler, S substeps of h = dt/S (odeint, pkpd/utils.py:68-94): y <- (1 + h be) y + h al, S times;
//   RK4, S steps: k1..k4 of the linear RHS give y <- R(z) y + h al P(z), z = h be,
//     R = 1 + z + z^2/2 + z^3/6 + z^4/24,  P = 1 + z/2 + z^2/6 + z^3/24, composed S times.
// The time loop is then one dependent FMA per step instead of ~10 (the RK4 chain's latency, not
// HBM, bounded small cohorts: DESIGN.md §5).  Results agree with the stage-by-stage evaluation to
// fp64 rounding (tests: rtol 1e-11 against the oracle's explicit stages).
__device__ __forceinline__ void interval_propagator(int method, int substeps, double h, double al, double be,
                                                    double& A, double& B) {
  double a1, b1;
  if (method == INSITE_METHOD_EULER) {
    a1 = fma(h, be, 1.0);
    b1 = h * al;
  } else {
    const double z = h * be;
    const double P = fma(z, fma(z, fma(z, 1.0 / 24.0, 1.0 / 6.0), 0.5), 1.0);  // 1 + z/2 + z^2/6 + z^3/24
    a1 = fma(z, P, 1.0);                                                        // R = 1 + z P
    b1 = h * al * P;
  }
  A = 1.0;
  B = 0.0;
  for (int s = 0; s < substeps; ++s) {
    B = fma(a1, B, b1);
    A *= a1;
  }
}

// Per-lane arm bytes of one 32-step tile, loaded straight from the lane's own row (32 contiguous
// bytes; AV = bytes per load instruction) through a range-checked buffer descriptor.
template <int AV, int KT>
struct ArmTile {
  static constexpr int NW = KT / 4;
  unsigned w[NW];
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t rs, unsigned off) {
    if constexpr (AV == 16) {
#pragma unroll
      for (int k = 0; k < NW / 4; ++k) {
        const u32x4 a = __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16 * k, 0, 0);
        w[4 * k] = a.x; w[4 * k + 1] = a.y; w[4 * k + 2] = a.z; w[4 * k + 3] = a.w;
      }
    } else if constexpr (AV == 4) {
#pragma unroll
      for (int k = 0; k < NW; ++k) w[k] = __builtin_amdgcn_raw_buffer_load_b32(rs, off + 4 * k, 0, 0);
    } else {
#pragma unroll
      for (int k = 0; k < NW; ++k) {
        unsigned v = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) v |= (unsigned)__builtin_amdgcn_raw_buffer_load_b8(rs, off + 4 * k + q, 0, 0) << (8 * q);
        w[k] = v;
      }
    }
  }
  __device__ __forceinline__ int at(int i) const { return (int)((w[i >> 2] >> (8 * (i & 3))) & 0xffu); }
};

// Lane = patient, ODE state in registers.  Per 32-step tile: the next tile's arm bytes are
// requested before this tile's stores (vmcnt counts loads and stores in issue order, so a load
// issued after the stores would wait for them), 32 steps are integrated, the [64 x 32] output
// tile is staged in LDS and written as 256-byte row segments (16 B per lane when YV = 2) through a
// range-checked buffer descriptor (rows past N and steps past T are dropped by the hardware).
#ifndef INSITE_RT
#define INSITE_RT 32
#endif
template <int METHOD, int NARM, bool PERROW, int AV, int YV>
__global__ void __launch_bounds__(kBlock) rollout_kernel(RolloutArgs ra, LibDesc lib) {
  constexpr int KT = INSITE_RT;  // steps per output tile (multiple of 16)
  constexpr int kYS = KT + 2;  // LDS row stride in doubles: rows 16-B aligned for 16-B reads
  __shared__ double ysm[kWavesPerBlock * kWave * kYS];
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);  // wave-uniform (SGPR)
  double* yt = ysm + wid * (kWave * kYS);

  const int64_t p0 = ((int64_t)blockIdx.x * kWavesPerBlock + wid) * kWave;
  if (p0 >= ra.N) return;  // whole wave idle (no block-level sync below)
  const int64_t p = p0 + lane;
  const bool active = p < ra.N;
  const int64_t pc = active ? p : ra.N - 1;
  const int64_t nrows = ra.N - p0 < kWave ? ra.N - p0 : kWave;
  const __amdgpu_buffer_rsrc_t ars =
      __builtin_amdgcn_make_buffer_rsrc((void*)(ra.arm + p0 * ra.lda), (short)0, (int)(nrows * ra.lda), 0x00020000);
  const __amdgpu_buffer_rsrc_t yrs =
      __builtin_amdgcn_make_buffer_rsrc((void*)(ra.y + p0 * ra.ldy), (short)0, (int)(nrows * ra.ldy * 8), 0x00020000);
  const unsigned arow = (unsigned)(lane * ra.lda);

  ArmTile<AV, KT> cur, nxt;
  cur.load(ars, arow);

  // ---- prologue: f_a(y) = alpha_a + beta_a * y for this patient's statics ----
  double uu[INSITE_MAX_STATICS];
#pragma unroll
  for (int t = 0; t < INSITE_MAX_STATICS; ++t) {
    const double q = ra.u[pc * lib.U + (t < lib.U ? t : 0)];
    uu[t] = (active && t < lib.U) ? q : 0.0;
  }
  double alpha[NARM], beta[NARM];  // padded arm slots (n_arms = 3 -> NARM = 4) stay 0
  affine_rates<NARM>(lib, ra.coef + (PERROW ? pc * ra.coef_stride : 0), ra.A, ra.drop, uu, alpha, beta);
  const double y0 = ra.y0[pc];
  double y = active ? y0 : 0.0;
  const double h = ra.dt / (double)ra.substeps;
  const double h2 = 0.5 * h;
  const double h6 = h / 6.0;

#ifndef INSITE_ROLLOUT_STAGEWISE
  double PA[NARM], PB[NARM];
#pragma unroll
  for (int a = 0; a < NARM; ++a) interval_propagator(METHOD, ra.substeps, h, alpha[a], beta[a], PA[a], PB[a]);
  auto step = [&](int a) {
    double A = PA[0], B = PB[0];
#pragma unroll
    for (int aa = 1; aa < NARM; ++aa) {
      A = (a == aa) ? PA[aa] : A;
      B = (a == aa) ? PB[aa] : B;
    }
    y = fma(A, y, B);
  };
#else
  auto step = [&](int a) {
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
  };
#endif

  for (int t0 = 0; t0 < ra.T; t0 += KT) {
#ifndef INSITE_ABLATE_NOARM
    if (t0 + KT < ra.T) nxt.load(ars, arow + (unsigned)(t0 + KT));
#endif
    if (t0 + KT <= ra.T) {
#pragma unroll
      for (int i = 0; i < KT; ++i) {
        step(cur.at(i));
        yt[lane * kYS + i] = y;
      }
    } else {
#pragma unroll
      for (int i = 0; i < KT; ++i) {
        if (t0 + i < ra.T) {
          step(cur.at(i));
          yt[lane * kYS + i] = y;
        }
      }
    }
    wave_lds_sync();
#ifdef INSITE_ABLATE_NOSTORE
    if (yt[lane * kYS] == 12345.678) ra.y[p] = y;  // keep the tile live
    continue;
#endif
    if constexpr (YV == 2) {  // 16 lanes x 16 B per row segment, 4 rows per instruction
      constexpr int LPR = KT / 2;        // lanes per row segment (16 B each)
      constexpr int RPI = kWave / LPR;   // rows per instruction
#pragma unroll
      for (int j = 0; j < kWave / RPI; ++j) {
        const int r = RPI * j + lane / LPR;
        const int c = (lane % LPR) * 2;
        const double2 v = *reinterpret_cast<const double2*>(yt + r * kYS + c);
        const unsigned off = (t0 + c < ra.T) ? (unsigned)((r * ra.ldy + t0 + c) * 8) : kOOB;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), yrs, off, 0, kStoreAux);
      }
    } else {  // 32 lanes x 8 B per row segment, 2 rows per instruction
      constexpr int LPR = KT;            // lanes per row segment (8 B each)
      constexpr int RPI = kWave / LPR;
#pragma unroll
      for (int j = 0; j < kWave / RPI; ++j) {
        const int r = RPI * j + lane / LPR;
        const int c = lane % LPR;
        const double v = yt[r * kYS + c];
        const unsigned off = (t0 + c < ra.T) ? (unsigned)((r * ra.ldy + t0 + c) * 8) : kOOB;
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), yrs, off, 0, kStoreAux);
      }
    }
    wave_lds_sync();
#pragma unroll
    for (int k = 0; k < KT / 4; ++k) cur.w[k] = nxt.w[k];
  }
}

// Time-major rollout (layout INSITE_LAYOUT_TIME_MAJOR): arm[k * lda + r], y[k * ldy + r].  Lane =
// PPL adjacent patients; per step the wave reads 64*PPL contiguous arm bytes and writes 512*PPL
// contiguous bytes of y — fully coalesced, no LDS staging.  Steps run in groups of kTG; the arm
// bytes of the next group are prefetched into a register ring while the current group integrates,
// and every buffer access is unconditional: the per-group descriptors' num_records clip the
// prefetch and the stores at step T (the tail group integrates a few dead steps whose stores the
// hardware drops), and inactive lanes carry an out-of-range offset.  So vmcnt waits are exact
// (never a drain of the outstanding stores).  With PPL = 2 every lane advances two independent
// RK4/Euler chains, doubling the instruction-level parallelism.
#ifndef INSITE_TG
#define INSITE_TG 16
#endif
constexpr int kTG = INSITE_TG;  // steps per group = arm prefetch distance
constexpr int64_t kTmMaxLd = ((int64_t)1 << 31) / (8 * kTG);  // group offsets stay below 2^31

// AFMT: kArmByte (one int8 per lane), kArmDword (the aligned dword holding the lane's PPL int8
// arms), kArmBits (time-major bitmask, n_arms <= 2: bit r & 31 of word r >> 5 of the step row).
constexpr int kArmByte = 0, kArmDword = 1, kArmBits = 2;

// Bit-packed arms, one patient per lane (the C2 / north-star layout): the 64-patient tile `tile`, its
// 32-step arm groups [g_begin, g_end).  Arm bits 32 steps at a time: lane l loads word (k0 + (l & 31),
// p0/32 + (l >> 5)) of the [T, N/32] mask (one 256-B request per wave), and a 32x32 bit transpose per
// half-wave leaves the lane's own 32 steps in one register.  Groups are requested kAG groups (128
// steps) ahead into compile-time ring slots, so the time loop never waits on arm data; per step it is
// one select + one FMA + one 512-B store per wave.  A range that starts inside the trajectory
// (g_begin > 0: the fused step kernel's balanced split of tiles x groups over waves) integrates the
// groups before it without storing them -- the same FMA sequence from y0, so the stored states are
// bitwise those of a whole-trajectory pass (32 FMAs per skipped group against 32 x 512 B of stores).
constexpr int kRollGS = 32;  // steps per arm group
// PR: 0 = one global model (ra.coef [A, F]), 1 = per-patient rows (ra.coef + p * coef_stride), 2 = the
// factual arm's row refitted in the prologue from the patient's moments (RefitArgs rf; C4's fit folded into
// its rollout: no per-patient coefficient round trip through HBM, one launch less).
// SR (step range): g_begin / g_end are STEPS [k_begin, k_end) instead of groups -- the stored steps of a range cut
// at any step (the deferred step's step-balanced rollout ranges); earlier steps of the first group integrate only.
// One 32-step group of a tile's arm bits, steps [k0, min(k0 + kRollGS, kend)) (empty past kend: returns 0).
// time-major bits [T, lda words] (lda > 0): a step's 2 words of this tile share a 128-B line with 15 other tiles'
// -- in a 1M-patient cohort those lines leave the XCD's L2 between the tiles' waves, ~16x the arm bytes re-fetched
// (PMC: 1.12x of the north-star step's algorithmic bytes).  Tile-major bits (lda < 0, INSITE_ARM_BITS_TILE_MAJOR:
// [ceil(N/64)][-lda steps][2 words]): a group's 32 steps of one tile are 256 contiguous bytes, read whole by this wave
__device__ __forceinline__ unsigned roll_arm_group_load(const RolloutArgs& ra, const int64_t tile, const int lane,
                                                        const int k0, const int kend) {
  const int64_t p0 = tile * kWave;
  const int nvalid = (int)(ra.N - p0 < kWave ? ra.N - p0 : kWave);
  const bool atile = ra.lda < 0;
  const int64_t arow = atile ? 8 : ra.lda * 4;  // bytes per step row
  const int64_t abase = atile ? tile * (-ra.lda) * 8 : (p0 >> 5) * 4;
  const int arec_tail = atile ? (nvalid > 32 ? 8 : 4) : ((nvalid + 31) >> 5) * 4;
  const unsigned goff = (unsigned)((lane & 31) * arow + (lane >> 5) * 4);
  const int rows = kend - k0 < kRollGS ? kend - k0 : kRollGS;
  const int bytes = rows > 0 ? (int)((int64_t)(rows - 1) * arow + arec_tail) : 0;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(ra.arm + (int64_t)(rows > 0 ? k0 : 0) * arow + abase), (short)0, bytes, 0x00020000);
  return __builtin_amdgcn_raw_buffer_load_b32(rs, goff, 0, 0);
}
constexpr int kRollAG = 4;  // arm groups in flight (the rollout's arm ring)
#ifndef INSITE_ROLL_SMASK
#define INSITE_ROLL_SMASK 1  // 2-arm bit rollouts: the step's arm bits as the lane mask (rollout_bits_range)
#endif
// A rollout range's per-lane inputs, requested ahead (rollout_units: the NEXT range's before this range's stores):
// vmcnt counts stores too and completes in order, so inputs loaded at a range's start made the wave wait for every
// store of the previous range still in flight -- one drained store queue per tile change.
struct RollPre {
  double u[INSITE_MAX_STATICS];
  double y0;
  unsigned ar[kRollAG];
};
__device__ __forceinline__ void roll_pre_issue(const RolloutArgs& ra, const LibDesc& lib, const int lane,
                                               const int64_t tile, const int g_end, RollPre& pr) {
  const int64_t p = tile * kWave + lane;
  const int64_t pc = p < ra.N ? p : ra.N - 1;
#pragma unroll
  for (int t = 0; t < INSITE_MAX_STATICS; ++t) pr.u[t] = ra.u[pc * lib.U + (t < lib.U ? t : 0)];
  pr.y0 = ra.y0[pc];
  const int kend = g_end * kRollGS < ra.T ? g_end * kRollGS : ra.T;
  if (INSITE_ROLL_SMASK == 1 && (ra.lda < 0 || 2 * tile + 1 < ra.lda)) return;  // (scalar step masks: no arm groups)
#pragma unroll
  for (int d = 0; d < kRollAG; ++d) pr.ar[d] = roll_arm_group_load(ra, tile, lane, d * kRollGS, kend);
}

// PF (PR = 0, SR = false): the lane's statics, y0 and first arm groups come from *pre (roll_pre_issue) and the
// global coefficient rows from *cvp (loaded once per wave) -- the same values, no loads at the range's start
template <int METHOD, int NARM, int PR, bool SR = false, bool PF = false>
__device__ __forceinline__ void rollout_bits_range(const RolloutArgs& ra, const LibDesc& lib, const int lane,
                                                   const int64_t tile, const int g_begin, const int g_end,
                                                   const RefitArgs rf = RefitArgs{}, const RollPre* pre = nullptr,
                                                   const double (*cvp)[NARM][INSITE_MAX_TERMS] = nullptr) {
  static_assert(!PF || (PR == 0 && !SR), "prefetched inputs: the global-coefficient range form");
  // rf by value: the address of the kernel's by-value argument would put a copy of it in scratch
  constexpr bool PERROW = PR == 1;
  const int64_t p0 = tile * kWave;
  const int64_t p = p0 + lane;
  const bool act = p < ra.N;
  const int64_t pc = act ? p : ra.N - 1;
  double PA[NARM], PB[NARM], y;
  {
    double uu[INSITE_MAX_STATICS];
#pragma unroll
    for (int t = 0; t < INSITE_MAX_STATICS; ++t) {
      const double v = PF ? pre->u[t] : ra.u[pc * lib.U + (t < lib.U ? t : 0)];
      uu[t] = (act && t < lib.U) ? v : 0.0;
    }
    double al[NARM], be[NARM];
    if constexpr (PR == 2) {
      double cv[NARM][INSITE_MAX_TERMS];
      load_coef_rows<NARM>(lib, rf.gcoef, ra.A, cv);
      const int af = rf.farm[pc];
      int L = rf.rows[pc];
      if (L > rf.n_steps) L = rf.n_steps;
      const bool fit = act && af >= 0 && af < ra.A;
      const double M[3] = {rf.mom[pc * 5 + 0], rf.mom[pc * 5 + 1], rf.mom[pc * 5 + 2]};
      const double Sd = rf.mom[pc * 5 + 3], Sdx = rf.mom[pc * 5 + 4];
      double c[INSITE_MAX_TERMS];
      unsigned init = 0u;
      const int it = patient_refit<INSITE_MAX_TERMS, false>(lib, uu, M, Sd, Sdx, L, rf.gcoef + (fit ? af : 0) * lib.F,
                                                             rf.sp, c, init);
#pragma unroll
      for (int a = 0; a < NARM; ++a)
#pragma unroll
        for (int j = 0; j < INSITE_MAX_TERMS; ++j) cv[a][j] = (fit && a == af) ? c[j] : cv[a][j];
      // (compile-time column loops: a run-time index into c[] would move it to scratch)
      if (act && rf.coef_out) {
#pragma unroll
        for (int a = 0; a < NARM; ++a)
#pragma unroll
          for (int j = 0; j < INSITE_MAX_TERMS; ++j)
            if (a < ra.A && j < lib.F)
              rf.coef_out[(p * ra.A + a) * lib.F + j] = (fit && a == af) ? c[j] : rf.gcoef[a * lib.F + j];
      }
      if (act && fit && rf.mask_out) {
#pragma unroll
        for (int j = 0; j < INSITE_MAX_TERMS; ++j)
          if (j < lib.F)
            rf.mask_out[p * lib.F + j] = (int8_t)(L < 5 ? (init >> j) & 1u : (fabs(c[j]) > 1e-14 ? 1u : 0u));
      }
      if (act && rf.iters_out) rf.iters_out[p] = fit ? it : -2;
      affine_rates_regs<NARM>(lib, cv, ra.A, ra.drop, uu, al, be);
    } else if constexpr (PF) {
      affine_rates_regs<NARM>(lib, *cvp, ra.A, ra.drop, uu, al, be);
    } else {
      affine_rates<NARM>(lib, ra.coef + (PERROW ? pc * ra.coef_stride : 0), ra.A, ra.drop, uu, al, be);
    }
    const double h = ra.dt / (double)ra.substeps;
#ifndef INSITE_ROLLOUT_STAGEWISE
#pragma unroll
    for (int a = 0; a < NARM; ++a) interval_propagator(METHOD, ra.substeps, h, al[a], be[a], PA[a], PB[a]);
#else  // ablation: PA / PB carry the rates, every step evaluates the method's stages explicitly
#pragma unroll
    for (int a = 0; a < NARM; ++a) {
      PA[a] = al[a];
      PB[a] = be[a];
    }
#endif
    const double v0 = PF ? pre->y0 : ra.y0[pc];
    y = act ? v0 : 0.0;
  }
  const int nvalid = (int)(ra.N - p0 < kWave ? ra.N - p0 : kWave);
  const unsigned yoff = act ? (unsigned)(lane * 8) : kOOB;
  const int kend = SR ? (g_end < ra.T ? g_end : ra.T)
                      : (g_end * kRollGS < ra.T ? g_end * kRollGS : ra.T);  // one past the last step of the range
  const int kbeg = SR ? g_begin : g_begin * kRollGS;                   // first stored step
  auto y_rsrc = [&](int k0) {  // rows [k0, min(k0 + kTG, kend)); empty (all stores dropped) past kend
    const int rows = kend - k0 < kTG ? kend - k0 : kTG;
    return __builtin_amdgcn_make_buffer_rsrc((void*)(ra.y + (int64_t)(rows > 0 ? k0 : 0) * ra.ldy + p0), (short)0,
                                             rows > 0 ? (int)(((int64_t)(rows - 1) * ra.ldy + nvalid) * 8) : 0,
                                             0x00020000);
  };
  constexpr int kAG = kRollAG;
  auto grp_load = [&](int k0) -> unsigned { return roll_arm_group_load(ra, tile, lane, k0, kend); };
#ifndef INSITE_ABL_ROLL
#define INSITE_ABL_ROLL 0  // profiling ablations only: 1 = no arm selects (arm 0 always), 2 = no prefix re-integration
#endif
#ifndef INSITE_ROLLOUT_STAGEWISE
  auto step = [&](int a) {
    double A = PA[0], B = PB[0];
#pragma unroll
    for (int aa = 1; aa < (INSITE_ABL_ROLL == 1 ? 1 : NARM); ++aa) {
      A = (a == aa) ? PA[aa] : A;
      B = (a == aa) ? PB[aa] : B;
    }
    y = fma(A, y, B);
  };
#else
  const double hs = ra.dt / (double)ra.substeps, hs2 = 0.5 * hs, hs6 = hs / 6.0;
  auto step = [&](int a) {  // the reference's stage arithmetic: Euler sub-steps / classical RK4 stages
    double al = PA[0], be = PB[0];
#pragma unroll
    for (int aa = 1; aa < NARM; ++aa) {
      al = (a == aa) ? PA[aa] : al;
      be = (a == aa) ? PB[aa] : be;
    }
    for (int s = 0; s < ra.substeps; ++s) {
      if constexpr (METHOD == INSITE_METHOD_EULER) {
        y = fma(fma(be, y, al), hs, y);
      } else {
        const double k1 = fma(be, y, al);
        const double k2 = fma(be, fma(hs2, k1, y), al);
        const double k3 = fma(be, fma(hs2, k2, y), al);
        const double k4 = fma(be, fma(hs, k3, y), al);
        y = fma(hs6, (k1 + 2.0 * k2) + (2.0 * k3 + k4), y);
      }
    }
  };
#endif
#if INSITE_ROLL_SMASK == 1 && !defined(INSITE_ROLLOUT_STAGEWISE)
  if constexpr (NARM == 2 && !SR) {
    // A step's 64 arm bits of this tile (bit l = patient p0 + l: the two 32-patient words as they lie in either
    // layout) ARE the wave's lane mask for the arm-1 select: one scalar load per step straight into an SGPR pair,
    // prefetched kTG steps ahead, and v_cndmask on it (inverse ballot) -- no per-lane bit transpose, extraction or
    // compare; per step two independent FMAs (arm 0 / arm 1, the same operands as the select-then-FMA form, so y is
    // bitwise unchanged) and a 64-bit select.  `wide`: both words exist (not so for a last tile of <= 32 patients in a
    // time-major [T, ceil(N/32)] array, which takes the per-lane form below).
    const bool wide = ra.lda < 0 || 2 * tile + 1 < ra.lda;  // uniform
    if (wide) {
      if (kend <= 0) return;
      typedef const __attribute__((address_space(4))) uint32_t* cu32p;  // scalar (constant) loads: arm bits are input
      const char* ab = reinterpret_cast<const char*>(ra.arm) + (ra.lda < 0 ? tile * (-ra.lda) * 8 : (p0 >> 5) * 4);
      const int64_t arow = ra.lda < 0 ? 8 : ra.lda * 4;
      const int klast = kend - 1;
      auto mload = [&](int k) -> uint64_t {  // clamped at the range's last step (the mask of steps past it is unused)
        if (INSITE_ABL_ROLL == 3) return 0x5555555555555555ull << (k & 1);  // (ablation: no mask loads)
        const cu32p q = (cu32p)(ab + (int64_t)(k < klast ? k : klast) * arow);
        return (uint64_t)q[0] | ((uint64_t)q[1] << 32);
      };
      const double A0 = PA[0], A1 = PA[1], B0 = PB[0], B1 = PB[1];
      auto step2 = [&](uint64_t m) {
        const bool b = __builtin_amdgcn_inverse_ballot_w64(m);
        const double y0 = fma(A0, y, B0), y1 = fma(A1, y, B1);
        y = b ? y1 : y0;
      };
      // the next chunk's masks are requested after the chunk's first step has used its own: scalar loads return out of
      // order, so a use of mc[] with loads outstanding waits for all of them (lgkmcnt(0)); issued behind that first use
      // (sched_barrier) they stay in flight for the rest of the chunk.  (Two mask sets used in turn instead of the
      // copy raised the kernel's SGPR spills into this loop.)
      uint64_t mc[kTG], mn[kTG];
#pragma unroll
      for (int i = 0; i < kTG; ++i) mc[i] = mload(i);
      for (int k0 = 0; k0 < kend; k0 += kTG) {
        auto next_masks = [&]() {
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int i = 0; i < kTG; ++i) mn[i] = mload(k0 + kTG + i);
          __builtin_amdgcn_sched_barrier(0);
        };
        if (k0 >= kbeg) {  // uniform: stored steps (kbeg is a multiple of kRollGS)
          const __amdgpu_buffer_rsrc_t ys = y_rsrc(k0);
#pragma unroll
          for (int i = 0; i < kTG; ++i) {
            step2(mc[i]);
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, y), ys, yoff + (unsigned)(i * ra.ldy * 8), 0,
                                                  kStoreAux);
            if (i == 0) next_masks();
          }
        } else {  // before the range: integrate only
#pragma unroll
          for (int i = 0; i < kTG; ++i) {
            if (INSITE_ABL_ROLL != 2) step2(mc[i]);
            if (i == 0) next_masks();
          }
        }
#pragma unroll
        for (int i = 0; i < kTG; ++i) mc[i] = mn[i];
      }
      return;
    }
  }
#endif
  unsigned aring[kAG];
#pragma unroll
  for (int d = 0; d < kAG; ++d) aring[d] = PF ? pre->ar[d] : grp_load(d * kRollGS);
#if INSITE_ROLL_SMASK == 2 && !defined(INSITE_ROLLOUT_STAGEWISE)
  if constexpr (NARM == 2) {
    // the group's raw words as loaded (lane l: step l & 31, patients 32 (l >> 5) ..): step i's lane mask is lanes i
    // and 32 + i, read into an SGPR pair (two v_readlane) -- the words arrive kAG groups ahead through the vector path
    const double A0 = PA[0], A1 = PA[1], B0 = PB[0], B1 = PB[1];
    auto step2 = [&](uint64_t m) {
      const bool b = __builtin_amdgcn_inverse_ballot_w64(m);
      const double y0 = fma(A0, y, B0), y1 = fma(A1, y, B1);
      y = b ? y1 : y0;
    };
    auto mask_of = [&](unsigned wv, int i) -> uint64_t {
      return (uint64_t)(unsigned)__builtin_amdgcn_readlane((int)wv, i) |
             ((uint64_t)(unsigned)__builtin_amdgcn_readlane((int)wv, 32 + i) << 32);
    };
    for (int k0 = 0; k0 < kend;) {
#pragma unroll
      for (int d = 0; d < kAG; ++d) {
        if (k0 < kend) {  // uniform
          const unsigned wv = aring[d];
          aring[d] = grp_load(k0 + kAG * kRollGS);
          if (SR ? k0 + kRollGS > kbeg : k0 >= kbeg) {  // uniform: a stored group
#pragma unroll
            for (int hh = 0; hh < kRollGS / kTG; ++hh) {
              const __amdgpu_buffer_rsrc_t ys = y_rsrc(k0 + hh * kTG);
#pragma unroll
              for (int i = 0; i < kTG; ++i) {
                step2(mask_of(wv, hh * kTG + i));
                const unsigned so = (!SR || k0 + hh * kTG + i >= kbeg) ? yoff + (unsigned)(i * ra.ldy * 8) : kOOB;
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, y), ys, so, 0, kStoreAux);
              }
            }
          } else if (INSITE_ABL_ROLL != 2) {
#pragma unroll
            for (int i = 0; i < kRollGS; ++i) step2(mask_of(wv, i));
          }
          k0 += kRollGS;
        }
      }
    }
    return;
  }
#endif
  for (int k0 = 0; k0 < kend;) {
#pragma unroll
    for (int d = 0; d < kAG; ++d) {
      if (k0 < kend) {  // uniform
        const unsigned wb = bit_transpose32(aring[d], lane);
        aring[d] = grp_load(k0 + kAG * kRollGS);
        if (SR ? k0 + kRollGS > kbeg : k0 >= kbeg) {  // uniform: a stored group
#pragma unroll
          for (int hh = 0; hh < kRollGS / kTG; ++hh) {
            const __amdgpu_buffer_rsrc_t ys = y_rsrc(k0 + hh * kTG);
#pragma unroll
            for (int i = 0; i < kTG; ++i) {
              step((int)((wb >> (hh * kTG + i)) & 1u));
              // SR: steps before kbeg (uniform) store through the dropped offset
              const unsigned so = (!SR || k0 + hh * kTG + i >= kbeg) ? yoff + (unsigned)(i * ra.ldy * 8) : kOOB;
              __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, y), ys, so, 0, kStoreAux);
            }
          }
        } else if (INSITE_ABL_ROLL != 2) {  // a group before the range: integrate only
#pragma unroll
          for (int i = 0; i < kRollGS; ++i) step((int)((wb >> i) & 1u));
        }
        k0 += kRollGS;
      }
    }
  }
}

template <int METHOD, int NARM, bool PERROW, int PPL, int AFMT>
__global__ void __launch_bounds__(kBlock) rollout_tm_kernel(RolloutArgs ra, LibDesc lib) {
  constexpr bool AW4 = AFMT != kArmByte;  // 32-bit ring elements
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);  // wave-uniform (SGPR)
  const int64_t p0 = ((int64_t)blockIdx.x * kWavesPerBlock + wid) * (kWave * PPL);
  if (p0 >= ra.N) return;
  if constexpr (AFMT == kArmBits && PPL == 1) {
    rollout_bits_range<METHOD, NARM, PERROW>(ra, lib, lane, p0 / kWave, 0, (ra.T + kRollGS - 1) / kRollGS);
    return;
  }
  INSITE_TSTAMP(32768 + blockIdx.x * kWavesPerBlock + wid, 0);
  INSITE_TREAL(32768 + blockIdx.x * kWavesPerBlock + wid, 8);
  double y[PPL], alpha[PPL][NARM], beta[PPL][NARM];
  bool act[PPL];
#pragma unroll
  for (int q = 0; q < PPL; ++q) {
    const int64_t p = p0 + PPL * lane + q;
    act[q] = p < ra.N;
    const int64_t pc = act[q] ? p : ra.N - 1;
    double uu[INSITE_MAX_STATICS];
#pragma unroll
    for (int t = 0; t < INSITE_MAX_STATICS; ++t) {
      const double v = ra.u[pc * lib.U + (t < lib.U ? t : 0)];
      uu[t] = (act[q] && t < lib.U) ? v : 0.0;
    }
    affine_rates<NARM>(lib, ra.coef + (PERROW ? pc * ra.coef_stride : 0), ra.A, ra.drop, uu, alpha[q], beta[q]);
    const double v0 = ra.y0[pc];
    y[q] = act[q] ? v0 : 0.0;
  }
  const double h = ra.dt / (double)ra.substeps;
  const double h2 = 0.5 * h;
  const double h6 = h / 6.0;
  const int nvalid = (int)(ra.N - p0 < kWave * PPL ? ra.N - p0 : kWave * PPL);
  // Inactive lanes (only in the last wavefront) store through an offset the hardware drops
  // (kOOB + group offsets stays >= 2^31 > num_records).
  const unsigned yoff = act[0] ? (unsigned)(PPL * lane * 8) : kOOB;

  // Descriptors cover rows [k0, min(k0 + kTG, T)) of a time-major matrix, based at column p0.
  // AW4: each lane loads the aligned dword holding its PPL arm bytes (lanes sharing a dword read
  // the same address) into a plain 32-bit ring, and extracts its bytes at the use.  Narrower ring
  // elements get packed by the compiler, which then waits for every prefetched load at the loop
  // latch.  Requires ld_arm % 4 == 0 and a 4-byte aligned base, so the last row's dword stays
  // inside the allocation; otherwise (AW4 = false) plain byte loads are used.
  static_assert(AW4 || PPL == 1, "several patients per lane need dword arm loads");
  using ArmT = std::conditional_t<AW4, uint32_t, uint8_t>;
  const unsigned abyte = (unsigned)(PPL * lane);  // the lane's first patient, relative to p0
  // byte offset of the lane's arm word within a step row (relative to the wave's base) and the
  // shift that brings its first patient's arm to bit 0
  const unsigned aoff = AFMT == kArmBits ? (abyte >> 5) * 4u : (AW4 ? (abyte & ~3u) : abyte);
  const unsigned ashift = AFMT == kArmBits ? (abyte & 31u) : (AW4 ? 8u * (abyte & 3u) : 0u);
  constexpr unsigned kArmStride = AFMT == kArmBits ? 1u : 8u;  // bit distance between lane patients
  constexpr unsigned kArmMask = AFMT == kArmBits ? 1u : 0xffu;
  // row stride and wave base in bytes (bit rows: lda counts 32-bit words; p0 is a multiple of 64)
  const int64_t arow = AFMT == kArmBits ? ra.lda * 4 : ra.lda;
  const int64_t abase = AFMT == kArmBits ? (p0 >> 5) * 4 : p0;
  const int arec_tail = AFMT == kArmBits ? ((nvalid + 31) >> 5) * 4 : (AW4 ? ((nvalid + 3) & ~3) : nvalid);
  auto arm_rsrc = [&](int k0) {
    const int rows = ra.T - k0 < kTG ? ra.T - k0 : kTG;
    const int bytes = rows > 0 ? (int)((int64_t)(rows - 1) * arow + arec_tail) : 0;
    return __builtin_amdgcn_make_buffer_rsrc((void*)(ra.arm + (int64_t)(rows > 0 ? k0 : 0) * arow + abase), (short)0,
                                             bytes, 0x00020000);
  };
  auto y_rsrc = [&](int k0) {  // rows [k0, min(k0 + kTG, T)); empty (all stores dropped) past T
    const int rows = ra.T - k0 < kTG ? ra.T - k0 : kTG;
    return __builtin_amdgcn_make_buffer_rsrc((void*)(ra.y + (int64_t)(rows > 0 ? k0 : 0) * ra.ldy + p0), (short)0,
                                             rows > 0 ? (int)(((int64_t)(rows - 1) * ra.ldy + nvalid) * 8) : 0,
                                             0x00020000);
  };
  auto load_arm = [&](__amdgpu_buffer_rsrc_t rs, int i) -> ArmT {  // step i of a group
#ifdef INSITE_ABLATE_NOARM
    return (ArmT)(i & 1);
#endif
    const unsigned off = aoff + (unsigned)(i * arow);
    if constexpr (AW4) return __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0);
    else return (ArmT)__builtin_amdgcn_raw_buffer_load_b8(rs, off, 0, 0);
  };
#ifndef INSITE_ROLLOUT_STAGEWISE
  double PA[PPL][NARM], PB[PPL][NARM];
#pragma unroll
  for (int q = 0; q < PPL; ++q)
#pragma unroll
    for (int a = 0; a < NARM; ++a) interval_propagator(METHOD, ra.substeps, h, alpha[q][a], beta[q][a], PA[q][a], PB[q][a]);
  auto step = [&](int q, int a) {
    double A = PA[q][0], B = PB[q][0];
#pragma unroll
    for (int aa = 1; aa < NARM; ++aa) {
      A = (a == aa) ? PA[q][aa] : A;
      B = (a == aa) ? PB[q][aa] : B;
    }
    y[q] = fma(A, y[q], B);
  };
#else
  auto step = [&](int q, int a) {
    double al = alpha[q][0], be = beta[q][0];
#pragma unroll
    for (int aa = 1; aa < NARM; ++aa) {
      al = (a == aa) ? alpha[q][aa] : al;
      be = (a == aa) ? beta[q][aa] : be;
    }
    double yy = y[q];
    if constexpr (METHOD == INSITE_METHOD_EULER) {
      for (int s = 0; s < ra.substeps; ++s) {
        const double f = fma(be, yy, al);
        yy = fma(f, h, yy);
      }
    } else {
      for (int s = 0; s < ra.substeps; ++s) {
        const double k1 = fma(be, yy, al);
        const double k2 = fma(be, fma(h2, k1, yy), al);
        const double k3 = fma(be, fma(h2, k2, yy), al);
        const double k4 = fma(be, fma(h, k3, yy), al);
        yy = fma(h6, (k1 + 2.0 * k2) + (2.0 * k3 + k4), yy);
      }
    }
    y[q] = yy;
  };
#endif

  INSITE_TSTAMP(32768 + blockIdx.x * kWavesPerBlock + wid, 1);
  ArmT ring[kTG];
  {
    const __amdgpu_buffer_rsrc_t rs = arm_rsrc(0);
#pragma unroll
    for (int i = 0; i < kTG; ++i) ring[i] = load_arm(rs, i);
  }
  for (int k0 = 0; k0 < ra.T; k0 += kTG) {
    const __amdgpu_buffer_rsrc_t rsn = arm_rsrc(k0 + kTG);  // empty past T: loads return 0
    const __amdgpu_buffer_rsrc_t ys = y_rsrc(k0);
#pragma unroll
    for (int i = 0; i < kTG; ++i) {
      const unsigned a2 = (unsigned)ring[i] >> ashift;
      // consume ring[i] before its refill is issued: otherwise the scheduler hoists the load, the
      // slot needs two registers and the latch copy waits for the load
      asm volatile("" ::"v"(a2) : "memory");
      ring[i] = load_arm(rsn, i);
#ifndef INSITE_ABLATE_NOCOMPUTE
#pragma unroll
      for (int q = 0; q < PPL; ++q) step(q, (int)((a2 >> (kArmStride * q)) & kArmMask));
#else
#pragma unroll
      for (int q = 0; q < PPL; ++q) y[q] += (double)((a2 >> (kArmStride * q)) & kArmMask);
#endif
      const unsigned off = yoff + (unsigned)(i * ra.ldy * 8);
#ifndef INSITE_ABLATE_NOSTORE
      if constexpr (PPL >= 2) {
        // groups of PPL patients are whole (the launcher requires N % PPL == 0); the last row's
        // columns >= nvalid are clipped by num_records
#pragma unroll
        for (int q2 = 0; q2 < PPL / 2; ++q2) {
          const double2 v = make_double2(y[2 * q2], y[2 * q2 + 1]);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), ys, off + 16u * q2, 0, kStoreAux);
        }
      } else {
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, y[0]), ys, off, 0, kStoreAux);
      }
#else
      if (y[0] == 12345.678) __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, y[0]), ys, off, 0, 0);
#endif
    }
  }
}

// Per-patient refit + rollout in one launch (C4; insite_refit_rollout_moments_f64): wave = 64-patient tile,
// the prologue refits the lane's factual-arm row from its moments (patient_refit, closed-form ridge) and
// the time loop is rollout_bits_range's.  Replaces patient_fit_kernel + the per-row rollout: the
// per-patient coefficient rows (N x A x F doubles written, then read) never touch HBM.
template <int METHOD, int NARM>
__global__ void __launch_bounds__(kBlock) refit_rollout_kernel(RolloutArgs ra, LibDesc lib, RefitArgs rf) {
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int64_t tile = (int64_t)blockIdx.x * kWavesPerBlock + wid;
  if (tile * kWave >= ra.N) return;
  rollout_bits_range<METHOD, NARM, 2>(ra, lib, lane, tile, 0, (ra.T + kRollGS - 1) / kRollGS, rf);
}

// =============================================================================================
// Fused step: the discovery of one cohort and the rollout of another in ONE launch (C2 pipeline)
// =============================================================================================
// A stream of cohorts (the C2 bench; a serving loop) discovers cohort k while it rolls out cohort
// k - 1 with the coefficients that discovery k - 1 wrote.  The two halves are independent HBM streams
// (the gram reads x, the rollout writes y), so one launch runs both at once: blocks [0, gblocks) run
// gram_body (in-launch fixed-order reduction and the fused F = 7 STLSQ, exactly as gram_kernel) and the
// other blocks the bit-arm rollout.  The grid is one resident round (every block persistent), and the
// rollout's work -- 64-patient tiles x 32-step arm groups, tile-major -- is cut into equal contiguous
// ranges, one per rollout wave, so both roles end together whatever the cohort size; a range that
// starts mid-trajectory re-integrates its tile's earlier groups without storing (rollout_bits_range),
// so every stored state is bitwise that of the standalone rollout.  Results do not depend on gblocks
// except through the gram's block count (the fixed-order reduction's association, as for gram_kernel's
// grid).  Replaces, per step, the gram + rollout launch pair on two streams and the events between them.
//
// Serial mode (gblocks == gridDim.x; INSITE_STEP_SERIAL, default): EVERY wave runs its gram range first and
// then rollout work, so the chip reads x with all its waves, then writes y with all of them (no read/write
// mix inside the HBM stream), and the gram's serial tail -- the last block's reduction and STLSQ, ~15 us
// after the last gram wave in the split schedule (profiles/r03/ timelines) -- overlaps the other waves'
// rollout.  The rollout work is a static part (the first INSITE_STEP_DYN_STATIC per mille of the units,
// equal contiguous ranges per wave) and a dynamic remainder of INSITE_STEP_DYN_CHUNK-unit chunks claimed
// with an agent-scope counter, so waves that leave the gram late (the tail block, slow CUs) take fewer
// chunks.  The claim order does not reach the results: every chunk is a rollout_bits_range (bitwise the
// standalone rollout).  Counters rc[0] (claims) / rc[1] (waves done claiming) sit in the workspace header;
// the last wave done resets both, so a launch leaves them zero (the header invariant).
#ifndef INSITE_STEP_DYN_STATIC
#define INSITE_STEP_DYN_STATIC 500
#endif
// The bit-arm rollout of the (tile, arm group) units [q, q1) (tile-major), one rollout_bits_range per tile.
// INSITE_ROLL_PF: every range's inputs requested one range ahead (RollPre), the coefficient rows once per wave.
#ifndef INSITE_ROLL_PF
#define INSITE_ROLL_PF 1
#endif
template <int METHOD>
__device__ __forceinline__ void rollout_units(const RolloutArgs& ra, const LibDesc& lib, const int lane, int64_t q,
                                              const int64_t q1, const int ng) {
#if INSITE_ROLL_PF
  if (q >= q1) return;
  double cv[2][INSITE_MAX_TERMS];
  load_coef_rows<2>(lib, ra.coef, ra.A, cv);
  int64_t tile = q / ng;
  int gb = (int)(q - tile * ng);
  int ge = q1 - q < (int64_t)(ng - gb) ? gb + (int)(q1 - q) : ng;
  RollPre cur;
  roll_pre_issue(ra, lib, lane, tile, ge, cur);
  for (;;) {
    const int64_t qn = q + (ge - gb);
    const bool more = qn < q1;  // uniform
    const int64_t tn = more ? qn / ng : 0;
    const int gbn = (int)(qn - tn * ng);
    const int gen = q1 - qn < (int64_t)(ng - gbn) ? gbn + (int)(q1 - qn) : ng;
    RollPre nxt;
    if (more) roll_pre_issue(ra, lib, lane, tn, gen, nxt);  // before this range's stores
    rollout_bits_range<METHOD, 2, 0, false, true>(ra, lib, lane, tile, gb, ge, RefitArgs{}, &cur, &cv);
    if (!more) break;
    cur = nxt;
    q = qn;
    tile = tn;
    gb = gbn;
    ge = gen;
  }
#else
  while (q < q1) {
    const int64_t tile = q / ng;
    const int gb = (int)(q - tile * ng);
    const int ge = q1 - q < (int64_t)(ng - gb) ? gb + (int)(q1 - q) : ng;
    rollout_bits_range<METHOD, 2, false>(ra, lib, lane, tile, gb, ge);
    q += ge - gb;
  }
#endif
}
// The bit-arm rollout of the (tile, step) pairs [s, s1) (tile-major, T steps a tile): one step-range
// rollout_bits_range per tile.  Every wave of the deferred step stores the same number of steps (+-1), where the
// (tile, 32-step group) units left ranges of 10 or 11 units with one or two 8-step tail groups among them: 272 to
// 328 stored steps per wave at C2's shape.
template <int METHOD>
__device__ __forceinline__ void rollout_steps(const RolloutArgs& ra, const LibDesc& lib, const int lane, int64_t s,
                                              const int64_t s1) {
  while (s < s1) {
    const int64_t tile = s / ra.T;
    const int kb = (int)(s - tile * ra.T);
    const int ke = s1 - s < (int64_t)(ra.T - kb) ? kb + (int)(s1 - s) : ra.T;
    rollout_bits_range<METHOD, 2, false, true>(ra, lib, lane, tile, kb, ke);
    s += ke - kb;
  }
}
// Units [S, units) in chunks of `chunk` units claimed with the agent-scope counter rc[0] (the next claim in flight
// while a chunk is stored); rc[1] counts the waves done claiming, and the last of the `waves` participants resets
// both.  Which wave stores a chunk never reaches y (every chunk is a rollout_bits_range).
template <int METHOD>
__device__ __forceinline__ void rollout_claimed(const RolloutArgs& ra, const LibDesc& lib, const int lane, const int64_t S,
                                                const int64_t units, const int ng, const int chunk,
                                                unsigned* __restrict__ rc, const int64_t waves) {
  const int64_t n_chunks = (units - S + chunk - 1) / chunk;
  auto claim = [&]() -> unsigned {  // lane 0 holds the claimed chunk index (read when it is needed)
    unsigned v = 0u;
    if (lane == 0) v = __hip_atomic_fetch_add(rc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return v;
  };
  unsigned nxt = claim();
  for (;;) {
    const int64_t c = (int64_t)__builtin_amdgcn_readfirstlane(nxt);
    if (c >= n_chunks) break;
    nxt = claim();
    const int64_t q = S + c * chunk;
    rollout_units<METHOD>(ra, lib, lane, q, q + chunk < units ? q + chunk : units, ng);
  }
  if (lane == 0) {
    const unsigned t = __hip_atomic_fetch_add(rc + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == (unsigned)waves - 1u) {
      __hip_atomic_store(rc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(rc + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}
#ifndef INSITE_STEP_DYN_CHUNK
#define INSITE_STEP_DYN_CHUNK 2
#endif
constexpr int kStepRcnt = 96;  // rc = cnt + kStepRcnt (the gram tail uses cnt[0 .. 64])
#ifndef INSITE_STEP_WPE
#define INSITE_STEP_WPE 2  // waves per SIMD the step kernel's register budget is sized for
#endif
template <bool SMOOTH, int METHOD>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(INSITE_STEP_WPE)))
step_kernel(const double* __restrict__ x, int64_t ldx, int n_steps, const double* __restrict__ u,
            const int8_t* __restrict__ arm, const int32_t* __restrict__ rows, int64_t N, int seg, int n_seg,
            GramW w, LibDesc lib, double* __restrict__ partial, unsigned* __restrict__ cnt, GramOut out,
            RolloutArgs ra, int gblocks) {
  __shared__ double smem[kGramSmem];
  if (gblocks == (int)gridDim.x) {  // serial mode: gram range, then rollout (static part + claimed chunks)
    gram_body<1, 2, SMOOTH, true, true, 0, 7>((int)blockIdx.x, gblocks, smem, x, ldx, n_steps, u, arm, rows, N,
                                                 seg, n_seg, w, lib, partial, cnt, out);
    const int lane = threadIdx.x & (kWave - 1);
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    const int64_t RW = (int64_t)gridDim.x * kWavesPerBlock;
    const int64_t rw = (int64_t)blockIdx.x * kWavesPerBlock + wid;
    INSITE_TREAL(32768 + rw, 8);
    const int ng = (ra.T + kRollGS - 1) / kRollGS;
    const int64_t units = (ra.N + kWave - 1) / kWave * ng;  // (tile, arm group) pairs, tile-major
    const int64_t S = units * INSITE_STEP_DYN_STATIC / 1000;
    rollout_units<METHOD>(ra, lib, lane, rw * S / RW, (rw + 1) * S / RW, ng);
    rollout_claimed<METHOD>(ra, lib, lane, S, units, ng, INSITE_STEP_DYN_CHUNK, cnt + kStepRcnt, RW);
    INSITE_TSTAMP(32768 + rw, 0);
    INSITE_TREAL(32768 + rw, 9);
    return;
  }
  if ((int)blockIdx.x < gblocks) {
    gram_body<1, 2, SMOOTH, true, true, 0, 7>((int)blockIdx.x, gblocks, smem, x, ldx, n_steps, u, arm, rows, N,
                                                 seg, n_seg, w, lib, partial, cnt, out);
    return;
  }
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int64_t RW = (int64_t)(gridDim.x - gblocks) * kWavesPerBlock;
  const int64_t rw = (int64_t)((int)blockIdx.x - gblocks) * kWavesPerBlock + wid;
  INSITE_TREAL(32768 + rw, 8);
  const int ng = (ra.T + kRollGS - 1) / kRollGS;
  const int64_t units = (ra.N + kWave - 1) / kWave * ng;  // (tile, arm group) pairs, tile-major
  int64_t q = rw * units / RW;
  const int64_t q1 = (rw + 1) * units / RW;
  while (q < q1) {
    const int64_t tile = q / ng;
    const int gb = (int)(q - tile * ng);
    const int ge = q1 - q < (int64_t)(ng - gb) ? gb + (int)(q1 - q) : ng;
    rollout_bits_range<METHOD, 2, false>(ra, lib, lane, tile, gb, ge);
    q += ge - gb;
  }
  INSITE_TSTAMP(32768 + rw, 0);
  INSITE_TREAL(32768 + rw, 9);
}

// The fused step with the discovery's finalisation deferred to the next launch (insite_fit_rollout_deferred_f64).
// In step_kernel the last gram block's reduction and STLSQ run after every other gram wave has ended (14 us of a
// 75 us C2 step in the phase timelines, profiles/r03/): the launch cannot end before that serial tail.  Here the
// gram blocks [0, gblocks) only stream cohort k and leave their compact partials in `part_cur`; block gblocks
// reduces the partials the PREVIOUS launch left in `part_prev` (cohort k-1: G|b, STLSQ -> coefficients) while
// the others stream; the remaining blocks roll out a cohort with coefficients finalised one launch earlier
// still (cohort k-2 in a stream).  Nothing in the launch waits on anything else in it: no counters, no tail.
// A/B knobs: INSITE_DEF_RSTATIC (per mille of the rollout units split statically; below 1000 the rest is claimed
// in INSITE_DEF_RCHUNK-unit chunks through the counters in the workspace header), INSITE_DEF_GPRIO (s_setprio of
// the gram waves).
#ifndef INSITE_DEF_RSTATIC
#define INSITE_DEF_RSTATIC 1000
#endif
#ifndef INSITE_DEF_RCHUNK
#define INSITE_DEF_RCHUNK 1
#endif
#ifndef INSITE_DEF_GPRIO
#define INSITE_DEF_GPRIO 0
#endif
// INSITE_DEF_DYN: the claimed gram tail (DynGram) -- 0 never, 1 always, 2 (default) by size: a launch takes the claimed
// instantiation when its gram waves stream at least INSITE_DEF_DYN_MIN (tile, kGT-step group) units each.  Measured
// (profiles/r06/dyn_ns/, dyn_c2/): at the north-star 1M x 500 (488 units a wave; the pieces are whole tiles, the slot's
// row budget) the claimed tail is 4-10 % faster, box to box; at C2's 100k x 200 (20 units a wave) 20-35 % slower -- the
// per-piece warm-ups, contractions and partial stores and the finaliser's ~1 MB of piece partials (one block,
// latency-bound beside the streaming) cost more than the ~10 us of spread they recover.  INSITE_DEF_DYN_TAIL: per mille
// of the tiles claimed (250: 1.686-1.690 vs 1.700-1.702 ms at 150, three runs each); INSITE_DEF_DYN_PG: kGT-step
// groups per piece (coarsened to fit the slot).
#ifndef INSITE_DEF_DYN
#define INSITE_DEF_DYN 2
#endif
#ifndef INSITE_DEF_DYN_MIN
#define INSITE_DEF_DYN_MIN 128
#endif
#ifndef INSITE_DEF_DYN_TAIL
#define INSITE_DEF_DYN_TAIL 250
#endif
#ifndef INSITE_DEF_DYN_PG
#define INSITE_DEF_DYN_PG 2
#endif
// Each slot's header records what its partials are: the launch that streams a slot writes
// {magic, gram blocks, entries} there, and the finalisation sums exactly the recorded number of partials, so a
// caller that changes the method / fd between calls (and with them the default block split) still gets the
// right G|b; a slot that was never streamed (or holds another system) is flagged instead of summed.
constexpr int kSlotRec = 112;  // unsigned index into the slot's 512-B header (counters use [0, 98))
constexpr unsigned kSlotMagic = 0x1E5D0A7Eu;
static_assert((kSlotRec + 4) * sizeof(unsigned) <= 512, "slot record inside the workspace header");
static_assert(kDynRecDone >= kSlotRec + 4 && (kDynRecP + 1) * sizeof(unsigned) <= 512, "DYN record words in the header");
// The slot record's 4th word: a fingerprint of the streamed system (FNV-1a over the library's column codes, F, the
// statics count and the arm count), so a slot streamed for another system of the same shape (same F and arm
// count, other exponents or statics) is flagged at finalisation like an unstreamed one.  The derivative kind,
// method and block count may change between calls (the partials are the same system's G|b).
__host__ __device__ inline unsigned slot_fingerprint(const LibDesc& lib, int n_arms) {
  unsigned h = 2166136261u;
  auto mix = [&](unsigned v) {
    for (int k = 0; k < 4; ++k) {
      h ^= (v >> (8 * k)) & 0xffu;
      h *= 16777619u;
    }
  };
  mix((unsigned)lib.F);
  mix((unsigned)lib.U);
  mix((unsigned)n_arms);
  for (int j = 0; j < lib.F && j < INSITE_MAX_TERMS; ++j) mix((unsigned)lib.ucode[j]);
  return h;
}

// A finalisation whose slot record does not match: NaN G|b (and with STF > 0 NaN coefficients, mask 0,
// iters -3), so a misuse is loud rather than silently wrong.
template <int STF>
__device__ void finalize_invalid(const LibDesc& lib, const GramOut& o) {
  const int F = lib.F;
  const double nan = __builtin_nan("");
  for (int i = threadIdx.x; i < o.n_arms * F * F; i += kBlock) o.G[i] = nan;
  for (int i = threadIdx.x; i < o.n_arms * F; i += kBlock) {
    o.b[i] = nan;
    if constexpr (STF > 0) {
      o.coef[i] = nan;
      if (o.mask) o.mask[i] = 0;
    }
  }
  if constexpr (STF > 0)
    if (o.iters && (int)threadIdx.x < o.n_arms) o.iters[threadIdx.x] = -3;
}

// The STLSQ of an already-reduced system in global memory (the lagged step, N > 1: G|b all-reduced across the
// ranks between launches).  One thread per arm, the solve of tail_finish on the lower triangle of G (the full
// symmetric G the reduction wrote), so every rank's replicated fit is bitwise that of a single rank given equal
// G|b.
template <int STF>
__device__ void fit_from_gb(const double* __restrict__ G, const double* __restrict__ b, const GramOut& o) {
  const int a = (int)threadIdx.x;
  if (a >= o.n_arms) return;
  double g[STF][STF], rhs[STF], c[STF];
#pragma unroll
  for (int i = 0; i < STF; ++i) {
    rhs[i] = b[a * STF + i];
#pragma unroll
    for (int j = 0; j <= i; ++j) g[i][j] = G[(a * STF + i) * STF + j];
  }
  unsigned sup = 0u;
  const int it = stlsq_solve<STF>(g, rhs, o.sp.thr, o.sp.alpha, o.sp.max_iter, o.sp.unbias, c, sup);
#pragma unroll
  for (int i = 0; i < STF; ++i) {
    o.coef[a * STF + i] = c[i];
    if (o.mask) o.mask[a * STF + i] = (int8_t)((sup >> i) & 1u);
  }
  if (o.iters) o.iters[a] = it;
}

// XCD-aware rollout ranges (INSITE_DEF_XCD): the hardware places block b on XCD b % 8, and the rollout role cuts its
// (tile, arm group) units into consecutive ranges per wave.  The arm-bit words of 16 neighbouring tiles share a
// 128-B line of the time-major bit mask, so with consecutive ranges on consecutive (round-robin) XCDs every XCD's L2
// fetched most of those lines: PMC reads 189 MB per launch against 167 MB of data (profiles/traffic_r04.json).  The
// rollout blocks are ranked XCD-major instead -- the blocks of one XCD take one contiguous eighth of the tiles -- so a
// line is fetched by one XCD (at the seven boundaries by two).  Which wave rolls out a patient never reaches y.
#ifndef INSITE_DEF_XCD
#define INSITE_DEF_XCD 1
#endif
// INSITE_DEF_STEPS (A/B, off): the rollout role's ranges balanced in stored steps (rollout_steps) instead of (tile,
// group) units.  Measured slower on one box, interleaved 3 x 100 steps: 0.0738-0.0743 ms vs 0.0715-0.0721 ms with the
// unit ranges (profiles/r04/steps/): the per-step store predicate and the mid-group range ends cost more than the
// 272-328 stored steps per wave of the unit split.
#ifndef INSITE_DEF_STEPS
#define INSITE_DEF_STEPS 0
#endif
#if INSITE_DEF_STEPS && INSITE_DEF_RSTATIC < 1000
#error "the claimed rollout tail (INSITE_DEF_RSTATIC < 1000) cuts (tile, group) units: build with INSITE_DEF_STEPS=0"
#endif
constexpr int kXcds = 8;
// #{ i in [0, n) : i % kXcds == x } for n >= 0
__device__ __forceinline__ int64_t xcd_count(int64_t n, int x) { return (n + kXcds - 1 - x) / kXcds; }
// The claimed rollout tail (INSITE_DEF_RSTATIC < 1000) with one head per XCD slot (INSITE_DEF_XHEADS, VERDICT r04
// item 5): round 3's single device-scope head took every claim of the chip -- 2-4k claims per launch against the
// ~88 dequeues / us one word sustains (MI355X_MICROARCH.md "dequeue") -- and measured 35-65 % slower.  Here the tail
// [S, units) is cut into kXcds contiguous segments; the waves of the rollout blocks with b % kXcds == x (XCD x under
// the dispatcher's round robin -- speed only: the protocol is agent-scope atomics, correct under any placement) claim
// chunks of segment x from head x, each head on its own 128-B line of the workspace's claim area (after the two
// slots), with its own done counter: the last wave of slot x to finish claiming resets both, so every launch leaves
// the area zero.  With fewer than kXcds rollout blocks one head serves all.
#ifndef INSITE_DEF_XHEADS
#define INSITE_DEF_XHEADS 1
#endif
constexpr int kClaimLineWords = 32;                      // one 128-B line per head (head word 0, done word 1)
constexpr size_t kDefClaimBytes = (size_t)kXcds * kClaimLineWords * sizeof(unsigned);
// The deferred step's workspace: [claim areas, kDefAreaBytes][slot 0][slot 1].  The claim areas (the claimed rollout
// tail's or the claimed gram tail's heads) sits at offset 0 so that its place does not move with the cohort size
// (a grow-only workspace reused for another N left the heads on stale partial bytes).
// [0, 2 KiB): the claimed gram tail's heads; [2 KiB, 4 KiB): the claimed rollout tail's (both may run in one launch)
constexpr size_t kDefAreaBytes = 4096;
constexpr size_t kDefRollClaimOff = 2048;
static_assert(kDynClaimBytes <= kDefRollClaimOff && kDefRollClaimOff + kDefClaimBytes <= kDefAreaBytes,
              "claim areas fit the header area");
// rank of block b among the blocks [lo, hi) ordered XCD-major (by b % kXcds, then b)
__device__ __forceinline__ int64_t xcd_rank(int64_t b, int64_t lo, int64_t hi) {
  const int x = (int)(b % kXcds);
  int64_t r = xcd_count(b, x) - xcd_count(lo, x);
  for (int q = 0; q < x; ++q) r += xcd_count(hi, q) - xcd_count(lo, q);
  return r;
}

// lagged = 1 (insite_fit_rollout_lagged_f64, the N > 1 schedule): block gblocks REDUCES the previous slot to the
// rank-local G|b (out.G, out.b; no STLSQ -- the ranks all-reduce it between launches) and then solves the STLSQ of
// an all-reduced system (G_fit, b_fit -> fit; a bucket the reduction never writes), so the rollout keeps the
// deferred step's blocks (INSITE_LAG_MERGED; 0: the solve on a block of its own, round 4, the rollout one block
// shorter).
#ifndef INSITE_LAG_MERGED
#define INSITE_LAG_MERGED 1
#endif
#ifndef INSITE_DEF_ROVS
#define INSITE_DEF_ROVS 1
#endif
// Profiling ablation only (tools/build_variant.sh): 1 = the gram role alone, 2 = the rollout role alone, 3 = both
#ifndef INSITE_DEF_ROLES
#define INSITE_DEF_ROLES 3
#endif
template <bool SMOOTH, int METHOD, int DYN = 0>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(INSITE_STEP_WPE)))
step_deferred_kernel(const double* __restrict__ x, int64_t ldx, int n_steps, const double* __restrict__ u,
                     const int8_t* __restrict__ arm, const int32_t* __restrict__ rows, int64_t N, GramW w, LibDesc lib,
                     double* __restrict__ part_cur, const double* __restrict__ part_prev, GramOut out, RolloutArgs ra,
                     int gblocks, unsigned* __restrict__ rc, unsigned* __restrict__ hdr_cur,
                     const unsigned* __restrict__ hdr_prev, int lagged, const double* __restrict__ G_fit,
                     const double* __restrict__ b_fit, GramOut fit, unsigned fprint, DynGram dg) {
  __shared__ double smem[kGramSmem];
  const int n_ent = out.n_arms * lib.nE;
  if ((int)blockIdx.x < gblocks) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      hdr_cur[kSlotRec] = kSlotMagic;
      hdr_cur[kSlotRec + 1] = (unsigned)gblocks;
      hdr_cur[kSlotRec + 2] = (unsigned)n_ent;
      hdr_cur[kSlotRec + 3] = fprint;
      // the slot's format for the next finalisation: P claimed pieces after the block partials (0: static), and the
      // processed count the last claiming wave stores at the end -- a sentinel until then (agent-scope stores, ordered
      // at the memory side: the same word is written from another XCD at the end of the launch)
      __hip_atomic_store(hdr_cur + kDynRecP, DYN ? (unsigned)dg.P : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (DYN) __hip_atomic_store(hdr_cur + kDynRecDone, 0xFFFFFFFFu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (INSITE_DEF_GPRIO) __builtin_amdgcn_s_setprio(INSITE_DEF_GPRIO);
    if (!(INSITE_DEF_ROLES & 1)) return;
    gram_body<1, 2, SMOOTH, true, true, 0, 7, DYN>((int)blockIdx.x, gblocks, smem, x, ldx, n_steps, u, arm,
                                                              rows, N, 0, 0, w, lib, part_cur, nullptr, out, &dg);
    return;
  }
  if ((int)blockIdx.x == gblocks) {
    if (part_prev) {
      INSITE_TREAL(49152, 8);
      const unsigned mg = hdr_prev[kSlotRec], nb = hdr_prev[kSlotRec + 1], ne = hdr_prev[kSlotRec + 2];
      bool ok = mg == kSlotMagic && ne == (unsigned)n_ent && nb >= 1u && nb <= (unsigned)kGramMaxBlocks &&
                hdr_prev[kSlotRec + 3] == fprint;
      // a slot streamed with the claimed tail: every claimed piece processed (rows = its block partials + its piece
      // partials, summed by dyn_finalize); a static slot (P = 0): the block partials (deferred_finalize)
      const unsigned np = hdr_prev[kDynRecP];
      if (np > 0u) ok = ok && hdr_prev[kDynRecDone] == np;
      if (!ok) {
        if (lagged) finalize_invalid<0>(lib, out);
        else finalize_invalid<7>(lib, out);
      } else if (np > 0u) {
        if (lagged) dyn_finalize<0>(part_prev, (int)(nb + np), n_ent, lib, out, smem);
        else dyn_finalize<7>(part_prev, (int)(nb + np), n_ent, lib, out, smem);
      } else if (lagged) {
        deferred_finalize<0>(part_prev, (int)nb, n_ent, lib, out, smem);
      } else {
        deferred_finalize<7>(part_prev, (int)nb, n_ent, lib, out, smem);
      }
      INSITE_TREAL(49152, 9);
      INSITE_TSTAMP(49152, 0);
    }
    if (INSITE_LAG_MERGED && lagged && G_fit) fit_from_gb<7>(G_fit, b_fit, fit);  // (another bucket: no sync)
    return;
  }
  int first = gblocks + 1;
  if (!(INSITE_DEF_ROLES & 2)) return;
  if (lagged && !INSITE_LAG_MERGED) {
    if ((int)blockIdx.x == gblocks + 1) {
      if (G_fit) fit_from_gb<7>(G_fit, b_fit, fit);
      return;
    }
    first = gblocks + 2;
  }
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int64_t RW = (int64_t)(gridDim.x - first) * kWavesPerBlock;
  const int64_t rblk = INSITE_DEF_XCD ? xcd_rank((int64_t)blockIdx.x, first, (int64_t)gridDim.x)
                                      : (int64_t)((int)blockIdx.x - first);
  const int64_t rw = rblk * kWavesPerBlock + wid;
  INSITE_TREAL(32768 + rw, 8);
  INSITE_THWID(32768 + rw);
  const int ng = (ra.T + kRollGS - 1) / kRollGS;
  const int64_t units = (ra.N + kWave - 1) / kWave * ng;  // (tile, arm group) pairs, tile-major
#if INSITE_DEF_STEPS  // (the claimed tail, INSITE_DEF_RSTATIC < 1000, needs INSITE_DEF_STEPS=0)
  (void)units;
  (void)rc;
  const int64_t SS = (ra.N + kWave - 1) / kWave * ra.T;  // (tile, step) pairs
  rollout_steps<METHOD>(ra, lib, lane, rw * SS / RW, (rw + 1) * SS / RW);
#else
  const int64_t S = rc ? units * INSITE_DEF_RSTATIC / 1000 : units;
  rollout_units<METHOD>(ra, lib, lane, rw * S / RW, (rw + 1) * S / RW, ng);
  // (compiled only into the claimed-tail build: the dead claim paths in the default kernel took it from 232 to 248
  // VGPRs with a 104-B stack frame and the C2 launch 0.066 -> 0.069 ms, profiles/r05/c2reg/)
  if (INSITE_DEF_RSTATIC < 1000 && rc) {
    const int64_t nrb = (int64_t)gridDim.x - first;
    if (INSITE_DEF_XHEADS && nrb >= kXcds) {
      const int xs = (int)(blockIdx.x % kXcds);
      const int64_t wx = (xcd_count((int64_t)gridDim.x, xs) - xcd_count(first, xs)) * kWavesPerBlock;
      const int64_t lo = S + (units - S) * xs / kXcds, hi = S + (units - S) * (xs + 1) / kXcds;
      rollout_claimed<METHOD>(ra, lib, lane, lo, hi, ng, INSITE_DEF_RCHUNK, rc + xs * kClaimLineWords, wx);
    } else {
      rollout_claimed<METHOD>(ra, lib, lane, S, units, ng, INSITE_DEF_RCHUNK, rc, RW);
    }
  }
#endif
  INSITE_TSTAMP(32768 + rw, 0);
  INSITE_TREAL(32768 + rw, 9);
}

// =============================================================================================
// Adaptive RK45 rollout on irregular observation grids (configuration C5)
// =============================================================================================
// scipy.integrate.solve_ivp(method='RK45') restated per observation interval (oracle/rk45_ref.py; scipy
// 1.15.3 _ivp/rk.py RungeKutta._step_impl + common.select_initial_step), the treatment held over the
// interval as the reference's odeint scan does (sindy.py:413-424).  Lane = patient: every lane runs its
// own step-size controller, so lanes of a wavefront take different numbers of steps per interval (the
// divergence C5 stresses: the wave runs until its slowest lane finishes the interval, finished lanes
// masked).  The RHS is state-affine, f_a(y) = alpha_a + beta_a y (per-patient rates from the library).
struct Rk45Args {
  const double* y0;
  const double* u;
  const uint32_t* arm;  // TIME_MAJOR_BITS [T_max, lda] / PATIENT_MAJOR_BITS [N, lda]: arm of interval k
  const double* t;      // [T_max, ldt] (time-major) / [N, ldt] (patient-major) observation times
  const int32_t* nobs;  // [N] observations per patient (intervals = nobs - 1)
  const double* coef;
  double* y;            // [T_max, ldy] / [N, ldy]: element k = state at t[k + 1]
  int32_t* steps;       // [N] RK45 step attempts (may be NULL)
  const int32_t* order; // [N] lane -> row (rows binned by n_obs, insite_rk45_order_i32), NULL = identity
  int64_t lda, ldt, ldy, coef_stride, N;
  int32_t Tmax, A;
  double rtol, atol, drop;
  int32_t ybuf;         // PM staging: y's byte offsets fit a buffer descriptor (< 2^31): branch-free flushes
};

// e^(-1/5) for the RK45 step-size rules (scipy rk.py: `error_norm ** error_exponent`, exponent -1/5, once
// per attempt; common.py select_initial_step: `(0.01 / max(d1, d2)) ** (1 / (order + 1))`, once per
// interval).  A fp32 hardware estimate (v_log_f32 / v_exp_f32 on the rounded argument, relative error
// ~1e-6 for |log2 e| <= 120) is refined by two division-free Newton steps on x^5 e = 1,
// x <- x (1 - r / 5), r = x^5 e - 1 (error 3 delta^2 per step): fp64 accuracy of the exact fifth root
// (pow's exponent is the double 0.2 = 1/5 + 1.1e-17, i.e. a relative 1.1e-17 |ln e| away: < 1 ulp for
// controller errors in [1e-6, 1e4]) in ~16 VALU ops instead of ocml's double-double pow_f64 (>100), the
// per-attempt cost that dominated the step loop.  Arguments outside [2^-120, 2^120] (x^5 e would leave
// the fp64 range's comfort zone / the fp32 estimate would flush) take the exactly range-reduced form
// e = m 2^(5q), m in [1, 64), on a branch no realistic controller error reaches; zero, infinite and NaN
// inputs get pow's values (inf, 0, NaN) by select, so no pow body is inlined into the loop's registers.
#ifndef INSITE_RK45_ROOT_BRANCH
#define INSITE_RK45_ROOT_BRANCH 0
#endif
__device__ __forceinline__ double rk45_inv_root5(double e) {
#if INSITE_RK45_ROOT_BRANCH  // A/B: round 2's exact range reduction on a (never taken) branch
  double m = e;
  int q = 0;
  if (!(e >= 0x1p-120 && e <= 0x1p120)) {
    if (!(e > 0.0 && e < INFINITY)) return e == 0.0 ? INFINITY : e == INFINITY ? 0.0 : __builtin_nan("");
    const int k = ilogb(e);
    q = (k >= 0 ? k : k - 4) / 5;  // floor(k / 5)
    m = ldexp(e, -5 * q);
  }
#else
  // Branch-free: the argument is clamped to [2^-120, 2^120].  Every use of the root is bounded by its callers
  // where the clamp bites: the step factor min(10, 0.9 x) is 10 for any e < 2^-120 (x > 2^24) and
  // max(0.2, 0.9 x) is 0.2 for any e > 2^120, and select_initial_step's min(100 h0, x, span) keeps 100 h0
  // (d1 > 1e34 makes h0 <= 1e-36 |y| / scale); NaN stays NaN (pow's value).  The branch cost ~10 scalar
  // and branch instructions per attempt for every wave (round 2's SQ_INSTS_SALU / _BRANCH, profiles/r02/c5_pmc/).
  const double m = fmin(fmax(e, 0x1p-120), 0x1p120);
  constexpr int q = 0;
#endif
  double x = (double)__builtin_amdgcn_exp2f(-0.2f * __builtin_amdgcn_logf((float)m));
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const double x2 = x * x;
    const double r = fma(x2 * x2 * x, m, -1.0);
    x = fma(-0.2 * x, r, x);
  }
#if INSITE_RK45_ROOT_BRANCH
  return q == 0 ? x : ldexp(x, -q);
#else
  (void)q;
  return e == e ? x : e;
#endif
}

// 1 / b for the controller's norms (b a positive normal double: atol + |y| rtol, |f| > 0): the hardware
// v_rcp_f64 estimate and two Newton steps, ~1 ulp, 5 VALU ops against the 11 of an IEEE division -- the
// quotients feed comparisons with 1 and 1e-5 and the fifth root, where an ulp only matters at exact ties.
__device__ __forceinline__ double rk45_rcp(double b) {
  double r = __builtin_amdgcn_rcp(b);
  r = fma(fma(-b, r, 1.0), r, r);
  return fma(fma(-b, r, 1.0), r, r);
}

#ifndef INSITE_RK45_WPE
#define INSITE_RK45_WPE 1  // waves per SIMD the register budget is sized for (1: unconstrained)
#endif
template <int NARM, bool PERROW>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(INSITE_RK45_WPE)))
rollout_rk45_kernel(Rk45Args ra, LibDesc lib) {
  constexpr double a21 = 1.0 / 5.0;
  constexpr double a31 = 3.0 / 40.0, a32 = 9.0 / 40.0;
  constexpr double a41 = 44.0 / 45.0, a42 = -56.0 / 15.0, a43 = 32.0 / 9.0;
  constexpr double a51 = 19372.0 / 6561.0, a52 = -25360.0 / 2187.0, a53 = 64448.0 / 6561.0, a54 = -212.0 / 729.0;
  constexpr double a61 = 9017.0 / 3168.0, a62 = -355.0 / 33.0, a63 = 46732.0 / 5247.0, a64 = 49.0 / 176.0,
                   a65 = -5103.0 / 18656.0;
  constexpr double b1 = 35.0 / 384.0, b3 = 500.0 / 1113.0, b4 = 125.0 / 192.0, b5 = -2187.0 / 6784.0, b6 = 11.0 / 84.0;
  constexpr double e1 = -71.0 / 57600.0, e3 = 71.0 / 16695.0, e4 = -71.0 / 1920.0, e5 = 17253.0 / 339200.0,
                   e6 = -22.0 / 525.0, e7 = 1.0 / 40.0;
  const int lane = threadIdx.x & (kWave - 1);
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int64_t p0 = ((int64_t)blockIdx.x * kWavesPerBlock + wid) * kWave;
  if (p0 >= ra.N) return;
  const int64_t p = p0 + lane;
  const bool act = p < ra.N;
  const int64_t pc = act ? p : ra.N - 1;
  double uu[INSITE_MAX_STATICS];
#pragma unroll
  for (int t = 0; t < INSITE_MAX_STATICS; ++t) {
    const double v = ra.u[pc * lib.U + (t < lib.U ? t : 0)];
    uu[t] = (act && t < lib.U) ? v : 0.0;
  }
  double alpha[NARM], beta[NARM];
  const double* cbase = ra.coef + (PERROW ? pc * ra.coef_stride : 0);
#pragma unroll
  for (int a = 0; a < NARM; ++a) {
    alpha[a] = 0.0;
    beta[a] = 0.0;
    if (a >= ra.A) continue;
    for (int j = 0; j < lib.F; ++j) {
      const double c = cbase[a * lib.F + j];
      if (fabs(c) > ra.drop) {
        const double t = c * monomial(lib, j, uu);
        if (col_ex(lib, j) == 0) alpha[a] += t;
        else beta[a] += t;
      }
    }
  }
  int n = act ? ra.nobs[pc] : 0;
  if (n > ra.Tmax) n = ra.Tmax;
  const int nmax = wave_max_i(n);
  double y = act ? ra.y0[pc] : 0.0;
  int attempts = 0;
  unsigned w = 0u;
  const double rtol = ra.rtol, atol = ra.atol;
  for (int k = 0; k + 1 < nmax; ++k) {
    if ((k & 31) == 0) {  // arm bits of intervals [k, k + 32): one word per lane, half-wave transpose
      const int kk = k + (lane & 31) < ra.Tmax ? k + (lane & 31) : ra.Tmax - 1;
      const int64_t col = (p0 >> 5) + (lane >> 5);
      const uint32_t v = col * 32 < ra.N ? ra.arm[(int64_t)kk * ra.lda + col] : 0u;
      w = bit_transpose32(v, lane);
    }
    const bool on = k + 1 < n;
    const int a = (int)((w >> (k & 31)) & 1u);
    double al = alpha[0], be = beta[0];
#pragma unroll
    for (int aa = 1; aa < NARM; ++aa) {
      al = (a == aa) ? alpha[aa] : al;
      be = (a == aa) ? beta[aa] : be;
    }
    double t = on ? ra.t[(int64_t)k * ra.ldt + pc] : 0.0;
    const double t1 = on ? ra.t[(int64_t)(k + 1) * ra.ldt + pc] : 0.0;
    if (on && t < t1) {
      // ---- select_initial_step (order 4, n = 1) ----
      double f = fma(be, y, al);
      const double interval = t1 - t;
      double h_abs;
      {
        const double scale = atol + fabs(y) * rtol;
        const double d0 = fabs(y / scale), d1 = fabs(f / scale);
        double h0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : 0.01 * d0 / d1;
        h0 = fmin(h0, interval);
        const double f1 = fma(be, y + h0 * f, al);
        const double d2 = fabs((f1 - f) / scale) / h0;
        const double h1 = (d1 <= 1e-15 && d2 <= 1e-15) ? fmax(1e-6, h0 * 1e-3) : rk45_inv_root5(fmax(d1, d2) * 100.0);
        h_abs = fmin(fmin(100.0 * h0, h1), interval);
      }
      // ---- accepted steps until t reaches t1 ----
      while (t < t1) {
        const double min_step = 10.0 * fabs(nextafter(t, INFINITY) - t);
        if (h_abs < min_step) h_abs = min_step;
        bool rejected = false;
        for (;;) {
          double t_new = t + h_abs;
          if (t_new > t1) t_new = t1;
          const double h = t_new - t;
          h_abs = fabs(h);
          const double k1 = f;
          const double k2 = fma(be, y + (k1 * a21) * h, al);
          const double k3 = fma(be, y + (k1 * a31 + k2 * a32) * h, al);
          const double k4 = fma(be, y + ((k1 * a41 + k2 * a42) + k3 * a43) * h, al);
          const double k5 = fma(be, y + (((k1 * a51 + k2 * a52) + k3 * a53) + k4 * a54) * h, al);
          const double k6 = fma(be, y + ((((k1 * a61 + k2 * a62) + k3 * a63) + k4 * a64) + k5 * a65) * h, al);
          const double y_new = y + h * ((((k1 * b1 + k3 * b3) + k4 * b4) + k5 * b5) + k6 * b6);
          const double f_new = fma(be, y_new, al);
          const double scale = atol + fmax(fabs(y), fabs(y_new)) * rtol;
          const double e = ((((k1 * e1 + k3 * e3) + k4 * e4) + k5 * e5) + k6 * e6) + f_new * e7;
          const double err = fabs(e * h / scale);
          ++attempts;
          if (err < 1.0) {
            double factor = err == 0.0 ? 10.0 : fmin(10.0, 0.9 * rk45_inv_root5(err));
            if (rejected) factor = fmin(1.0, factor);
            h_abs *= factor;
            t = t_new;
            y = y_new;
            f = f_new;
            break;
          }
          h_abs *= fmax(0.2, 0.9 * rk45_inv_root5(err));
          rejected = true;
        }
      }
    }
    if (on) __builtin_nontemporal_store(y, ra.y + (int64_t)k * ra.ldy + p);
  }
  if (act && ra.steps) ra.steps[p] = attempts;
}

// Flat-loop form of the same controller (the default).  Each lane runs its own state machine over
// (interval k, accepted step, attempt); one loop iteration = one step attempt of every lane, whatever
// interval each lane is in.  The per-interval form above synchronises the wave at every interval
// boundary AND at every accepted step (nested divergent loops: each accepted step waits for the lane
// with the most rejections, each interval for the lane with the most steps), so a wave paid
// sum_k sum_steps max_lanes(...); here it pays max_lanes(total attempts).
// Closed-form attempt: the RHS is affine in y on an interval, f(y) = al + be y, so the Dormand-Prince
// stages are k_i = F q_i(z) with F = f(y), z = h be, and the tableau collapses (exact rational algebra,
// DESIGN.md §5) to
//   y_new = y + h F Q(z),  Q = 1 + z/2 + z^2/6 + z^3/24 + z^4/120 + z^5/600,
//   f_new = F (1 + z Q(z)),   error = h F z^4 (97/120000 - 13 z/40000 + z^2/24000):
// ~20 fp64 ops per attempt instead of ~60, and the error estimate loses the stage form's cancellation
// (sum e_i = 0 over O(F) stages leaves an O(F z^4) result with ~eps/z^4 relative rounding; here it is
// exact to rounding).  Step-size rules, acceptance and select_initial_step are scipy's (rk.py /
// common.py), as in the per-interval kernel; attempt counts agree with the stage-form oracle except where
// an err sits within its rounding of 1.
// One fifth root per iteration: every branch any lane takes is issued for the whole wave, and the two
// e^(-1/5) of the controller never meet in one lane-iteration -- the step factor of an accepted step that
// ENDS its interval is discarded (solve_ivp restarts per interval, so the next interval's h comes from
// select_initial_step), so that lane roots the initial-step argument instead.  The accept / reject / open
// updates of h_abs are selects; only the interval close (a store and an LDS read) branches.
// Observation times come from a per-lane LDS window t[base .. base + kRkWin) ([slot][lane] layout: a wave's
// ds_read_b64 is conflict-free), refilled for every live lane of the wave at once when some lane's next close
// would run past its window: a vector-memory wait is paid once per refill (every ~kRkWin intervals of the
// fastest lane), not once per iteration.  (vmcnt is per wave: with a load issued at every close, and some
// lane closing in nearly every iteration, a register queue waits on the previous iteration's load.)
#ifndef INSITE_RK45_WIN
#define INSITE_RK45_WIN 8  // 8: 32 KB of LDS per block with the output staging -> 5 blocks per CU (16: 3; 0.94 -> 0.88 ms, profiles/r03/v23)
#endif
// PM: patient-major t / y / arm bits (INSITE_LAYOUT_PATIENT_MAJOR_BITS): a lane's window refill reads one
// contiguous run and its y elements share lines that only this lane writes, whatever rows the lanes hold
// -- the layout that lets rows be binned by n_obs without scattering the memory traffic.
#ifndef INSITE_RK45_PM_NT
#define INSITE_RK45_PM_NT 0
#endif
// PM output staging: a lane's y elements go to an 8-slot LDS ring indexed by their address within a 64-B
// sector and are stored as one 64-B run (4 x 16 B) when the sector's last element arrives (partial sectors at
// a row's ends element by element).  With one 8-B store per close the lane's sectors were written back
// piecewise: L2 evicted a partly written line between two closes of the same lane (1M lanes x 480 B rows),
// PMC WRITE_SIZE 1.35 GB per launch against 312 MB of y (profiles/r02/c5_pmc/).
#ifndef INSITE_RK45_STAGE
#define INSITE_RK45_STAGE 1
#endif
#ifndef INSITE_RK45_BUFREFILL
#define INSITE_RK45_BUFREFILL 1
#endif
#ifndef INSITE_RK45_FULLSEC
#define INSITE_RK45_FULLSEC 1  // whole-sector flushes as 16-B stores (0: every flush element by element)
#endif
#ifndef INSITE_RK45_MINSTEP_BRANCH
#define INSITE_RK45_MINSTEP_BRANCH 0
#endif
#ifndef INSITE_RK45_HSEL
#define INSITE_RK45_HSEL 1
#endif
#ifndef INSITE_RK45_CLOSE_BRANCH
#define INSITE_RK45_CLOSE_BRANCH 1  // the close block under `if (close)` (0: branch-free selects, A/B)
#endif
constexpr int kRkWin = INSITE_RK45_WIN;
constexpr int kRkStage = INSITE_RK45_STAGE ? 8 : 1;
template <int NARM, bool PERROW, bool PM>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(INSITE_RK45_WPE)))
rollout_rk45_flat_kernel(Rk45Args ra, LibDesc lib) {
  constexpr double q2 = 1.0 / 2.0, q3 = 1.0 / 6.0, q4 = 1.0 / 24.0, q5 = 1.0 / 120.0, q6 = 1.0 / 600.0;
  constexpr double p0 = 97.0 / 120000.0, p1 = -13.0 / 40000.0, p2 = 1.0 / 24000.0;
  __shared__ double t_win[kWavesPerBlock * kRkWin * kWave];
  __shared__ double y_ring[kWavesPerBlock * kRkStage * kWave];  // PM staging ring [slot][lane]
  const int64_t lane_id = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  const bool act = lane_id < ra.N;
  // this lane's row (an order entry out of range -- never from insite_rk45_order_i32 -- is clamped, not followed)
  int64_t p = act ? (ra.order ? (int64_t)min((unsigned)ra.order[lane_id], (unsigned)(ra.N - 1)) : lane_id) : ra.N - 1;
  p = p < 0 ? 0 : p >= ra.N ? ra.N - 1 : p;  // memory-safe on a malformed order (documented: a permutation)
  const int64_t pc = p;
  double* tw = t_win + (threadIdx.x / kWave) * (kRkWin * kWave) + (threadIdx.x & (kWave - 1));
  double* yr = y_ring + (threadIdx.x / kWave) * (kRkStage * kWave) + (threadIdx.x & (kWave - 1));
  constexpr bool kStage = PM && INSITE_RK45_STAGE && !INSITE_RK45_PM_NT;
  int slot_lo = -1;  // kStage: first slot of the current sector holding a staged element (-1: none)
  double uu[INSITE_MAX_STATICS];
#pragma unroll
  for (int t = 0; t < INSITE_MAX_STATICS; ++t) {
    const double v = ra.u[pc * lib.U + (t < lib.U ? t : 0)];
    uu[t] = (act && t < lib.U) ? v : 0.0;
  }
  double alpha[NARM], beta[NARM];
  affine_rates<NARM>(lib, ra.coef + (PERROW ? pc * ra.coef_stride : 0), ra.A, ra.drop, uu, alpha, beta);
  int n = act ? ra.nobs[pc] : 0;
  if (n > ra.Tmax) n = ra.Tmax;
  const double rtol = ra.rtol, atol = ra.atol;
  const int64_t wrd = PM ? pc * ra.lda : pc >> 5;  // PM: the row's first word; else the word column
  const unsigned bit = PM ? 0u : (unsigned)(pc & 31);
  // arms of up to 64 intervals gathered once into a per-lane mask (PM: the row's two words; time-major:
  // 16 independent loads in flight per round, clamped rows, masked bits); longer grids read each
  // interval's bit when the interval opens
  const bool amask_ok = ra.Tmax <= 64;
  unsigned long long amask = 0ull;
  if (PM && NARM > 1 && amask_ok) {
    const uint32_t w0 = ra.arm[wrd], w1 = ra.Tmax > 33 ? ra.arm[wrd + 1] : 0u;
    amask = (unsigned long long)w0 | ((unsigned long long)w1 << 32);
  }
  if (!PM && NARM > 1 && amask_ok) {
    for (int k0 = 0; k0 + 1 < ra.Tmax; k0 += 16) {
      uint32_t w[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int kk = k0 + j < ra.Tmax - 1 ? k0 + j : ra.Tmax - 2;
        w[j] = ra.arm[(int64_t)(kk < 0 ? 0 : kk) * ra.lda + wrd];
      }
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (k0 + j + 1 < ra.Tmax) amask |= (unsigned long long)((w[j] >> bit) & 1u) << (k0 + j);
    }
  }
  double y = act ? ra.y0[pc] : 0.0;
  int attempts = 0;
  // lane state: interval k with end t1 and rates al/be; time t, f = f(y), h_abs; rejected = the current
  // step has had a rejected attempt; the window holds t[base .. base + kRkWin); yp = row k of y
  int k = 0, base = 0;
  double t = 0.0, t1 = 0.0, al = alpha[0], be = beta[0], f = 0.0, h_abs = 0.0;
  bool rejected = false;
  double* yp = ra.y + (PM ? p * ra.ldy : p);
  const int64_t ystep = PM ? 1 : ra.ldy;
  const int64_t tstep = PM ? 1 : ra.ldt;
  const double* trow = ra.t + (PM ? pc * ra.ldt : pc);
  // INSITE_RK45_BUFREFILL (PM): the window through a buffer descriptor over t -- one 32-bit offset per lane and
  // immediate offsets for the 8 elements, unclamped (elements past the row's last observation are never used; past
  // the array the hardware returns 0) -- instead of 8 clamped 64-bit addresses (~30 VALU per refill event).  The
  // records end at the last row's T_max-th element, not at N * ldt: a t_obs view whose last row is narrower than
  // ldt (as_strided) is never read past its storage
  const int64_t t_rec = ((int64_t)(ra.N - 1) * ra.ldt + ra.Tmax) * 8;
  const bool tbuf = PM && INSITE_RK45_BUFREFILL && t_rec <= (int64_t)INT32_MAX;
  const __amdgpu_buffer_rsrc_t trs =
      __builtin_amdgcn_make_buffer_rsrc((void*)ra.t, (short)0, (int)(tbuf ? t_rec : 0), 0x00020000);
  auto refill = [&](int from) {  // elements clamped to n - 1 (n >= 2 for a live lane)
    base = from;
    if (tbuf) {
      const unsigned off = (unsigned)((pc * ra.ldt + from) * 8);
#pragma unroll
      for (int j = 0; j < kRkWin; ++j)
        tw[j * kWave] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(trs, off + 8u * j, 0, 0));
      return;
    }
#pragma unroll
    for (int j0 = 0; j0 < kRkWin; j0 += 8) {
      double v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int r = from + j0 + j < n ? from + j0 + j : n - 1;
        v[j] = trow[(int64_t)r * tstep];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) tw[(j0 + j) * kWave] = v[j];
    }
  };
  auto rates = [&]() {
    if (NARM > 1) {
      const int a = amask_ok ? (int)((amask >> k) & 1ull)
                    : PM ? (int)((ra.arm[wrd + (k >> 5)] >> (k & 31)) & 1u)
                         : (int)((ra.arm[(int64_t)k * ra.lda + wrd] >> bit) & 1u);
      al = alpha[0];
      be = beta[0];
#pragma unroll
      for (int aa = 1; aa < NARM; ++aa) {
        al = (a == aa) ? alpha[aa] : al;
        be = (a == aa) ? beta[aa] : be;
      }
    }
  };
  // select_initial_step (order 4, n = 1; common.py), split around the shared fifth root.  Affine RHS:
  // f(y + h0 f) - f = be h0 f, so d2 = |f(y + h0 f) - f| / scale / h0 = |be| d1 exactly.
  double h0 = 0.0, span = 0.0;
  bool small = false;
  auto init_front = [&]() -> double {  // returns the root argument max(d1, d2) * 100 = (0.01 / max)^-1
    f = fma(be, y, al);
    span = t1 - t;
    const double scale = atol + fabs(y) * rtol;
    const double d1 = fabs(f) * rk45_rcp(scale);
    const bool tiny = fabs(y) < 1e-5 * scale || d1 < 1e-5;  // d0 < 1e-5 or d1 < 1e-5
    h0 = fmin(tiny ? 1e-6 : 0.01 * fabs(y) * rk45_rcp(fabs(f)), span);  // 0.01 d0 / d1 (|f| > 0 when used)
    const double d2 = fabs(be) * d1;
    small = d1 <= 1e-15 && d2 <= 1e-15;
    return small ? 1.0 : fmax(d1, d2) * 100.0;
  };
  auto init_h = [&](double r) { return fmin(fmin(100.0 * h0, small ? fmax(1e-6, h0 * 1e-3) : r), span); };
  // start of a step (rk.py _step_impl): min_step = 10 |nextafter(t, inf) - t|, the neighbour taken on the
  // bit pattern of |t| (+1 above a non-negative t, -1 below |t| for a negative one)
  auto min_step = [&]() {
    // |neighbour - |t||: the same two values as the two-sided form, as one select on the bit step (the
    // two-sided expression compiled to an exec-mask branch per accepted attempt)
    const double at = fabs(t);
    const long long tb = __double_as_longlong(at);
#if INSITE_RK45_MINSTEP_BRANCH  // A/B: the two-sided form
    return 10.0 * (t >= 0.0 ? __longlong_as_double(tb + 1ll) - at : at - __longlong_as_double(tb - 1ll));
#else
    return 10.0 * fabs(__longlong_as_double(tb + (t >= 0.0 ? 1ll : -1ll)) - at);
#endif
  };
  bool live = false;
  if (act && 1 < n) {
    t = trow[0];
    refill(1);
    t1 = tw[0];
    rates();
    live = true;
    h_abs = fmax(init_h(rk45_inv_root5(init_front())), min_step());
  }
  while (__builtin_amdgcn_ballot_w64(live) != 0ull) {
    // a close in this iteration reads t[k + 2]: refill every live lane when some lane's window ends before
    if (__builtin_amdgcn_ballot_w64(live && k + 2 >= base + kRkWin) != 0ull)
      if (live) refill(k + 2);
    if (live) {
      // ---- one attempt (closed form of the Dormand-Prince stages for the affine RHS) ----
      const bool open = t < t1;  // false: zero-length / reversed interval, closed with h = 0, no attempt
      double t_new = t + h_abs;
      if (t_new > t1) t_new = t1;
      if (!open) t_new = t;
      const double h = t_new - t;
      h_abs = fabs(h);
      const double z = h * be;
      const double Q = fma(fma(fma(fma(fma(q6, z, q5), z, q4), z, q3), z, q2), z, 1.0);
      const double hF = h * f;
      const double y_new = fma(hF, Q, y);
      const double f_new = fma(f * z, Q, f);
      const double z2 = z * z;
      const double scale = atol + fmax(fabs(y), fabs(y_new)) * rtol;
      const double err = fabs(hF * (z2 * z2) * fma(fma(p2, z, p1), z, p0)) * rk45_rcp(scale);
      attempts += open;
      const bool acc = err < 1.0;
      const bool close = acc && !(t_new < t1);  // the interval is done: its step factor is discarded
      double rarg = err == 0.0 ? 1.0 : err;
      if (acc) {
        t = t_new;
        y = y_new;
        f = f_new;
      }
#if INSITE_RK45_CLOSE_BRANCH
      if (close) {  // store y at t_{k+1} (row k), open interval k + 1 from the window
#else
      // The interval close, branch-free except for the store: nearly every iteration some lane of the wave
      // closes an interval, so the close work is issued for the whole wave anyway; computing the next
      // interval's values for every lane and selecting them drops the exec-mask and branch instructions
      // around it.  Only the output store (and its LDS staging) stays under `close`.
      {
        const int kn = k + (close ? 1 : 0);
        const double t1n = tw[(kn + 1 - base) * kWave];  // k + 1 - base when not closing: the current t1 slot
        double aln = al, ben = be;
        if (NARM > 1) {
          if (amask_ok) {  // uniform
            const int an = (int)((amask >> kn) & 1ull);
            aln = alpha[0];
            ben = beta[0];
#pragma unroll
            for (int aa = 1; aa < NARM; ++aa) {
              aln = (an == aa) ? alpha[aa] : aln;
              ben = (an == aa) ? beta[aa] : ben;
            }
          } else if (close) {
            const int kk = k;
            k = kn;
            rates();
            aln = al;
            ben = be;
            k = kk;
          }
        }
        // select_initial_step of interval kn from (t1, y): the front half, every lane
        const double fi = fma(ben, y, aln);
        const double spani = t1n - t1;
        const double scale_i = atol + fabs(y) * rtol;
        const double d1 = fabs(fi) * rk45_rcp(scale_i);
        const bool tiny = fabs(y) < 1e-5 * scale_i || d1 < 1e-5;
        const double h0i = fmin(tiny ? 1e-6 : 0.01 * fabs(y) * rk45_rcp(fabs(fi)), spani);
        const double d2 = fabs(ben) * d1;
        const bool smalli = d1 <= 1e-15 && d2 <= 1e-15;
        const double argi = smalli ? 1.0 : fmax(d1, d2) * 100.0;
        if (close) {
#endif
        if constexpr (kStage) {
          // element slot within its 64-B sector; the sector goes out when its last slot arrives or the row ends
          const int slot = (int)(((uintptr_t)yp >> 3) & 7u);
          yr[slot * kWave] = y;
          if (slot_lo < 0) slot_lo = slot;
          if (slot == 7 || !(k + 2 < n)) {
            double* sec = yp - slot;
            if (ra.ybuf) {  // uniform: the sector's staged elements [slot_lo, slot] as 8-B buffer stores, the
                            // others to an offset the hardware drops (no per-element exec-mask branches)
              const __amdgpu_buffer_rsrc_t yrs = __builtin_amdgcn_make_buffer_rsrc(
                  (void*)ra.y, (short)0, (int)(ra.N * ra.ldy * 8), 0x00020000);
              const unsigned sb = (unsigned)((sec - ra.y) * 8);
              double v[8];
#pragma unroll
              for (int j = 0; j < 8; ++j) v[j] = yr[j * kWave];
#if INSITE_RK45_FULLSEC
              // a whole sector (every flush but a row's first / last partial one): four 16-B stores at immediate
              // offsets -- the per-element form below costs ~35 VALU of offset selects, and with 64 lanes some lane
              // flushes in ~94 % of the iterations, so the wave paid them nearly every attempt
              if (slot_lo == 0 && slot == 7) {
                typedef double d2 __attribute__((ext_vector_type(2)));
#pragma unroll
                for (int j = 0; j < 8; j += 2)
                  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, d2{v[j], v[j + 1]}), yrs,
                                                         sb + 8u * j, 0, 0);
              } else {
#pragma unroll
                for (int j = 0; j < 8; ++j)
                  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v[j]), yrs,
                                                        (j >= slot_lo && j <= slot) ? sb + 8u * j : kOOB, 0, 0);
              }
#else
#pragma unroll
              for (int j = 0; j < 8; ++j)
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v[j]), yrs,
                                                      (j >= slot_lo && j <= slot) ? sb + 8u * j : kOOB, 0, 0);
#endif
            } else if (slot_lo == 0 && slot == 7) {
              double v[8];
#pragma unroll
              for (int j = 0; j < 8; ++j) v[j] = yr[j * kWave];
#pragma unroll
              for (int j = 0; j < 8; j += 2) {
                typedef double d2 __attribute__((ext_vector_type(2)));
                *reinterpret_cast<d2*>(sec + j) = d2{v[j], v[j + 1]};
              }
            } else {
              for (int j = slot_lo; j <= slot; ++j) sec[j] = yr[j * kWave];
            }
            slot_lo = -1;
          }
        } else if (PM && !INSITE_RK45_PM_NT) {
          *yp = y;  // PM: cached store, the lane's own line fills in L2
        } else {
          __builtin_nontemporal_store(y, yp);
        }
#if INSITE_RK45_CLOSE_BRANCH
        yp += ystep;
        t = t1;
        ++k;
        t1 = tw[(k + 1 - base) * kWave];
        rates();
        live = k + 1 < n;
        rarg = init_front();
      }
#else
        }
        yp = close ? yp + ystep : yp;
        t = close ? t1 : t;
        k = kn;
        t1 = close ? t1n : t1;
        al = close ? aln : al;
        be = close ? ben : be;
        f = close ? fi : f;
        span = close ? spani : span;
        h0 = close ? h0i : h0;
        small = close ? smalli : small;
        rarg = close ? argi : rarg;
        live = k + 1 < n;
      }
#endif
      const double r5 = rk45_inv_root5(rarg);
#if INSITE_RK45_HSEL
      // every candidate computed, then selected: the conditional form compiled to three exec-mask branches
      double factor = fmin(10.0, 0.9 * r5);
      factor = err == 0.0 ? 10.0 : factor;
      const double factor_r = fmin(1.0, factor);
      factor = rejected ? factor_r : factor;
      const double h_init = init_h(r5);
      const double h_acc = h_abs * factor;
      const double h_rej = h_abs * fmax(0.2, 0.9 * r5);
      const double ms = min_step();
      double h_next = acc ? h_acc : h_rej;
      h_next = close ? h_init : h_next;
      const double h_new = fmax(h_next, ms);
      h_abs = acc ? h_new : h_next;
#else
      double factor = err == 0.0 ? 10.0 : fmin(10.0, 0.9 * r5);
      if (rejected) factor = fmin(1.0, factor);
      const double h_next = close ? init_h(r5) : acc ? h_abs * factor : h_abs * fmax(0.2, 0.9 * r5);
      // a new step starts after an accept or a close (gating the bit-exact min_step on a wave ballot of the
      // steps it could raise measured slower: 0.93 -> 0.98 ms, profiles/r02/c5_minstep/)
      h_abs = acc ? fmax(h_next, min_step()) : h_next;
#endif
      rejected = !acc;
    }
  }
  if (act && ra.steps) ra.steps[p] = attempts;
}

// Row binning for the RK45 rollout: a wave runs until its slowest lane has finished, and a patient's
// attempt count grows with its number of observation intervals, so lanes are given rows grouped by n_obs
// (descending: the longest waves are dispatched first and short ones fill the tail).  Counting sort in two
// passes over n_obs; the order inside a bin is whatever the atomics give -- every row's trajectory is
// independent of the lane it runs on, so outputs do not depend on it.  A block's rows of one bin land together
// (one cursor atomic per bin and block): with 4096-row chunks a wave's rows mostly come from one 4096-row range,
// which the rollout's row-major reads like -- 1024- and 2048-row chunks measured 0.785 / 0.748 ms against 0.733
// (kernel), 8192 the same, 16384 slower (profiles/r05/c5_order/).  Measured and dropped (round 5): the histogram's
// scan in the count pass's last block (a ticket after device-scope fences: the count pass 9 -> 21 us) and both
// passes as one launch with a grid barrier on per-block epoch flags (63 us against ~26 for memset + two passes).
#ifndef INSITE_RK45_ORDER_SELFRESET  // 1: a self-resetting workspace instead of the memset (measured slower, round 6:
#define INSITE_RK45_ORDER_SELFRESET 0  // C5 0.672 vs 0.663 ms, INSITE 1.236 vs 1.225 -- the per-block fence + ticket)
#endif
constexpr int kRkBinMax = 1024;   // bins: key = min(n_obs, min(T_max, kRkBinMax - 1))
#ifndef INSITE_RK45_BIN_CHUNK
#define INSITE_RK45_BIN_CHUNK 4096  // rows per block of the two passes
#endif
constexpr int kRkBinChunk = INSITE_RK45_BIN_CHUNK;
static_assert(kRkBinChunk % kBlock == 0, "rows per binning block: a multiple of the block");
__device__ __forceinline__ int rk45_bin(int32_t n, int nb) { return nb - 1 - (n < 0 ? 0 : n > nb - 1 ? nb - 1 : n); }

__global__ void __launch_bounds__(kBlock) rk45_bin_count_kernel(const int32_t* __restrict__ nobs, int64_t N, int nb,
                                                                 unsigned* __restrict__ hist) {
  __shared__ unsigned h[kRkBinMax];
  constexpr int kPer = kRkBinChunk / kBlock;
  for (int b = threadIdx.x; b < nb; b += kBlock) h[b] = 0u;
  __syncthreads();
  const int64_t lo = (int64_t)blockIdx.x * kRkBinChunk;
  int bin[kPer];
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const int64_t i = lo + q * kBlock + threadIdx.x;
    bin[q] = i < N ? rk45_bin(nobs[i], nb) : -1;
  }
#pragma unroll
  for (int q = 0; q < kPer; ++q)
    if (bin[q] >= 0) atomicAdd(&h[bin[q]], 1u);
  __syncthreads();
  for (int b = threadIdx.x; b < nb; b += kBlock)
    if (h[b]) atomicAdd(&hist[b], h[b]);
}

// every block scans the (small) global histogram itself: the bins' totals loaded by all threads at once, then one
// wave's shuffle scan (lane l owns bins [l per, (l + 1) per)) -- round 4 had thread 0 walk it serially
__global__ void __launch_bounds__(kBlock) rk45_bin_scatter_kernel(const int32_t* __restrict__ nobs, int64_t N, int nb,
                                                                   unsigned* __restrict__ hist,
                                                                   unsigned* __restrict__ cursor,
                                                                   int32_t* __restrict__ order) {
  __shared__ unsigned base[kRkBinMax], cnt[kRkBinMax], tot[kRkBinMax];
  constexpr int kPer = kRkBinChunk / kBlock;
  const int64_t lo = (int64_t)blockIdx.x * kRkBinChunk;
  int bin[kPer];
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const int64_t i = lo + q * kBlock + threadIdx.x;
    bin[q] = i < N ? rk45_bin(nobs[i], nb) : -1;
  }
  for (int b = threadIdx.x; b < nb; b += kBlock) {
    cnt[b] = 0u;
    tot[b] = hist[b];
  }
  __syncthreads();
  if (threadIdx.x < kWave) {
    const int lane = threadIdx.x, per = (nb + kWave - 1) / kWave, b0 = lane * per;
    unsigned sum = 0u;
    for (int j = 0; j < per; ++j)
      if (b0 + j < nb) sum += tot[b0 + j];
    unsigned inc = sum;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
      const unsigned u = __shfl_up(inc, off);
      if (lane >= off) inc += u;
    }
    unsigned acc = inc - sum;
    for (int j = 0; j < per; ++j)
      if (b0 + j < nb) {
        base[b0 + j] = acc;
        acc += tot[b0 + j];
      }
  }
  unsigned rank[kPer];
#pragma unroll
  for (int q = 0; q < kPer; ++q) rank[q] = bin[q] >= 0 ? atomicAdd(&cnt[bin[q]], 1u) : 0u;
  __syncthreads();
  for (int b = threadIdx.x; b < nb; b += kBlock)
    if (cnt[b]) base[b] += atomicAdd(&cursor[b], cnt[b]);
  __syncthreads();
#pragma unroll
  for (int q = 0; q < kPer; ++q)
    if (bin[q] >= 0) order[base[bin[q]] + rank[q]] = (int32_t)(lo + q * kBlock + threadIdx.x);
#if INSITE_RK45_ORDER_SELFRESET
  // (knob) the workspace resets itself instead of the memset before the count pass: every block has read the totals
  // and taken its cursor slots before its ticket, and the last block to arrive zeroes the totals, the cursors and the
  // ticket for the next call
  __shared__ bool last;
  if (threadIdx.x == 0) {
    __threadfence();
    last = atomicAdd(cursor + nb, 1u) == gridDim.x - 1u;
  }
  __syncthreads();
  if (last) {
    __threadfence();
    for (int b = threadIdx.x; b < nb; b += kBlock) {
      hist[b] = 0u;
      cursor[b] = 0u;
    }
    if (threadIdx.x == 0) cursor[nb] = 0u;
  }
#endif
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
  if (e > kMaxEntries) return INSITE_E_UNSUPPORTED;
  // atoms: distinct u-exponent tuples of the columns
  bool fits = true;
  lib->n_atoms = 0;
  for (int j = 0; j < F; ++j) {
    int found = -1;
    for (int a = 0; a < lib->n_atoms; ++a) {
      bool same = true;
      for (int t = 0; t < INSITE_MAX_STATICS; ++t) same = same && lib->atom_exp[a][t] == (t < U ? lib->eu[j][t] : 0);
      if (same) found = a;
    }
    if (found < 0) {
      found = lib->n_atoms++;
      for (int t = 0; t < INSITE_MAX_STATICS; ++t) {
        const int8_t ee = t < U ? lib->eu[j][t] : 0;
        lib->atom_exp[found][t] = ee;
        if (ee > 2) fits = false;
      }
    }
    lib->col_atom[j] = (int8_t)found;
  }
  for (int j = 0; j < F; ++j) {
    int c = (int)lib->ex[j] << 24;
    for (int t = 0; t < U; ++t) c |= (int)lib->eu[j][t] << (8 * t);
    lib->ucode[j] = c;
  }
  // Q columns: (atom of the column index, moment) pairs, deduplicated; the atom of "1" for b
  int one_atom = -1;
  for (int a = 0; a < lib->n_atoms; ++a)
    if (lib->atom_exp[a][0] == 0 && lib->atom_exp[a][1] == 0 && lib->atom_exp[a][2] == 0) one_atom = a;
  if (one_atom < 0) {
    if (lib->n_atoms < 16) {
      one_atom = lib->n_atoms++;
      for (int t = 0; t < INSITE_MAX_STATICS; ++t) lib->atom_exp[one_atom][t] = 0;
    } else {
      fits = false;
    }
  }
  for (int a = 0; a < lib->n_atoms; ++a)
    lib->acode[a] = (int)lib->atom_exp[a][0] | (int)lib->atom_exp[a][1] << 8 | (int)lib->atom_exp[a][2] << 16;
  lib->nq = 0;
  for (int q = 0; q < lib->nE && fits; ++q) {
    const int i = lib->ei[q], k = lib->ek[q];
    const int at = k >= 0 ? lib->col_atom[k] : one_atom;
    const int mom = k >= 0 ? lib->ex[i] + lib->ex[k] : 3 + lib->ex[i];
    int found = -1;
    for (int c = 0; c < lib->nq; ++c)
      if (lib->qmom[c] == mom && lib->qatom[c] == at) found = c;
    if (found < 0) {
      if (lib->nq >= 16) {
        fits = false;
        break;
      }
      found = lib->nq++;
      lib->qmom[found] = (int8_t)mom;
      lib->qatom[found] = (int8_t)at;
    }
    lib->qcol[q] = (int8_t)found;
  }
  lib->mfma = fits ? 1 : 0;  // refined by the caller with the arm count (NARM * F <= 16)
  return INSITE_OK;
}

inline int narm_pad(int n_arms) { return n_arms <= 1 ? 1 : (n_arms <= 2 ? 2 : 4); }
// step_kernel work split over one resident round of `resident` blocks: gblocks run the gram (default
// INSITE_STEP_GSHARE per mille of the round; gram_blocks > 0 overrides), the rest the rollout.  The
// gram's time segments are chosen so its (tile, segment) items spread evenly over the gram waves
// (a wave that takes one item more than the others sets the gram's end): the segment count with the
// smallest max/mean items per wave, a small charge per extra segment for its warm-up and contraction.
// Range mode (INSITE_STEP_RANGED, default): the gram role cuts its (tile, 16-step group) units into one equal
// contiguous range per wave (gram_body, n_seg = 0), so its waves end together at any block count, and the
// default split is half the resident blocks: blocks b and b + resident/2 share a CU under the dispatcher's
// round-robin placement, so every CU holds one gram block and one rollout block (one HBM read stream and one
// write stream per CU; profiles/r03/ timelines).  Item mode (0, round 2) keeps the segment search below.
#ifndef INSITE_STEP_RANGED
#define INSITE_STEP_RANGED 1
#endif
#ifndef INSITE_STEP_SERIAL
#define INSITE_STEP_SERIAL 0  // 1: every block runs its gram range, then rollout work (step_kernel serial mode)
#endif
#ifndef INSITE_STEP_GSHARE
#define INSITE_STEP_GSHARE (INSITE_STEP_RANGED ? 500 : 600)
#endif
struct StepPlan {
  int grid, gblocks, seg, n_seg;
};
inline StepPlan step_plan(int64_t N, int64_t n_steps, int resident, int gram_blocks) {
  StepPlan pl;
  if (resident < 2) resident = 2;
  int gb = gram_blocks > 0 ? gram_blocks : (int)(((int64_t)resident * INSITE_STEP_GSHARE + 500) / 1000);
  if (gb < 1) gb = 1;
  if (gb > resident - 1) gb = resident - 1;
  if (gb > kGramMaxBlocks) gb = kGramMaxBlocks;
  pl.gblocks = gb;
  pl.grid = resident;
  if (INSITE_STEP_RANGED) {
    pl.seg = 0;
    pl.n_seg = 0;
    if (INSITE_STEP_SERIAL && gram_blocks <= 0 && resident <= kGramMaxBlocks) pl.gblocks = pl.grid;  // serial mode
    return pl;
  }
  const int64_t tiles = (N + kWave - 1) / kWave;
  const int64_t T = n_steps > 0 ? n_steps : 1;
  const int64_t gw = (int64_t)gb * kWavesPerBlock;
  const int64_t ns_max = T / 48 > 1 ? T / 48 : 1;
  double best = 1e30;
  pl.seg = (int)((T + kGT - 1) / kGT * kGT);
  pl.n_seg = 1;
  for (int64_t ns = 1; ns <= ns_max && tiles > 0; ++ns) {
    int64_t seg = (T + ns - 1) / ns;
    seg = (seg + kGT - 1) / kGT * kGT;
    const int64_t nseg = (T + seg - 1) / seg;
    const int64_t items = tiles * nseg;
    const int64_t per = (items + gw - 1) / gw;  // items of the busiest gram wave
    const double cost = (double)per * (double)seg + 24.0 * (double)(per - 1);  // steps (+ warm-up/contraction)
    if (cost < best - 1e-9) {
      best = cost;
      pl.seg = (int)seg;
      pl.n_seg = (int)nseg;
    }
  }
  return pl;
}


struct GramPlan {
  int grid, seg, n_seg;
};

// Resident wavefronts of a kernel instance on the current device (occupancy query, cached per
// instance and device; a planning hint only — correctness never depends on residency).
template <typename K>
int resident_waves(K kernel) {
  static std::atomic<int> cache[16];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) dev = 0;
  const int slot = dev < 16 ? dev : 15;
  int v = cache[slot].load(std::memory_order_relaxed);
  if (v > 0) return v;
  int cus = 0, per_cu = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kBlock, 0) != hipSuccess || per_cu <= 0) per_cu = 2;
  v = cus * per_cu * kWavesPerBlock;
  cache[slot].store(v, std::memory_order_relaxed);
  return v;
}

// Work decomposition: 64-patient tiles x time segments.  Segments add parallelism for small
// cohorts, but every work item pays a warm-up and a Gram contraction, and a second partial round
// of items leaves the chip under-occupied, so the item count is sized to one resident round.
inline GramPlan gram_plan(int64_t N, int64_t n_steps, int resident) {
  GramPlan pl;
  const int64_t tiles = (N + kWave - 1) / kWave;
  const int64_t T = n_steps > 0 ? n_steps : 1;
  int64_t ns = tiles > 0 ? resident / tiles : 1;
#ifdef INSITE_GRAM_NS_MIN
  if (ns < INSITE_GRAM_NS_MIN) ns = INSITE_GRAM_NS_MIN;
#endif
  const int64_t ns_max = T / 48 > 1 ? T / 48 : 1;
  if (ns > ns_max) ns = ns_max;
  if (ns < 1) ns = 1;
  int64_t seg = (T + ns - 1) / ns;
  seg = (seg + kGT - 1) / kGT * kGT;
  pl.seg = (int)seg;
  pl.n_seg = (int)((T + seg - 1) / seg);
  int64_t g = (tiles * pl.n_seg + kWavesPerBlock - 1) / kWavesPerBlock;
  const int64_t gres = resident / kWavesPerBlock > 0 ? resident / kWavesPerBlock : 1;
  if (g > gres) g = gres;
  if (g > kGramMaxBlocks) g = kGramMaxBlocks;
  if (g < 1) g = 1;
  pl.grid = (int)g;
  return pl;
}

constexpr size_t kGramWsHeader = 512;  // counters: gram_tail cnt[0..64] / finalize ticket (+ padding; one memset block)
static_assert((1 + (kGramMaxBlocks + kTailGroup - 1) / kTailGroup) * sizeof(unsigned) <= kGramWsHeader, "counters");
static_assert(1 + (kGramMaxBlocks + kTailGroup - 1) / kTailGroup <= kStepRcnt && (kStepRcnt + 2) * sizeof(unsigned) <= kGramWsHeader,
              "step kernel claim counters sit in the header, clear of the gram tail's");

inline int sse_grid(int64_t n_rows) {
  int64_t g = (n_rows + 63) / 64;
  if (g < 1) g = 1;
  if (g > 1024) g = 1024;
  return (int)g;
}


struct GramLaunch {
  const double* x;
  int64_t ldx;
  int n_steps;
  const double* u;
  const int8_t* arm;
  const int32_t* rows;
  int64_t N;
  GramW w;
  LibDesc lib;
  double* part;
  unsigned* cnt;  // gram_tail counters (zeroed per call); MOM: unused
  GramOut out;
};

// INSITE_GRAM_RANGED: the standalone time-major gram in range mode (gram_body, n_seg = 0) over one resident
// round instead of the (tile, segment) items of gram_plan (0 = items: C2 cold gram 50.4 vs 47.6 us ranged,
// profiles/r03/).
#ifndef INSITE_GRAM_RANGED
#define INSITE_GRAM_RANGED 1
#endif
template <int VEC, int NARM, bool SMOOTH, bool MFMA, bool TM, int MOM = 0, int STF = 0>
int launch_gram4(hipStream_t st, const GramLaunch& g) {
  auto kern = gram_kernel<VEC, NARM, SMOOTH, MFMA, TM, MOM, STF>;
  GramPlan pl = gram_plan(g.N, g.n_steps, resident_waves(kern));
  if constexpr (MOM != 0) {  // one segment per patient: the lane holds the patient's complete moments
    const int64_t tiles = (g.N + kWave - 1) / kWave;
    const int64_t gres = resident_waves(kern) / kWavesPerBlock;
    int64_t gb = (tiles + kWavesPerBlock - 1) / kWavesPerBlock;
    if (gb > gres && gres > 0) gb = gres;
    pl.grid = (int)(gb < 1 ? 1 : gb);
    pl.n_seg = 1;
    pl.seg = (int)((g.n_steps + kGT - 1) / kGT * kGT);
    if (pl.seg < kGT) pl.seg = kGT;
  } else if (INSITE_GRAM_RANGED && TM) {  // equal contiguous (tile, 16-step group) ranges over one resident round
    const int64_t units = (g.N + kWave - 1) / kWave * ((g.n_steps + kGT - 1) / kGT);
    int64_t gb = resident_waves(kern) / kWavesPerBlock;
    if (gb > (units + kWavesPerBlock - 1) / kWavesPerBlock) gb = (units + kWavesPerBlock - 1) / kWavesPerBlock;
    if (gb > kGramMaxBlocks) gb = kGramMaxBlocks;
    pl.grid = (int)(gb < 1 ? 1 : gb);
    pl.seg = 0;
    pl.n_seg = 0;
  }
  kern<<<dim3(pl.grid), kBlock, 0, st>>>(g.x, g.ldx, g.n_steps, g.u, g.arm, g.rows, g.N, pl.seg, pl.n_seg, g.w,
                                          g.lib, g.part, g.cnt, g.out);
  return pl.grid;
}

template <int NARM, bool SMOOTH, bool MFMA>
int launch_gram3(int mode, hipStream_t st, const GramLaunch& g) {  // mode: 0 PM/8-B, 1 PM/16-B, 2 TM
  if (mode == 3) return launch_gram4<1, NARM, SMOOTH, MFMA, true, 0, 7>(st, g);  // TM + fused F = 7 STLSQ
  // moments + Gram in one pass (insite_gram_moments_f64): 4 TM + fused F = 7 STLSQ, 5 TM, 6 patient-major
  if (mode == 4) return launch_gram4<1, NARM, SMOOTH, MFMA, true, 2, 7>(st, g);
  if (mode == 5) return launch_gram4<1, NARM, SMOOTH, MFMA, true, 2>(st, g);
  if (mode == 6) return launch_gram4<1, NARM, SMOOTH, MFMA, false, 2>(st, g);
  if (mode == 2) return launch_gram4<1, NARM, SMOOTH, MFMA, true>(st, g);
  if (mode == 1) return launch_gram4<2, NARM, SMOOTH, MFMA, false>(st, g);
  return launch_gram4<1, NARM, SMOOTH, MFMA, false>(st, g);
}

template <int NARM>
int launch_gram(int mode, bool smooth, hipStream_t st, const GramLaunch& g) {
  if (g.lib.mfma) {
    return smooth ? launch_gram3<NARM, true, true>(mode, st, g) : launch_gram3<NARM, false, true>(mode, st, g);
  }
  return smooth ? launch_gram3<NARM, true, false>(mode, st, g) : launch_gram3<NARM, false, false>(mode, st, g);
}

inline GramW make_gram_w(double dt) {
  GramW w;
  w.sg0 = 17.0 / 35.0;  // savgol(5,3) interior taps [-3, 12, 17, 12, -3] / 35
  w.sg1 = 12.0 / 35.0;
  w.sg2 = -3.0 / 35.0;
  w.inv_dt = 1.0 / dt;
  w.fd1 = (2.0 / 3.0) * w.inv_dt;  // 5-point first derivative [1, -8, 0, 8, -1] / 12 dt
  w.fd2 = (-1.0 / 12.0) * w.inv_dt;
  return w;
}

template <bool SMOOTH>
int launch_moments(int mode, hipStream_t st, const GramLaunch& g) {
  if (mode == 2) return launch_gram4<1, 1, SMOOTH, false, true, 1>(st, g);
  if (mode == 1) return launch_gram4<2, 1, SMOOTH, false, false, 1>(st, g);
  return launch_gram4<1, 1, SMOOTH, false, false, 1>(st, g);
}

// gram kernel with its in-launch reduction to G / b (+ the STLSQ launch when sp.enabled)
int32_t run_discovery(const double* x, int64_t ldx, int32_t layout, int32_t n_steps, const double* u,
                      const int8_t* arm, const int32_t* rows, int64_t n_patients, int32_t n_statics, int32_t n_arms,
                      const int8_t* exps, int32_t n_terms, int32_t fd_kind, double dt, double* G_out, double* b_out,
                      void* workspace, size_t workspace_bytes, void* stream, const StlsqParams& sp,
                      double* coef_out, int8_t* mask_out, int32_t* iters_out, double* mom_out = nullptr) {
  const bool tm = layout == INSITE_LAYOUT_TIME_MAJOR;
  if (layout != INSITE_LAYOUT_PATIENT_MAJOR && !tm) return INSITE_E_INVALID_ARG;
  if (n_patients < 0 || !G_out || !b_out || n_arms < 1 || n_arms > INSITE_MAX_ARMS || ldx < 1 || !(dt > 0.0) ||
      n_steps < 0 || (tm ? ldx < n_patients : ldx < n_steps))
    return INSITE_E_INVALID_ARG;
  if (n_patients > 0 && (!x || !arm || !rows || (n_statics > 0 && !u))) return INSITE_E_INVALID_ARG;
  if (fd_kind != INSITE_FD_SMOOTHED4 && fd_kind != INSITE_FD_ORDER4) return INSITE_E_UNSUPPORTED;
  LibDesc lib;
  int32_t st = build_lib(exps, n_terms, n_statics, &lib);
  if (st != INSITE_OK) return st;
  if (workspace_bytes < insite_gram_workspace_bytes(n_patients, n_arms, n_terms) || !workspace)
    return INSITE_E_WORKSPACE;
  hipStream_t hs = reinterpret_cast<hipStream_t>(stream);
  const int na = narm_pad(n_arms);
  if (na * lib.F > 16) lib.mfma = 0;
  unsigned* cnt = static_cast<unsigned*>(workspace);
  double* part = reinterpret_cast<double*>(static_cast<char*>(workspace) + kGramWsHeader);
  if (tm && ldx > ((int64_t)1 << 31) / (8 * kGT)) return INSITE_E_UNSUPPORTED;  // 32-bit tile offsets
  const bool vec2 = (ldx % 2 == 0) && ((reinterpret_cast<uintptr_t>(x) & 15u) == 0);
  const int mode = tm ? 2 : (vec2 ? 1 : 0);
  const bool smooth = fd_kind == INSITE_FD_SMOOTHED4;
  if (n_statics == 0) u = x;  // kernels load u unconditionally (values unused when U = 0)
#ifdef INSITE_GRAM_MEMSET  // ablation: re-zero gram_tail's counters with a memset node every call
  if (hipMemsetAsync(cnt, 0, kGramWsHeader, hs) != hipSuccess) return INSITE_E_HIP;
#endif
  // time-major F = 7 (C2): the STLSQ runs in the gram's last block (no second launch, G / b from LDS)
#ifndef INSITE_STLSQ_SEPARATE
  const bool fused = sp.enabled && tm && n_terms == 7;
#else
  const bool fused = false;
#endif
  const GramLaunch g{x, ldx, n_steps, u, arm, rows, n_patients, make_gram_w(dt), lib, part, cnt,
                     GramOut{G_out, b_out, n_arms, coef_out, mask_out, iters_out, sp, mom_out}};
  int lmode = fused ? 3 : mode;
  if (mom_out) {  // moments + Gram in one pass (the moments need whole trajectories: one segment per patient)
    if (!lib.mfma) return INSITE_E_UNSUPPORTED;
    lmode = tm ? (fused ? 4 : 5) : 6;
  }
  if (na == 1) launch_gram<1>(lmode, smooth, hs, g);
  else if (na == 2) launch_gram<2>(lmode, smooth, hs, g);
  else launch_gram<4>(lmode, smooth, hs, g);
  st = launch_status();
  if (st != INSITE_OK || !sp.enabled || fused) return st;
  switch (n_terms) {  // one thread per arm, register-resident STLSQ (SINDy.fit: reference sindy.py:190-192)
#define INSITE_STL_CASE(FF)                                                                             \
  case FF:                                                                                              \
    stlsq_kernel<FF><<<1, kBlock, 0, hs>>>(G_out, b_out, n_arms, sp.thr, sp.alpha, sp.max_iter, sp.unbias, \
                                           coef_out, mask_out, iters_out);                              \
    break;
    INSITE_STL_CASE(1)
    INSITE_STL_CASE(2)
    INSITE_STL_CASE(3)
    INSITE_STL_CASE(4)
    INSITE_STL_CASE(5)
    INSITE_STL_CASE(6)
    INSITE_STL_CASE(7)
    INSITE_STL_CASE(8)
    INSITE_STL_CASE(9)
#undef INSITE_STL_CASE
    default:
      return INSITE_E_UNSUPPORTED;
  }
  return launch_status();
}

inline int64_t seg_grid(int64_t N) {
  int64_t g = ((N + kWave - 1) / kWave + kWavesPerBlock - 1) / kWavesPerBlock;
  if (g > kSegMaxBlocks) g = kSegMaxBlocks;
  return g < 1 ? 1 : g;
}

template <int NARM, bool SMOOTH1, int STF>
int launch_gram_seg(hipStream_t st, const double* x, int64_t xsp, int64_t xsk, const int8_t* arm, int64_t asp,
                    int64_t ask, const int32_t* seq_len, int n_steps, const double* u, int64_t N, double inv_dt,
                    const LibDesc& lib, double* part, unsigned* cnt, const GramOut& out) {
  auto kern = gram_seg_kernel<NARM, SMOOTH1, STF>;
  // ranged: one resident round of waves, each with an equal contiguous range of (tile, chunk) units;
  // otherwise one 64-patient tile per wave up to kSegMaxBlocks blocks (the dispatcher hands freed slots to the
  // next block, which balanced the tail better than a resident grid striding over 5-6 whole tiles per wave)
  int64_t g = seg_grid(N);
  if (INSITE_SEG_RANGED) {
    const int64_t units = (N + kWave - 1) / kWave * (((n_steps > 1 ? n_steps - 1 : 1) + kSegKC - 1) / kSegKC);
    int64_t r = resident_waves(kern) / kWavesPerBlock;
    if (r > (units + kWavesPerBlock - 1) / kWavesPerBlock) r = (units + kWavesPerBlock - 1) / kWavesPerBlock;
    g = r < 1 ? 1 : (r > kSegMaxBlocks ? kSegMaxBlocks : r);
  }
  kern<<<dim3((unsigned)g), kBlock, 0, st>>>(x, xsp, xsk, arm, asp, ask, seq_len, n_steps, u, N, inv_dt, lib, part,
                                             cnt, out);
  return (int)g;
}

// segment-split Gram (+ fused finalize / STLSQ when sp.enabled): insite_gram_segments_f64 /
// insite_sindy_fit_segments_f64
int32_t run_segment_discovery(const double* x, int64_t ldx, const int8_t* arm, int64_t ld_arm, int32_t layout,
                              int32_t n_steps, const int32_t* seq_len, const double* u, int64_t n_patients,
                              int32_t n_statics, int32_t n_arms, const int8_t* exps, int32_t n_terms, int32_t fd_kind,
                              double dt, double* G_out, double* b_out, void* workspace, size_t workspace_bytes,
                              void* stream, const StlsqParams& sp, double* coef_out, int8_t* mask_out,
                              int32_t* iters_out) {
  const bool tm = layout == INSITE_LAYOUT_TIME_MAJOR;
  if (layout != INSITE_LAYOUT_PATIENT_MAJOR && !tm) return INSITE_E_INVALID_ARG;
  if (n_patients < 0 || !G_out || !b_out || n_arms < 1 || n_arms > INSITE_MAX_ARMS || !(dt > 0.0) || n_steps < 1 ||
      ldx < 1 || ld_arm < 1)
    return INSITE_E_INVALID_ARG;
  if (tm ? (ldx < n_patients || ld_arm < n_patients) : (ldx < n_steps || ld_arm < n_steps - 1))
    return INSITE_E_INVALID_ARG;
  if (n_patients > 0 && (!x || !arm || !seq_len || (n_statics > 0 && !u))) return INSITE_E_INVALID_ARG;
  if (fd_kind != INSITE_FD_ORDER1 && fd_kind != INSITE_FD_SMOOTHED1) return INSITE_E_UNSUPPORTED;
  // 32-bit buffer offsets: a chunk of kSegKC + 2 steps (time-major) or a wave's 64 rows (patient-major)
  const int64_t span = tm ? (int64_t)(kSegKC + 2) : (int64_t)kWave;
  if (ldx > ((int64_t)1 << 31) / (8 * span) || ld_arm > ((int64_t)1 << 31) / span) return INSITE_E_UNSUPPORTED;
  LibDesc lib;
  int32_t st = build_lib(exps, n_terms, n_statics, &lib);
  if (st != INSITE_OK) return st;
  if (!workspace || workspace_bytes < insite_gram_segments_workspace_bytes(n_patients, n_arms, n_terms))
    return INSITE_E_WORKSPACE;
  lib.mfma = 0;
  hipStream_t hs = reinterpret_cast<hipStream_t>(stream);
  const int na = narm_pad(n_arms);
  unsigned* ticket = static_cast<unsigned*>(workspace);
  double* part = reinterpret_cast<double*>(static_cast<char*>(workspace) + kGramWsHeader);
  if (n_statics == 0) u = x;
  if (n_patients == 0) {  // G = b = 0 (and the fit of an all-zero system) through the same finalize
    x = G_out;
    arm = reinterpret_cast<const int8_t*>(G_out);
    seq_len = reinterpret_cast<const int32_t*>(G_out);
    u = G_out;
  }
  const int64_t xsp = tm ? 1 : ldx, xsk = tm ? ldx : 1;
  const int64_t asp = tm ? 1 : ld_arm, ask = tm ? ld_arm : 1;
  const double inv_dt = 1.0 / dt;
  const bool sm = fd_kind == INSITE_FD_SMOOTHED1;
  // STLSQ fused into the tail for the cancer_sim / EQ_5 library (F = 4); other libraries: the tail writes G|b and
  // one stlsq_kernel launch fits the arms
  const bool fuse = sp.enabled && n_terms == 4;
  const GramOut go{G_out, b_out, n_arms, coef_out, mask_out, iters_out, sp, nullptr};
#define INSITE_SEG_LAUNCH(NA, SF)                                                                                      \
  sm ? launch_gram_seg<NA, true, SF>(hs, x, xsp, xsk, arm, asp, ask, seq_len, n_steps, u, n_patients, inv_dt, lib, part, \
                                     ticket, go)                                                                       \
     : launch_gram_seg<NA, false, SF>(hs, x, xsp, xsk, arm, asp, ask, seq_len, n_steps, u, n_patients, inv_dt, lib,    \
                                      part, ticket, go)
  if (fuse) {
    if (na == 1) INSITE_SEG_LAUNCH(1, 4);
    else if (na == 2) INSITE_SEG_LAUNCH(2, 4);
    else INSITE_SEG_LAUNCH(4, 4);
  } else {
    if (na == 1) INSITE_SEG_LAUNCH(1, 0);
    else if (na == 2) INSITE_SEG_LAUNCH(2, 0);
    else INSITE_SEG_LAUNCH(4, 0);
  }
#undef INSITE_SEG_LAUNCH
  st = launch_status();
  if (st != INSITE_OK || !sp.enabled || fuse) return st;
  return insite_stlsq_f64(G_out, b_out, n_arms, n_terms, sp.thr, sp.alpha, sp.max_iter, sp.unbias, coef_out, mask_out,
                          iters_out, stream);
}

template <int METHOD, int NARM, bool PERROW>
void launch_rollout_a(int av, bool yv2, dim3 grid, hipStream_t st, const RolloutArgs& ra, const LibDesc& lib) {
  if (yv2) {
    if (av == 16) rollout_kernel<METHOD, NARM, PERROW, 16, 2><<<grid, kBlock, 0, st>>>(ra, lib);
    else if (av == 4) rollout_kernel<METHOD, NARM, PERROW, 4, 2><<<grid, kBlock, 0, st>>>(ra, lib);
    else rollout_kernel<METHOD, NARM, PERROW, 1, 2><<<grid, kBlock, 0, st>>>(ra, lib);
  } else {
    if (av == 16) rollout_kernel<METHOD, NARM, PERROW, 16, 1><<<grid, kBlock, 0, st>>>(ra, lib);
    else if (av == 4) rollout_kernel<METHOD, NARM, PERROW, 4, 1><<<grid, kBlock, 0, st>>>(ra, lib);
    else rollout_kernel<METHOD, NARM, PERROW, 1, 1><<<grid, kBlock, 0, st>>>(ra, lib);
  }
}

template <int METHOD, int NARM>
void launch_rollout_p(bool perrow, int av, bool yv2, dim3 grid, hipStream_t st, const RolloutArgs& ra,
                      const LibDesc& lib) {
  if (perrow) launch_rollout_a<METHOD, NARM, true>(av, yv2, grid, st, ra, lib);
  else launch_rollout_a<METHOD, NARM, false>(av, yv2, grid, st, ra, lib);
}

template <int METHOD, int NARM, int PPL>
void launch_rollout_tm_w(bool perrow, int afmt, dim3 grid, hipStream_t st, const RolloutArgs& ra, const LibDesc& lib) {
  // PPL > 1 is only chosen with dword-aligned arm rows (the lane's PPL int8 arms share one dword)
  if (afmt == kArmBits) {
    if (perrow) rollout_tm_kernel<METHOD, NARM, true, PPL, kArmBits><<<grid, kBlock, 0, st>>>(ra, lib);
    else rollout_tm_kernel<METHOD, NARM, false, PPL, kArmBits><<<grid, kBlock, 0, st>>>(ra, lib);
  } else if (PPL > 1 || afmt == kArmDword) {
    if (perrow) rollout_tm_kernel<METHOD, NARM, true, PPL, kArmDword><<<grid, kBlock, 0, st>>>(ra, lib);
    else rollout_tm_kernel<METHOD, NARM, false, PPL, kArmDword><<<grid, kBlock, 0, st>>>(ra, lib);
  } else {
    if (perrow) rollout_tm_kernel<METHOD, NARM, true, 1, kArmByte><<<grid, kBlock, 0, st>>>(ra, lib);
    else rollout_tm_kernel<METHOD, NARM, false, 1, kArmByte><<<grid, kBlock, 0, st>>>(ra, lib);
  }
}

template <int METHOD, int NARM>
void launch_rollout_tm(bool perrow, int ppl, int afmt, dim3 grid, hipStream_t st, const RolloutArgs& ra,
                       const LibDesc& lib) {
  if (ppl == 4) launch_rollout_tm_w<METHOD, NARM, 4>(perrow, afmt, grid, st, ra, lib);
  else if (ppl == 2) launch_rollout_tm_w<METHOD, NARM, 2>(perrow, afmt, grid, st, ra, lib);
  else launch_rollout_tm_w<METHOD, NARM, 1>(perrow, afmt, grid, st, ra, lib);
}

template <int METHOD>
void launch_rollout_m(int narm, bool perrow, int av, bool yv2, dim3 grid, hipStream_t st,
                      const RolloutArgs& ra, const LibDesc& lib) {
  if (narm == 1) launch_rollout_p<METHOD, 1>(perrow, av, yv2, grid, st, ra, lib);
  else if (narm == 2) launch_rollout_p<METHOD, 2>(perrow, av, yv2, grid, st, ra, lib);
  else launch_rollout_p<METHOD, 4>(perrow, av, yv2, grid, st, ra, lib);
}

template <int METHOD>
void launch_rollout_tm_m(int narm, bool perrow, int ppl, int afmt, dim3 grid, hipStream_t st, const RolloutArgs& ra,
                         const LibDesc& lib) {
  if (narm == 1) launch_rollout_tm<METHOD, 1>(perrow, ppl, afmt, grid, st, ra, lib);
  else if (narm == 2) launch_rollout_tm<METHOD, 2>(perrow, ppl, afmt, grid, st, ra, lib);
  else launch_rollout_tm<METHOD, 4>(perrow, ppl, afmt, grid, st, ra, lib);
}

// one thread per patient: STLSQ from the global support on the patient's moments (patient_fit_kernel)
int32_t launch_patient_fit(const double* mom, const double* u, const int8_t* arm, const int32_t* rows, int64_t n_patients,
                           int32_t n_steps, int32_t n_arms, const LibDesc& lib, const double* global_coef,
                           const StlsqParams& sp, double* coef_out, int8_t* mask_out, int32_t* iters_out,
                           hipStream_t hs) {
  const dim3 grid((unsigned)((n_patients + kBlock - 1) / kBlock));
  switch (lib.F) {
#define INSITE_PP_CASE(FF)                                                                                      \
  case FF:                                                                                                     \
    if (sp.alpha > 0.0)                                                                                        \
      patient_fit_kernel<FF, false><<<grid, kBlock, 0, hs>>>(mom, u, arm, rows, n_patients, n_steps, n_arms, lib, \
                                                             global_coef, sp, coef_out, mask_out, iters_out);  \
    else                                                                                                       \
      patient_fit_kernel<FF, true><<<grid, kBlock, 0, hs>>>(mom, u, arm, rows, n_patients, n_steps, n_arms, lib,  \
                                                            global_coef, sp, coef_out, mask_out, iters_out);   \
    break;
    INSITE_PP_CASE(1)
    INSITE_PP_CASE(2)
    INSITE_PP_CASE(3)
    INSITE_PP_CASE(4)
    INSITE_PP_CASE(5)
    INSITE_PP_CASE(6)
    INSITE_PP_CASE(7)
    INSITE_PP_CASE(8)
    INSITE_PP_CASE(9)
#undef INSITE_PP_CASE
    default:
      return INSITE_E_UNSUPPORTED;
  }
  return launch_status();
}

}  // namespace

// =============================================================================================
// C ABI
// =============================================================================================
extern "C" {

int32_t insite_abi_version(void) { return INSITE_ABI_VERSION; }

#ifdef INSITE_TIMING
// profiling builds only: copy / clear the phase timestamps (host buffer of kTsWaves * kTsSlots u64)
int32_t insite_debug_tstamps(unsigned long long* host, int32_t clear) {
  if (clear) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_tstamp)) != hipSuccess) return INSITE_E_HIP;
    return hipMemset(p, 0, sizeof(unsigned long long) * kTsWaves * kTsSlots) == hipSuccess ? INSITE_OK : INSITE_E_HIP;
  }
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_tstamp), sizeof(unsigned long long) * kTsWaves * kTsSlots) == hipSuccess
             ? INSITE_OK : INSITE_E_HIP;
}
#endif

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
  const size_t per_block = narm_pad(n_arms) * kWave > 256 ? (size_t)narm_pad(n_arms) * kWave : 256;
  const size_t groups = (kGramMaxBlocks + kTailGroup - 1) / kTailGroup;  // gram_tail's group partials
  return kGramWsHeader + (size_t)(kGramMaxBlocks + groups) * per_block * sizeof(double);  // >= compact size
}

int32_t insite_gram_f64(const double* x, int64_t ldx, int32_t layout, int32_t n_steps, const double* u,
                        const int8_t* arm, const int32_t* rows, int64_t n_patients, int32_t n_statics,
                        int32_t n_arms, const int8_t* exps, int32_t n_terms, int32_t fd_kind, double dt,
                        double* G_out, double* b_out, void* workspace, size_t workspace_bytes,
                        void* stream) {
  StlsqParams sp{0.0, 0.0, 0, 0, 0};
  return run_discovery(x, ldx, layout, n_steps, u, arm, rows, n_patients, n_statics, n_arms, exps, n_terms, fd_kind,
                       dt, G_out, b_out, workspace, workspace_bytes, stream, sp, nullptr, nullptr, nullptr);
}

// insite_fit_rollout_f64 (deferred = 0) and insite_fit_rollout_deferred_f64 (deferred = 1: partial slot `slot`,
// finalise the other slot when finalize_prev).
static int32_t run_fit_rollout(const double* x, int64_t ldx, int32_t n_steps, const double* u, const int8_t* arm,
                               const int32_t* rows, int64_t n_patients, int32_t n_statics, int32_t n_arms,
                               const int8_t* exps, int32_t n_terms, int32_t fd_kind, double dt, double threshold,
                               double alpha, int32_t max_iter, int32_t unbias, double* G_out, double* b_out,
                               double* coef_out, int8_t* mask_out, int32_t* iters_out, const double* y0,
                               const double* ru, const uint32_t* arm_bits, int64_t ld_arm, const double* coef_in,
                               int64_t n_rows, int32_t T, double rdt, int32_t method, int32_t substeps,
                               double drop_below, double* y_out, int64_t ld_y, int32_t gram_blocks, void* workspace,
                               size_t workspace_bytes, void* stream, int deferred, int32_t slot, int32_t finalize_prev,
                               int lagged = 0, const double* G_fit = nullptr, const double* b_fit = nullptr) {
  // ---- discovery half: insite_sindy_fit_f64's checks, restricted to the fused kernel's shape ----
  if (n_patients < 0 || !G_out || !b_out || !coef_out || n_arms != 2 || ldx < 1 || !(dt > 0.0) || n_steps < 0 ||
      ldx < n_patients || max_iter < 0 || !(threshold >= 0.0) || !(alpha >= 0.0))
    return INSITE_E_INVALID_ARG;
  if (n_patients > 0 && (!x || !arm || !rows || (n_statics > 0 && !u))) return INSITE_E_INVALID_ARG;
  if (fd_kind != INSITE_FD_SMOOTHED4 && fd_kind != INSITE_FD_ORDER4) return INSITE_E_UNSUPPORTED;
  if (n_terms != 7) return INSITE_E_UNSUPPORTED;  // the fused STLSQ is instantiated for F = 7 (C2's library)
  LibDesc lib;
  int32_t st = build_lib(exps, n_terms, n_statics, &lib);
  if (st != INSITE_OK) return st;
  if (!lib.mfma) return INSITE_E_UNSUPPORTED;
  {  // state degree <= 1 (the affine rollout)
    for (int j = 0; j < n_terms; ++j)
      if (exps[j * (1 + n_statics)] > INSITE_MAX_STATE_DEGREE) return INSITE_E_UNSUPPORTED;
  }
  const size_t ws_one = insite_gram_workspace_bytes(n_patients, n_arms, n_terms);
  if (!workspace || workspace_bytes < (deferred ? 2 * ws_one + kDefAreaBytes : ws_one)) return INSITE_E_WORKSPACE;
  if (deferred && (slot < 0 || slot > 1 || finalize_prev < 0 || finalize_prev > 1)) return INSITE_E_INVALID_ARG;
  if (lagged && ((G_fit == nullptr) != (b_fit == nullptr))) return INSITE_E_INVALID_ARG;
  if (ldx > ((int64_t)1 << 31) / (8 * kGT)) return INSITE_E_UNSUPPORTED;
  // ---- rollout half: insite_rollout_f64's checks for TIME_MAJOR_BITS, shared library ----
  // ld_arm > 0: time-major bits [T, ld_arm]; ld_arm < 0: tile-major bits [ceil(n_rows / 64)][-ld_arm >= T][2]
  if (n_rows < 0 || T < 0 || substeps < 1 || !(rdt >= 0.0) || ld_y < n_rows ||
      (ld_arm >= 0 ? ld_arm < (n_rows + 31) / 32 : -ld_arm < (int64_t)T))
    return INSITE_E_INVALID_ARG;
  if (method != INSITE_METHOD_EULER && method != INSITE_METHOD_RK4) return INSITE_E_UNSUPPORTED;
  const bool roll = n_rows > 0 && T > 0;
  if (roll && (!y0 || !arm_bits || !coef_in || !y_out || (n_statics > 0 && !ru))) return INSITE_E_INVALID_ARG;
  if (roll && (reinterpret_cast<uintptr_t>(arm_bits) & 3u) != 0) return INSITE_E_INVALID_ARG;
  if ((ld_arm >= 0 ? ld_arm * 4 : (int64_t)8) > kTmMaxLd || ld_y > kTmMaxLd) return INSITE_E_UNSUPPORTED;
  if (gram_blocks < 0) return INSITE_E_INVALID_ARG;
  hipStream_t hs = reinterpret_cast<hipStream_t>(stream);
  RolloutArgs ra;
  ra.y0 = roll ? y0 : coef_out;  // empty rollout: pointers never dereferenced (no units)
  ra.u = (roll && n_statics > 0) ? ru : ra.y0;
  ra.arm = reinterpret_cast<const int8_t*>(roll ? (const void*)arm_bits : (const void*)coef_out);
  ra.coef = roll ? coef_in : coef_out;
  ra.y = roll ? y_out : coef_out;
  ra.lda = ld_arm;
  ra.ldy = ld_y;
  ra.coef_stride = 0;
  ra.N = roll ? n_rows : 0;
  ra.T = roll ? T : 1;
  ra.substeps = substeps;
  ra.A = n_arms;
  ra.dt = rdt;
  ra.drop = drop_below;
  const StlsqParams sp{threshold, alpha, max_iter, unbias, 1};
  const GramOut go{G_out, b_out, n_arms, coef_out, mask_out, iters_out, sp};
  unsigned* cnt = static_cast<unsigned*>(workspace);
  double* part = reinterpret_cast<double*>(static_cast<char*>(workspace) + kGramWsHeader);
  const bool smooth = fd_kind == INSITE_FD_SMOOTHED4;
  if (n_statics == 0) u = x ? x : G_out;
  if (deferred) {
    auto pick = [&](auto k_t_rk4, auto k_t_eu, auto k_f_rk4, auto k_f_eu) {
      return smooth ? (method == INSITE_METHOD_RK4 ? k_t_rk4 : k_t_eu) : (method == INSITE_METHOD_RK4 ? k_f_rk4 : k_f_eu);
    };
    auto kd0 = pick(step_deferred_kernel<true, INSITE_METHOD_RK4, 0>, step_deferred_kernel<true, INSITE_METHOD_EULER, 0>,
                    step_deferred_kernel<false, INSITE_METHOD_RK4, 0>, step_deferred_kernel<false, INSITE_METHOD_EULER, 0>);
    auto kd1 = pick(step_deferred_kernel<true, INSITE_METHOD_RK4, 1>, step_deferred_kernel<true, INSITE_METHOD_EULER, 1>,
                    step_deferred_kernel<false, INSITE_METHOD_RK4, 1>, step_deferred_kernel<false, INSITE_METHOD_EULER, 1>);
    const int nfin = lagged && !INSITE_LAG_MERGED ? 2 : 1;  // finalisation blocks (the reduction [+ the STLSQ])
    // half the resident blocks stream the gram (blocks b and b + grid/2 share a CU), nfin finalise, the rest roll out
    auto split = [&](auto k, int& grid_, int& gb_) {
      grid_ = resident_waves(k) / kWavesPerBlock;
      if (grid_ < 2 + nfin) grid_ = 2 + nfin;
      gb_ = gram_blocks > 0 ? gram_blocks : grid_ / 2;
      if (gb_ > grid_ - 1 - nfin) gb_ = grid_ - 1 - nfin;
      if (gb_ > kGramMaxBlocks) gb_ = kGramMaxBlocks;
    };
    int grid = 0, gb = 0;
    split(kd0, grid, gb);
    // the claimed gram tail (INSITE_DEF_DYN) where the gram waves' ranges are long enough to pay for it
    const int64_t units_all = (n_patients + kWave - 1) / kWave * ((n_steps + kGT - 1) / kGT);
    const bool dyn = n_patients > 0 && (INSITE_DEF_DYN == 1 ||
                                        (INSITE_DEF_DYN == 2 && units_all >= (int64_t)INSITE_DEF_DYN_MIN * gb * kWavesPerBlock));
    if (dyn) split(kd1, grid, gb);
    // INSITE_DEF_ROVS > 1: the rollout blocks oversubscribe the resident round (shorter ranges, the dispatcher hands
    // the later ones to whichever CU frees a slot first); y does not depend on the ranges (rollout_bits_range)
    if (INSITE_DEF_ROVS > 1) grid = gb + nfin + (grid - gb - nfin) * INSITE_DEF_ROVS;
    char* wsb = static_cast<char*>(workspace);
    char* slots = wsb + kDefAreaBytes;
    double* part_cur = reinterpret_cast<double*>(slots + (size_t)slot * ws_one + kGramWsHeader);
    const double* part_prev =
        finalize_prev ? reinterpret_cast<const double*>(slots + (size_t)(1 - slot) * ws_one + kGramWsHeader) : nullptr;
    unsigned* hdr_cur = reinterpret_cast<unsigned*>(slots + (size_t)slot * ws_one);
    const unsigned* hdr_prev = reinterpret_cast<const unsigned*>(slots + (size_t)(1 - slot) * ws_one);
    // lagged: `go` reduces only (G|b out, no STLSQ); `gf` solves the all-reduced G_fit|b_fit into coef/mask/iters
    const GramOut gred{G_out, b_out, n_arms, nullptr, nullptr, nullptr, sp};
    const GramOut gf{nullptr, nullptr, n_arms, coef_out, mask_out, iters_out, sp};
    if (n_patients == 0) {  // the gram blocks leave zero partials
      x = G_out;
      arm = reinterpret_cast<const int8_t*>(G_out);
      rows = reinterpret_cast<const int32_t*>(G_out);
      u = G_out;
    }
    // the claim area at offset 0 (the claimed rollout tail's, INSITE_DEF_RSTATIC < 1000, a knob build: zeroed before
    // every launch, since the chunks its heads skip would otherwise go unrolled silently)
    unsigned* rc = INSITE_DEF_RSTATIC < 1000 ? reinterpret_cast<unsigned*>(wsb + kDefRollClaimOff) : nullptr;
    if (rc && hipMemsetAsync(rc, 0, kDefClaimBytes, hs) != hipSuccess) return INSITE_E_HIP;
    // the claimed gram tail (INSITE_DEF_DYN): its heads in the same area, self-resetting; a stale area shows up as a
    // piece count that does not add up, which the next finalisation flags (NaN G|b, iters -3)
    DynGram dg{reinterpret_cast<unsigned*>(wsb), nullptr, hdr_cur, 0, 0, 1, 1, gb * kWavesPerBlock};
    if (dyn) {
      const int64_t n_tiles = (n_patients + kWave - 1) / kWave;
      const int ngs = (n_steps + kGT - 1) / kGT;
      const int n_ent = n_arms * lib.nE;
      const size_t per_block = narm_pad(n_arms) * kWave > 256 ? (size_t)narm_pad(n_arms) * kWave : 256;
      const int64_t rows_cap = (int64_t)((kGramMaxBlocks + (kGramMaxBlocks + kTailGroup - 1) / kTailGroup) * per_block /
                                         (size_t)n_ent);
      const int64_t pcap = rows_cap - gb;  // piece rows after the gb block rows, inside one slot
      int64_t tail = n_tiles * INSITE_DEF_DYN_TAIL / 1000;
      int pg = INSITE_DEF_DYN_PG < 1 ? 1 : (INSITE_DEF_DYN_PG > ngs ? ngs : INSITE_DEF_DYN_PG);
      int ppt = (ngs + pg - 1) / pg;
      if (tail * ppt > pcap && tail > 0) {  // coarser pieces, then fewer tail tiles, to stay inside the slot
        const int64_t pmax = pcap / tail > 1 ? pcap / tail : 1;
        pg = (int)((ngs + pmax - 1) / pmax);
        ppt = (ngs + pg - 1) / pg;
        if (tail * ppt > pcap) tail = pcap / ppt;
      }
      dg.ppart = part_cur + (int64_t)gb * n_ent;
      dg.tile0 = n_tiles - tail;
      dg.P = tail * ppt;
      dg.pg = pg;
      dg.ppt = ppt;
    }
    auto kd = dyn ? kd1 : kd0;
    kd<<<dim3(grid), kBlock, 0, hs>>>(x, ldx, n_steps, u, arm, rows, n_patients, make_gram_w(dt), lib, part_cur,
                                      part_prev, lagged ? gred : go, ra, gb, rc, hdr_cur, hdr_prev, lagged, G_fit,
                                      b_fit, gf, slot_fingerprint(lib, n_arms), dg);
    return launch_status();
  }
  // (a two-patients-per-lane rollout role with 16-B stores measured slower: 46 vs 37 us rollout-only)
  auto kern = smooth ? (method == INSITE_METHOD_RK4 ? step_kernel<true, INSITE_METHOD_RK4> : step_kernel<true, INSITE_METHOD_EULER>)
                     : (method == INSITE_METHOD_RK4 ? step_kernel<false, INSITE_METHOD_RK4> : step_kernel<false, INSITE_METHOD_EULER>);
  const StepPlan pl = step_plan(n_patients, n_steps, resident_waves(kern) / kWavesPerBlock, gram_blocks);
  if (n_patients == 0) {  // G = b = 0 and the fit of the zero system, through the same tail
    x = G_out;
    arm = reinterpret_cast<const int8_t*>(G_out);
    rows = reinterpret_cast<const int32_t*>(G_out);
    u = G_out;
  }
  kern<<<dim3(pl.grid), kBlock, 0, hs>>>(x, ldx, n_steps, u, arm, rows, n_patients, pl.seg, pl.n_seg,
                                        make_gram_w(dt), lib, part, cnt, go, ra, pl.gblocks);
  return launch_status();
}

int32_t insite_fit_rollout_f64(const double* x, int64_t ldx, int32_t n_steps, const double* u, const int8_t* arm,
                               const int32_t* rows, int64_t n_patients, int32_t n_statics, int32_t n_arms,
                               const int8_t* exps, int32_t n_terms, int32_t fd_kind, double dt, double threshold,
                               double alpha, int32_t max_iter, int32_t unbias, double* G_out, double* b_out,
                               double* coef_out, int8_t* mask_out, int32_t* iters_out, const double* y0,
                               const double* ru, const uint32_t* arm_bits, int64_t ld_arm, const double* coef_in,
                               int64_t n_rows, int32_t T, double rdt, int32_t method, int32_t substeps,
                               double drop_below, double* y_out, int64_t ld_y, int32_t gram_blocks, void* workspace,
                               size_t workspace_bytes, void* stream) {
  return run_fit_rollout(x, ldx, n_steps, u, arm, rows, n_patients, n_statics, n_arms, exps, n_terms, fd_kind, dt,
                         threshold, alpha, max_iter, unbias, G_out, b_out, coef_out, mask_out, iters_out, y0, ru,
                         arm_bits, ld_arm, coef_in, n_rows, T, rdt, method, substeps, drop_below, y_out, ld_y,
                         gram_blocks, workspace, workspace_bytes, stream, 0, 0, 0);
}

size_t insite_fit_rollout_deferred_workspace_bytes(int64_t n_patients, int32_t n_arms, int32_t n_terms) {
  const size_t one = insite_gram_workspace_bytes(n_patients, n_arms, n_terms);
  return one ? 2 * one + kDefAreaBytes : 0;
}

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
                                        void* stream) {
  return run_fit_rollout(x, ldx, n_steps, u, arm, rows, n_patients, n_statics, n_arms, exps, n_terms, fd_kind, dt,
                         threshold, alpha, max_iter, unbias, G_out, b_out, coef_out, mask_out, iters_out, y0, ru,
                         arm_bits, ld_arm, coef_in, n_rows, T, rdt, method, substeps, drop_below, y_out, ld_y,
                         gram_blocks, workspace, workspace_bytes, stream, 1, slot, finalize_prev);
}

int32_t insite_fit_rollout_lagged_f64(const double* x, int64_t ldx, int32_t n_steps, const double* u,
                                      const int8_t* arm, const int32_t* rows, int64_t n_patients, int32_t n_statics,
                                      int32_t n_arms, const int8_t* exps, int32_t n_terms, int32_t fd_kind, double dt,
                                      double threshold, double alpha, int32_t max_iter, int32_t unbias, double* G_out,
                                      double* b_out, const double* G_fit, const double* b_fit, double* coef_out,
                                      int8_t* mask_out, int32_t* iters_out, const double* y0, const double* ru,
                                      const uint32_t* arm_bits, int64_t ld_arm, const double* coef_in, int64_t n_rows,
                                      int32_t T, double rdt, int32_t method, int32_t substeps, double drop_below,
                                      double* y_out, int64_t ld_y, int32_t gram_blocks, int32_t slot,
                                      int32_t reduce_prev, void* workspace, size_t workspace_bytes, void* stream) {
  if (G_fit && !coef_out) return INSITE_E_INVALID_ARG;
  double* co = coef_out ? coef_out : G_out;  // run_fit_rollout's non-null check; never written without G_fit
  return run_fit_rollout(x, ldx, n_steps, u, arm, rows, n_patients, n_statics, n_arms, exps, n_terms, fd_kind, dt,
                         threshold, alpha, max_iter, unbias, G_out, b_out, co, coef_out ? mask_out : nullptr,
                         coef_out ? iters_out : nullptr, y0, ru, arm_bits, ld_arm, coef_in, n_rows, T, rdt, method,
                         substeps, drop_below, y_out, ld_y, gram_blocks, workspace, workspace_bytes, stream, 1, slot,
                         reduce_prev, 1, G_fit, b_fit);
}

int32_t insite_sindy_fit_f64(const double* x, int64_t ldx, int32_t layout, int32_t n_steps, const double* u,
                             const int8_t* arm, const int32_t* rows, int64_t n_patients, int32_t n_statics,
                             int32_t n_arms, const int8_t* exps, int32_t n_terms, int32_t fd_kind, double dt,
                             double threshold, double alpha, int32_t max_iter, int32_t unbias,
                             double* G_out, double* b_out, double* coef_out, int8_t* mask_out,
                             int32_t* iters_out, void* workspace, size_t workspace_bytes, void* stream) {
  if (!coef_out || max_iter < 0 || !(threshold >= 0.0) || !(alpha >= 0.0)) return INSITE_E_INVALID_ARG;
  StlsqParams sp{threshold, alpha, max_iter, unbias, 1};
  return run_discovery(x, ldx, layout, n_steps, u, arm, rows, n_patients, n_statics, n_arms, exps, n_terms, fd_kind,
                       dt, G_out, b_out, workspace, workspace_bytes, stream, sp, coef_out, mask_out, iters_out);
}

int32_t insite_gram_moments_f64(const double* x, int64_t ldx, int32_t layout, int32_t n_steps, const double* u,
                                const int8_t* arm, const int32_t* rows, int64_t n_patients, int32_t n_statics,
                                int32_t n_arms, const int8_t* exps, int32_t n_terms, int32_t fd_kind, double dt,
                                double threshold, double alpha, int32_t max_iter, int32_t unbias, double* G_out,
                                double* b_out, double* coef_out, int8_t* mask_out, int32_t* iters_out, double* mom_out,
                                void* workspace, size_t workspace_bytes, void* stream) {
  if (!mom_out || max_iter < 0 || !(threshold >= 0.0) || !(alpha >= 0.0)) return INSITE_E_INVALID_ARG;
  const StlsqParams sp{threshold, alpha, max_iter, unbias, coef_out ? 1 : 0};
  return run_discovery(x, ldx, layout, n_steps, u, arm, rows, n_patients, n_statics, n_arms, exps, n_terms, fd_kind,
                       dt, G_out, b_out, workspace, workspace_bytes, stream, sp, coef_out, mask_out, iters_out, mom_out);
}

int32_t insite_fit_per_patient_moments_f64(const double* mom, const double* u, const int8_t* arm, const int32_t* rows,
                                           int64_t n_patients, int32_t n_steps, int32_t n_statics, int32_t n_arms,
                                           const int8_t* exps, int32_t n_terms, const double* global_coef,
                                           double threshold, double alpha, int32_t max_iter, int32_t unbias,
                                           double* coef_out, int8_t* mask_out, int32_t* iters_out, void* stream) {
  if (n_patients < 0 || n_arms < 1 || n_arms > INSITE_MAX_ARMS || n_steps < 0 || max_iter < 0 ||
      !(threshold >= 0.0) || !(alpha >= 0.0))
    return INSITE_E_INVALID_ARG;
  LibDesc lib;
  int32_t st = build_lib(exps, n_terms, n_statics, &lib);
  if (st != INSITE_OK) return st;
  if (n_patients == 0) return INSITE_OK;
  if (!mom || !arm || !rows || !global_coef || !coef_out || (n_statics > 0 && !u)) return INSITE_E_INVALID_ARG;
  if (n_statics == 0) u = mom;
  return launch_patient_fit(mom, u, arm, rows, n_patients, n_steps, n_arms, lib, global_coef,
                            StlsqParams{threshold, alpha, max_iter, unbias, 1}, coef_out, mask_out, iters_out,
                            reinterpret_cast<hipStream_t>(stream));
}

int32_t insite_refit_rollout_moments_f64(const double* mom, const int8_t* arm, const int32_t* rows, int64_t n_patients,
                                         int32_t n_steps, int32_t n_statics, int32_t n_arms, const int8_t* exps,
                                         int32_t n_terms, const double* global_coef, double threshold, double alpha,
                                         int32_t max_iter, int32_t unbias, const double* y0, const double* u,
                                         const uint32_t* arm_bits, int64_t ld_bits, int32_t T, double dt,
                                         int32_t method, int32_t substeps, double drop_below, double* y_out,
                                         int64_t ld_y, double* coef_out, int8_t* mask_out, int32_t* iters_out,
                                         void* stream) {
  if (n_patients < 0 || n_arms < 1 || n_arms > 2 || n_steps < 0 || max_iter < 0 || !(threshold >= 0.0) ||
      !(alpha >= 0.0) || T < 0 || substeps < 1 || !(dt >= 0.0) ||
      (ld_bits >= 0 ? ld_bits < (n_patients + 31) / 32 : -ld_bits < (int64_t)T) ||  // < 0: tile-major bits
      ld_y < n_patients)
    return INSITE_E_INVALID_ARG;
  if (method != INSITE_METHOD_EULER && method != INSITE_METHOD_RK4) return INSITE_E_UNSUPPORTED;
  if (!(alpha > 0.0)) return INSITE_E_UNSUPPORTED;  // the closed-form refit needs a ridge: use the two calls
  LibDesc lib;
  int32_t st = build_lib(exps, n_terms, n_statics, &lib);
  if (st != INSITE_OK) return st;
  for (int j = 0; j < n_terms; ++j)
    if (exps[j * (1 + n_statics)] > 1) return INSITE_E_UNSUPPORTED;  // state degree <= 1 (the moments' model)
  if (n_patients == 0 || T == 0) return INSITE_OK;
  if (!mom || !arm || !rows || !global_coef || !y0 || !arm_bits || !y_out || (n_statics > 0 && !u))
    return INSITE_E_INVALID_ARG;
  if ((reinterpret_cast<uintptr_t>(arm_bits) & 3u) != 0) return INSITE_E_INVALID_ARG;
  if ((ld_bits >= 0 ? ld_bits * 4 : (int64_t)8) > kTmMaxLd || ld_y > kTmMaxLd) return INSITE_E_UNSUPPORTED;
  RolloutArgs ra;
  ra.y0 = y0;
  ra.u = n_statics == 0 ? y0 : u;
  ra.arm = reinterpret_cast<const int8_t*>(arm_bits);
  ra.coef = global_coef;
  ra.y = y_out;
  ra.lda = ld_bits;
  ra.ldy = ld_y;
  ra.coef_stride = 0;
  ra.N = n_patients;
  ra.T = T;
  ra.substeps = substeps;
  ra.A = n_arms;
  ra.dt = dt;
  ra.drop = drop_below;
  RefitArgs rf{mom, arm, rows, global_coef, coef_out, mask_out, iters_out,
               StlsqParams{threshold, alpha, max_iter, unbias, 1}, n_steps};
  hipStream_t hs = reinterpret_cast<hipStream_t>(stream);
  const int64_t tiles = (n_patients + kWave - 1) / kWave;
  const dim3 grid((unsigned)((tiles + kWavesPerBlock - 1) / kWavesPerBlock));
  const int na = narm_pad(n_arms);
  if (method == INSITE_METHOD_EULER) {
    if (na == 1) refit_rollout_kernel<INSITE_METHOD_EULER, 1><<<grid, kBlock, 0, hs>>>(ra, lib, rf);
    else refit_rollout_kernel<INSITE_METHOD_EULER, 2><<<grid, kBlock, 0, hs>>>(ra, lib, rf);
  } else {
    if (na == 1) refit_rollout_kernel<INSITE_METHOD_RK4, 1><<<grid, kBlock, 0, hs>>>(ra, lib, rf);
    else refit_rollout_kernel<INSITE_METHOD_RK4, 2><<<grid, kBlock, 0, hs>>>(ra, lib, rf);
  }
  return launch_status();
}

size_t insite_gram_segments_workspace_bytes(int64_t n_patients, int32_t n_arms, int32_t n_terms) {
  (void)n_terms;
  if (n_patients < 0 || n_arms < 1 || n_arms > INSITE_MAX_ARMS) return 0;
  // block partials [grid][n_arms * nE] and <= kTailMaxGroups group partials (gram_tail), nE <= 54
  const size_t ent = (size_t)n_arms * (INSITE_MAX_TERMS * (INSITE_MAX_TERMS + 1) / 2 + INSITE_MAX_TERMS);
  return kGramWsHeader + ((size_t)seg_grid(n_patients) + kTailMaxGroups) * ent * sizeof(double);
}

int32_t insite_gram_segments_f64(const double* x, int64_t ldx, const int8_t* arm, int64_t ld_arm, int32_t layout,
                                 int32_t n_steps, const int32_t* seq_len, const double* u, int64_t n_patients,
                                 int32_t n_statics, int32_t n_arms, const int8_t* exps, int32_t n_terms,
                                 int32_t fd_kind, double dt, double* G_out, double* b_out, void* workspace,
                                 size_t workspace_bytes, void* stream) {
  StlsqParams sp{0.0, 0.0, 0, 0, 0};
  return run_segment_discovery(x, ldx, arm, ld_arm, layout, n_steps, seq_len, u, n_patients, n_statics, n_arms, exps,
                               n_terms, fd_kind, dt, G_out, b_out, workspace, workspace_bytes, stream, sp, nullptr,
                               nullptr, nullptr);
}

int32_t insite_sindy_fit_segments_f64(const double* x, int64_t ldx, const int8_t* arm, int64_t ld_arm, int32_t layout,
                                      int32_t n_steps, const int32_t* seq_len, const double* u, int64_t n_patients,
                                      int32_t n_statics, int32_t n_arms, const int8_t* exps, int32_t n_terms,
                                      int32_t fd_kind, double dt, double threshold, double alpha, int32_t max_iter,
                                      int32_t unbias, double* G_out, double* b_out, double* coef_out, int8_t* mask_out,
                                      int32_t* iters_out, void* workspace, size_t workspace_bytes, void* stream) {
  if (!coef_out || max_iter < 0 || !(threshold >= 0.0) || !(alpha >= 0.0)) return INSITE_E_INVALID_ARG;
  StlsqParams sp{threshold, alpha, max_iter, unbias, 1};
  return run_segment_discovery(x, ldx, arm, ld_arm, layout, n_steps, seq_len, u, n_patients, n_statics, n_arms, exps,
                               n_terms, fd_kind, dt, G_out, b_out, workspace, workspace_bytes, stream, sp, coef_out,
                               mask_out, iters_out);
}

size_t insite_per_patient_workspace_bytes(int64_t n_patients) {
  if (n_patients < 0) return 0;
  return kGramWsHeader + (size_t)n_patients * 5 * sizeof(double);
}

int32_t insite_sindy_fit_per_patient_f64(const double* x, int64_t ldx, int32_t layout, int32_t n_steps,
                                         const double* u, const int8_t* arm, const int32_t* rows,
                                         int64_t n_patients, int32_t n_statics, int32_t n_arms, const int8_t* exps,
                                         int32_t n_terms, int32_t fd_kind, double dt, const double* global_coef,
                                         double threshold, double alpha, int32_t max_iter, int32_t unbias,
                                         double* coef_out, int8_t* mask_out, int32_t* iters_out, void* workspace,
                                         size_t workspace_bytes, void* stream) {
  const bool tm = layout == INSITE_LAYOUT_TIME_MAJOR;
  if (layout != INSITE_LAYOUT_PATIENT_MAJOR && !tm) return INSITE_E_INVALID_ARG;
  if (n_patients < 0 || n_arms < 1 || n_arms > INSITE_MAX_ARMS || ldx < 1 || !(dt > 0.0) || n_steps < 0 ||
      (tm ? ldx < n_patients : ldx < n_steps) || max_iter < 0 || !(threshold >= 0.0) || !(alpha >= 0.0))
    return INSITE_E_INVALID_ARG;
  if (n_patients == 0) return INSITE_OK;
  if (!x || !arm || !rows || !global_coef || !coef_out || (n_statics > 0 && !u)) return INSITE_E_INVALID_ARG;
  if (fd_kind != INSITE_FD_SMOOTHED4 && fd_kind != INSITE_FD_ORDER4) return INSITE_E_UNSUPPORTED;
  if (tm && ldx > ((int64_t)1 << 31) / (8 * kGT)) return INSITE_E_UNSUPPORTED;
  LibDesc lib;
  int32_t st = build_lib(exps, n_terms, n_statics, &lib);
  if (st != INSITE_OK) return st;
  if (!workspace || workspace_bytes < insite_per_patient_workspace_bytes(n_patients)) return INSITE_E_WORKSPACE;
  hipStream_t hs = reinterpret_cast<hipStream_t>(stream);
  unsigned* ticket = static_cast<unsigned*>(workspace);
  double* mom = reinterpret_cast<double*>(static_cast<char*>(workspace) + kGramWsHeader);
  const bool vec2 = (ldx % 2 == 0) && ((reinterpret_cast<uintptr_t>(x) & 15u) == 0);
  const int mode = tm ? 2 : (vec2 ? 1 : 0);
  if (n_statics == 0) u = x;
  lib.mfma = 0;
  const GramLaunch g{x, ldx, n_steps, u, arm, rows, n_patients, make_gram_w(dt), lib, mom, ticket,
                     GramOut{nullptr, nullptr, 0}};
  if (fd_kind == INSITE_FD_SMOOTHED4) launch_moments<true>(mode, hs, g);
  else launch_moments<false>(mode, hs, g);
  st = launch_status();
  if (st != INSITE_OK) return st;
  return launch_patient_fit(mom, u, arm, rows, n_patients, n_steps, n_arms, lib, global_coef,
                            StlsqParams{threshold, alpha, max_iter, unbias, 1}, coef_out, mask_out, iters_out, hs);
}

int32_t insite_stlsq_f64(const double* G, const double* b, int64_t n_sys, int32_t n_terms,
                         double threshold, double alpha, int32_t max_iter, int32_t unbias,
                         double* coef_out, int8_t* mask_out, int32_t* iters_out, void* stream) {
  if (n_sys < 0 || max_iter < 0 || !(threshold >= 0.0) || !(alpha >= 0.0)) return INSITE_E_INVALID_ARG;
  if (n_sys == 0) return INSITE_OK;
  if (!G || !b || !coef_out) return INSITE_E_INVALID_ARG;
  if (n_terms > INSITE_MAX_TERMS)  // F <= 64: one wavefront per system (insite_gen.hip)
    return insite_stlsq_wave64_f64(G, b, n_sys, n_terms, threshold, alpha, max_iter, unbias, coef_out, mask_out,
                                   iters_out, stream);
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
                           double drop_below, double* y_out, int64_t ld_y, int32_t layout, void* stream) {
  const bool bits = layout == INSITE_LAYOUT_TIME_MAJOR_BITS;
  const bool tm = layout == INSITE_LAYOUT_TIME_MAJOR || bits;
  if (layout != INSITE_LAYOUT_PATIENT_MAJOR && !tm) return INSITE_E_INVALID_ARG;
  const int64_t minld = tm ? n_rows : (int64_t)T;
  const int64_t minld_arm = bits ? (n_rows + 31) / 32 : minld;
  // bits: ld_arm < 0 is the tile-major bit layout [ceil(n_rows / 64)][-ld_arm >= T][2] (rollout_bits_range)
  const bool tiles = bits && ld_arm < 0;
  if (n_rows < 0 || T < 0 || n_arms < 1 || n_arms > INSITE_MAX_ARMS || substeps < 1 ||
      !(dt >= 0.0) || (tiles ? -ld_arm < (int64_t)T : ld_arm < minld_arm) || ld_y < minld || coef_row_stride < 0 ||
      (bits && n_arms > 2))
    return INSITE_E_INVALID_ARG;
  if (method != INSITE_METHOD_EULER && method != INSITE_METHOD_RK4) return INSITE_E_UNSUPPORTED;
  if (n_rows == 0 || T == 0) return INSITE_OK;
  if (!y0 || !arm || !coef || !y_out || (n_statics > 0 && !u)) return INSITE_E_INVALID_ARG;
  if (coef_row_stride != 0 && coef_row_stride < (int64_t)n_arms * n_terms) return INSITE_E_INVALID_ARG;
  if (exps && n_terms > 0 && n_statics >= 0) {  // state degree > 1: the stage-evaluated polynomial rollout
    int deg = 0;
    for (int j = 0; j < n_terms; ++j) deg = exps[j * (1 + n_statics)] > deg ? exps[j * (1 + n_statics)] : deg;
    if (deg > INSITE_MAX_STATE_DEGREE) {
      if (bits) return INSITE_E_UNSUPPORTED;
      return insite_rollout_poly_f64(y0, u, arm, ld_arm, coef, coef_row_stride, exps, n_terms, n_rows, T, n_statics,
                                     n_arms, dt, method, substeps, drop_below, y_out, ld_y, layout, stream);
    }
  }
  LibDesc lib;
  int32_t st = build_lib(exps, n_terms, n_statics, &lib);
  if (st != INSITE_OK) return st;
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
  hipStream_t hs = reinterpret_cast<hipStream_t>(stream);
  const bool perrow = coef_row_stride != 0;
  const int na = narm_pad(n_arms);
  if (tm) {
    if ((tiles ? (int64_t)8 : bits ? ld_arm * 4 : ld_arm) > kTmMaxLd || ld_y > kTmMaxLd)
      return INSITE_E_UNSUPPORTED;  // 32-bit offsets per step group
    if (n_statics == 0) ra.u = y0;
    if (bits && (reinterpret_cast<uintptr_t>(arm) & 3u) != 0) return INSITE_E_INVALID_ARG;
    const bool aw4 = bits || (ld_arm % 4 == 0 && (reinterpret_cast<uintptr_t>(arm) & 3u) == 0);
    const bool y16 = ld_y % 2 == 0 && (reinterpret_cast<uintptr_t>(y_out) & 15u) == 0;
    const int afmt = bits ? kArmBits : (aw4 ? kArmDword : kArmByte);
    int ppl = 1;  // patients per lane: more independent chains per lane for big cohorts
#ifdef INSITE_FORCE_PPL
    ppl = INSITE_FORCE_PPL;
#else
    // one patient per lane: with the interval propagator the time loop is store-bound, more chains per
    // lane buy nothing; since the prologue loads its coefficient row in one burst (affine_rates), two
    // patients per lane (16-B stores) is slower too: F4's 1M x 60 4-arm int8 rollout 0.117 ms at PPL 2,
    // 0.094 ms at PPL 1, 0.168 ms at PPL 4 (profiles/r02/ppl/); INSITE_FORCE_PPL keeps the others
#endif
    if (ppl >= 2 && !(y16 && aw4 && n_rows % ppl == 0)) ppl = 1;
    if (tiles) ppl = 1;  // (the tile-major bits are read by rollout_bits_range, the one-patient-per-lane form)
    const int64_t per_block = (int64_t)kBlock * ppl;
    const dim3 grid((unsigned)((n_rows + per_block - 1) / per_block));
    if (method == INSITE_METHOD_EULER) launch_rollout_tm_m<INSITE_METHOD_EULER>(na, perrow, ppl, afmt, grid, hs, ra, lib);
    else launch_rollout_tm_m<INSITE_METHOD_RK4>(na, perrow, ppl, afmt, grid, hs, ra, lib);
    return launch_status();
  }
  if (ld_arm > (int64_t)0x1FFFFFF || ld_y > (int64_t)0x3FFFFF) return INSITE_E_UNSUPPORTED;  // 32-bit buffer offsets
  const uintptr_t ab = reinterpret_cast<uintptr_t>(arm), yb = reinterpret_cast<uintptr_t>(y_out);
  const int av = (ld_arm % 16 == 0 && (ab & 15u) == 0) ? 16 : ((ld_arm % 4 == 0 && (ab & 3u) == 0) ? 4 : 1);
  const bool yv2 = (ld_y % 2 == 0) && (T % 2 == 0) && ((yb & 15u) == 0);
  if (n_statics == 0) ra.u = y0;  // loaded unconditionally, unused when U = 0
  const int64_t waves = (n_rows + kWave - 1) / kWave;
  const dim3 grid((unsigned)((waves + kWavesPerBlock - 1) / kWavesPerBlock));
  if (method == INSITE_METHOD_EULER) launch_rollout_m<INSITE_METHOD_EULER>(na, perrow, av, yv2, grid, hs, ra, lib);
  else launch_rollout_m<INSITE_METHOD_RK4>(na, perrow, av, yv2, grid, hs, ra, lib);
  return launch_status();
}

extern "C++" {
namespace {
template <bool PM>
void launch_rk45_flat(int32_t n_arms, bool perrow, dim3 grid, hipStream_t hs, const Rk45Args& ra, const LibDesc& lib) {
  if (n_arms == 1) {
    if (perrow) rollout_rk45_flat_kernel<1, true, PM><<<grid, kBlock, 0, hs>>>(ra, lib);
    else rollout_rk45_flat_kernel<1, false, PM><<<grid, kBlock, 0, hs>>>(ra, lib);
  } else {
    if (perrow) rollout_rk45_flat_kernel<2, true, PM><<<grid, kBlock, 0, hs>>>(ra, lib);
    else rollout_rk45_flat_kernel<2, false, PM><<<grid, kBlock, 0, hs>>>(ra, lib);
  }
}
}  // namespace
}  // extern "C++"

int32_t insite_rollout_rk45_f64(const double* y0, const double* u, const uint32_t* arm_bits, int64_t ld_arm,
                                const double* t_obs, int64_t ld_t, const int32_t* n_obs, const double* coef,
                                int64_t coef_row_stride, const int8_t* exps, int32_t n_terms, int64_t n_rows,
                                int32_t T_max, int32_t n_statics, int32_t n_arms, double rtol, double atol,
                                double drop_below, double* y_out, int64_t ld_y, int32_t* steps_out,
                                const int32_t* row_order, int32_t layout, void* stream) {
  const bool pm = layout == INSITE_LAYOUT_PATIENT_MAJOR_BITS;
  if (!pm && layout != INSITE_LAYOUT_TIME_MAJOR_BITS) return INSITE_E_INVALID_ARG;
  const int64_t words = pm ? ((int64_t)T_max - 1 + 31) / 32 : (n_rows + 31) / 32;
  if (n_rows < 0 || T_max < 1 || n_arms < 1 || n_arms > 2 || !(rtol > 0.0) || !(atol > 0.0) ||
      ld_t < (pm ? T_max : n_rows) || ld_y < (pm ? T_max : n_rows) || ld_arm < (words > 0 ? words : 1) ||
      coef_row_stride < 0)
    return INSITE_E_INVALID_ARG;
  if (n_rows == 0) return INSITE_OK;
  if (!y0 || !arm_bits || !t_obs || !n_obs || !coef || !y_out || (n_statics > 0 && !u)) return INSITE_E_INVALID_ARG;
  LibDesc lib;
  int32_t st = build_lib(exps, n_terms, n_statics, &lib);
  if (st != INSITE_OK) return st;
  if (coef_row_stride != 0 && coef_row_stride < (int64_t)n_arms * n_terms) return INSITE_E_INVALID_ARG;
  Rk45Args ra{y0, n_statics > 0 ? u : y0, arm_bits, t_obs, n_obs, coef, y_out, steps_out, row_order, ld_arm, ld_t, ld_y,
              coef_row_stride, n_rows, T_max, n_arms, rtol, atol, drop_below,
              (pm && n_rows * ld_y * 8 < ((int64_t)1 << 31) - 64) ? 1 : 0};
  const int64_t waves = (n_rows + kWave - 1) / kWave;
  const dim3 grid((unsigned)((waves + kWavesPerBlock - 1) / kWavesPerBlock));
  hipStream_t hs = reinterpret_cast<hipStream_t>(stream);
  const bool perrow = coef_row_stride != 0;
#ifdef INSITE_RK45_PER_INTERVAL  // the per-interval form (A/B builds, tools/build_ablation.sh): time-major only
  if (pm) return INSITE_E_UNSUPPORTED;
  if (n_arms == 1) {
    if (perrow) rollout_rk45_kernel<1, true><<<grid, kBlock, 0, hs>>>(ra, lib);
    else rollout_rk45_kernel<1, false><<<grid, kBlock, 0, hs>>>(ra, lib);
  } else {
    if (perrow) rollout_rk45_kernel<2, true><<<grid, kBlock, 0, hs>>>(ra, lib);
    else rollout_rk45_kernel<2, false><<<grid, kBlock, 0, hs>>>(ra, lib);
  }
#else
  if (pm) launch_rk45_flat<true>(n_arms, perrow, grid, hs, ra, lib);
  else launch_rk45_flat<false>(n_arms, perrow, grid, hs, ra, lib);
#endif
  return launch_status();
}

size_t insite_rk45_order_workspace_bytes(int32_t T_max) {
  const int nb = (T_max < kRkBinMax - 1 ? (T_max < 1 ? 1 : T_max) : kRkBinMax - 1) + 1;
  return (size_t)(2 * nb + 1) * sizeof(unsigned);  // totals, cursors, the self-reset ticket
}

int32_t insite_rk45_order_i32(const int32_t* n_obs, int64_t n_rows, int32_t T_max, int32_t* order_out, void* workspace,
                              size_t workspace_bytes, void* stream) {
  if (n_rows < 0 || n_rows > INT32_MAX || T_max < 1) return INSITE_E_INVALID_ARG;
  if (n_rows == 0) return INSITE_OK;
  if (!n_obs || !order_out || !workspace) return INSITE_E_INVALID_ARG;
  if (workspace_bytes < insite_rk45_order_workspace_bytes(T_max)) return INSITE_E_WORKSPACE;
  const int nb = (T_max < kRkBinMax - 1 ? T_max : kRkBinMax - 1) + 1;
  unsigned* hist = static_cast<unsigned*>(workspace);
  hipStream_t hs = reinterpret_cast<hipStream_t>(stream);
  if (!INSITE_RK45_ORDER_SELFRESET && hipMemsetAsync(hist, 0, (size_t)2 * nb * sizeof(unsigned), hs) != hipSuccess)
    return INSITE_E_HIP;
  const dim3 grid((unsigned)((n_rows + kRkBinChunk - 1) / kRkBinChunk));
  rk45_bin_count_kernel<<<grid, kBlock, 0, hs>>>(n_obs, n_rows, nb, hist);
  rk45_bin_scatter_kernel<<<grid, kBlock, 0, hs>>>(n_obs, n_rows, nb, hist, hist + nb, order_out);
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
