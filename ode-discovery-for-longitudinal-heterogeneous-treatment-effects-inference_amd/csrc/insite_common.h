// insite_common.h — device helpers shared by the INSITE HIP translation units (insite_hip.hip: one-state
// PK/PD path; insite_ms.hip: multi-state path).  Everything lives in an anonymous namespace: each
// translation unit gets its own internal copy.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "insite_hip.h"

namespace {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWave * kWavesPerBlock;

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

// Butterfly reductions over a full wave; every lane holds the result, returned through
// readfirstlane so the compiler treats it as wave-uniform (SGPR: scalar branches, uniform
// buffer descriptors without waterfall loops).
__device__ __forceinline__ int wave_min_i(int v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = min(v, __shfl_xor(v, off, kWave));
  return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = max(v, __shfl_xor(v, off, kWave));
  return __builtin_amdgcn_readfirstlane(v);
}

// 32x32 bit transpose across each half-wave: lane j holds row j (bit i = column i); afterwards
// lane i holds column i (bit j = row j).  Five butterfly stages (ds_swizzle/bpermute).
__device__ __forceinline__ unsigned bit_transpose32(unsigned x, int lane) {
  const unsigned m[5] = {0x0000FFFFu, 0x00FF00FFu, 0x0F0F0F0Fu, 0x33333333u, 0x55555555u};
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const int sh = 16 >> k;
    const unsigned y = (unsigned)__shfl_xor((int)x, sh, kWave);
    x = (lane & sh) ? ((x & ~m[k]) | ((y >> sh) & m[k])) : ((x & m[k]) | ((y << sh) & ~m[k]));
  }
  return x;
}

// Streaming weights; 1/dt folded into the finite-difference weights.
struct GramW {
  double sg0, sg1, sg2;  // savgol interior: sg0*x[k] + sg1*(x[k-1]+x[k+1]) + sg2*(x[k-2]+x[k+2])
  double fd1, fd2;       // FD4 interior:   fd1*(v[k+1]-v[k-1]) + fd2*(v[k+2]-v[k-2])
  double inv_dt;
};

__device__ __forceinline__ double sg_int(const GramW& w, double a, double b, double c, double d, double e) {
  return w.sg0 * c + w.sg1 * (b + d) + w.sg2 * (a + e);
}
__device__ __forceinline__ double fd_int(const GramW& w, double a, double b, double d, double e) {
  return w.fd1 * (d - b) + w.fd2 * (e - a);
}

typedef double dbl4 __attribute__((ext_vector_type(4)));
constexpr unsigned kOOB = 0x80000000u;  // buffer offset beyond every descriptor: access dropped

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

struct StlsqParams {
  double thr, alpha;
  int32_t max_iter, unbias, enabled;
};


#ifndef INSITE_STORE_AUX
#define INSITE_STORE_AUX 2
#endif
// Cache policy of the trajectory stores: non-temporal (aux bit 1).  Trajectories are written once
// and read by a later consumer; kept out of the Infinity Cache they do not leave ~160 MB of dirty
// lines that the next discovery pass would have to write back while it streams its own input
// (C2 step: 87.5 -> 76 us measured, tools/build_ablation.sh NT).
constexpr int kStoreAux = INSITE_STORE_AUX;

inline int32_t launch_status() { return hipGetLastError() == hipSuccess ? INSITE_OK : INSITE_E_HIP; }

}  // namespace
