// C2-shape HBM probe (tooling, not product): the deferred step's byte mix without its arithmetic, in the two
// layouts a 64-patient tile can have in HBM.
//   time-major : element (step s, patient p) at s * N + p          -- a tile's step is a 512-B run, row stride N * 8 B
//   tile-major : element (step s, patient p) at (p / 64) * T * 64 + s * 64 + p % 64 -- a tile's steps are contiguous
// Work units are (64-patient tile, GS-step group), tile-major; every wave takes one equal contiguous range of them
// (the step kernel's range mode). Roles as in step_deferred_kernel: blocks [0, grid/2) read (sum) x, blocks
// [grid/2, grid) write y (one FMA chain a step, the rollout's store shape); "mixed": every wave reads one unit of x and
// writes one unit of y in turn. Two cohorts alternate per launch (4 x 160 MB, past the 256 MB Infinity Cache).
// Prints one JSON object: microseconds per launch and TB/s of algorithmic bytes (x read + y written).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#define CK(x)                                                 \
  do {                                                        \
    hipError_t e = (x);                                       \
    if (e != hipSuccess) {                                    \
      printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                               \
    }                                                         \
  } while (0)

struct Shape {
  int64_t N;  // patients (a multiple of 64)
  int T, G;   // steps, groups per tile (T / GS)
};

template <bool TM>
__device__ __forceinline__ int64_t at(const Shape& s, int64_t tile, int step) {
  return TM ? (int64_t)step * s.N + tile * 64 : tile * 64 * s.T + (int64_t)step * 64;
}

template <bool TM, int GS>
__device__ void read_range(const double* __restrict__ x, Shape s, int64_t u0, int64_t u1, int lane, double* sink) {
  double acc = 0.0, cur[GS], nxt[GS];
  if (u0 >= u1) return;
  {
    const int64_t t = u0 / s.G;
    const int st = (int)(u0 % s.G) * GS;
#pragma unroll
    for (int i = 0; i < GS; ++i) cur[i] = __builtin_nontemporal_load(x + at<TM>(s, t, st + i) + lane);
  }
  for (int64_t u = u0; u < u1; ++u) {
    const int64_t un = u + 1 < u1 ? u + 1 : u;
    const int64_t t = un / s.G;
    const int st = (int)(un % s.G) * GS;
#pragma unroll
    for (int i = 0; i < GS; ++i) nxt[i] = __builtin_nontemporal_load(x + at<TM>(s, t, st + i) + lane);
#pragma unroll
    for (int i = 0; i < GS; ++i) acc = fma(acc, 0.999, cur[i]);
#pragma unroll
    for (int i = 0; i < GS; ++i) cur[i] = nxt[i];
  }
  if (acc == 1234.5) sink[0] = acc;
}

template <bool TM, int GS>
__device__ void write_range(double* __restrict__ y, Shape s, int64_t u0, int64_t u1, int lane) {
  double v = (double)lane;
  for (int64_t u = u0; u < u1; ++u) {
    const int64_t t = u / s.G;
    const int st = (int)(u % s.G) * GS;
#pragma unroll
    for (int i = 0; i < GS; ++i) {
      v = fma(v, 1.0000001, 1.0);
      __builtin_nontemporal_store(v, y + at<TM>(s, t, st + i) + lane);
    }
  }
}

template <bool TM, int GS, int ROLES = 3>  // ROLES: 1 read role only, 2 write role only, 3 both
__global__ void __launch_bounds__(256) split_k(const double* __restrict__ x, double* __restrict__ y, Shape s,
                                               double* sink) {
  const int lane = threadIdx.x & 63;
  const int half = (int)gridDim.x / 2;
  const bool rd = (int)blockIdx.x < half;
  const int64_t W = (int64_t)half * 4;
  const int64_t w = (int64_t)((int)blockIdx.x - (rd ? 0 : half)) * 4 + (threadIdx.x >> 6);
  const int64_t U = s.N / 64 * s.G;
  if (rd) {
    if (ROLES & 1) read_range<TM, GS>(x, s, w * U / W, (w + 1) * U / W, lane, sink);
  } else if (ROLES & 2) {
    write_range<TM, GS>(y, s, w * U / W, (w + 1) * U / W, lane);
  }
}

template <bool TM, int GS>
__global__ void __launch_bounds__(256) mixed_k(const double* __restrict__ x, double* __restrict__ y, Shape s,
                                               double* sink) {
  const int lane = threadIdx.x & 63;
  const int64_t W = (int64_t)gridDim.x * 4;
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t U = s.N / 64 * s.G;
  const int64_t u0 = w * U / W, u1 = (w + 1) * U / W;
  double acc = 0.0, v = (double)lane, cur[GS];
  for (int64_t u = u0; u < u1; ++u) {
    const int64_t t = u / s.G;
    const int st = (int)(u % s.G) * GS;
#pragma unroll
    for (int i = 0; i < GS; ++i) cur[i] = __builtin_nontemporal_load(x + at<TM>(s, t, st + i) + lane);
#pragma unroll
    for (int i = 0; i < GS; ++i) {
      v = fma(v, 1.0000001, 1.0);
      __builtin_nontemporal_store(v, y + at<TM>(s, t, st + i) + lane);
    }
#pragma unroll
    for (int i = 0; i < GS; ++i) acc = fma(acc, 0.999, cur[i]);
  }
  if (acc == 1234.5) sink[0] = acc;
}

int main(int argc, char** argv) {
  Shape s;
  s.N = (argc > 1 ? atoll(argv[1]) : 100032) / 64 * 64;
  s.T = argc > 2 ? atoi(argv[2]) : 200;
  const int iters = 20;
  const size_t bytes = (size_t)s.N * s.T * 8;
  double *x[2], *y[2], *sink;
  for (int c = 0; c < 2; ++c) {
    CK(hipMalloc(&x[c], bytes));
    CK(hipMalloc(&y[c], bytes));
    CK(hipMemset(x[c], 0, bytes));
    CK(hipMemset(y[c], 0, bytes));
  }
  CK(hipMalloc(&sink, 64));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  printf("{\"N\": %lld, \"T\": %d", (long long)s.N, s.T);
  auto run = [&](const char* name, int T_eff, double dirs, auto launch) -> int {
    for (int i = 0; i < 3; ++i) launch(i & 1);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; ++i) launch(i & 1);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / iters;
    printf(", \"%s_us\": %.2f, \"%s_TBps\": %.3f", name, us, name, dirs * s.N * T_eff * 8 / (us * 1e-6) / 1e12);
    fflush(stdout);
    return 0;
  };
  const int mode = argc > 3 ? atoi(argv[3]) : 0;
  for (int grid : {512, 1024}) {
    char nm[64];
#define RUN(KERN, TMV, GSV, LABEL, DIRS, ...)                                                          \
  {                                                                                                    \
    Shape ss = s;                                                                                      \
    ss.G = s.T / GSV;                                                                                  \
    snprintf(nm, sizeof nm, "%s_%s_gs%d_g%d", LABEL, TMV ? "tm" : "tile", GSV, grid);                  \
    if (run(nm, ss.G * GSV, DIRS, [&](int c) { KERN<TMV, GSV, ##__VA_ARGS__><<<grid, 256>>>(x[c], y[c], ss, sink); })) \
      return 1;                                                                                        \
  }
    if (mode == 0) {
      RUN(split_k, true, 8, "split", 2.0);
      RUN(split_k, false, 8, "split", 2.0);
      RUN(split_k, true, 20, "split", 2.0);
      RUN(split_k, false, 20, "split", 2.0);
      RUN(mixed_k, true, 8, "mixed", 2.0);
      RUN(mixed_k, false, 8, "mixed", 2.0);
    } else {
      RUN(split_k, true, 16, "split", 2.0);
      RUN(split_k, true, 25, "split", 2.0);
      RUN(split_k, true, 40, "split", 2.0);
      RUN(split_k, true, 16, "readonly", 1.0, 1);
      RUN(split_k, true, 40, "readonly", 1.0, 1);
      RUN(split_k, true, 16, "writeonly", 1.0, 2);
    }
  }
  printf("}\n");
  CK(hipGetLastError());
  return 0;
}
