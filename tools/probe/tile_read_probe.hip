// Read-side HBM probe for the C2 gram's access pattern (tooling, not product).  x is time-major [T, ld] f64
// (T = 200, N = ld = 100k: 160 MB); two copies are alternated per launch so nothing is served from the
// 256 MB Infinity Cache.  Patterns (every one reads every byte once, sums it, and prints TB/s):
//   linear      : grid-stride 16-B loads over the flat buffer (calibration)
//   tile<GT,D>  : the gram's shape -- a wave owns a 64-patient tile (lane = patient), walks the steps in
//                 tiles of GT steps (GT buffer loads of 512 B, one per step row), D tiles in flight;
//                 work items = (tile, time segment), `order` 0: tile-major (item / nseg = tile, as
//                 gram_body), 1: segment-major (item % ntiles = tile: concurrent waves read adjacent
//                 columns of the same steps); grid = `waves` waves in blocks of 4
// Prints one JSON object.
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

typedef double d2 __attribute__((ext_vector_type(2)));

__global__ void __launch_bounds__(256) linear_k(const d2* __restrict__ a, int64_t n, double* sink) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  d2 s = {0.0, 0.0};
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    d2 v0 = a[i], v1 = a[i + stride], v2 = a[i + 2 * stride], v3 = a[i + 3 * stride];
    s += v0 + v1 + v2 + v3;
  }
  for (; i < n; i += stride) s += a[i];
  if (s.x == 1234.5) sink[0] = s.y;
}

template <int GT, int D>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
tile_k(const double* __restrict__ x, int64_t ld, int T, int64_t N, int nseg, int order, double* sink) {
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t ntiles = (N + 63) / 64;
  const int64_t nitems = ntiles * nseg;
  const int seg = (T + nseg - 1) / nseg;
  double s = 0.0;
  const int64_t W = (int64_t)gridDim.x * 4;
  for (int64_t item = (int64_t)blockIdx.x * 4 + wid; item < nitems; item += W) {
    const int64_t tile = order == 0 ? item / nseg : item % ntiles;
    const int sidx = order == 0 ? (int)(item - tile * nseg) : (int)(item / ntiles);
    const int t0 = sidx * seg, t1 = min(t0 + seg, T);
    const int64_t p0 = tile * 64;
    const int valid = (int)(N - p0 < 64 ? N - p0 : 64);
    const unsigned off = lane < valid ? (unsigned)lane * 8u : 0x80000000u;
    double v[D][GT];
    auto ld_tile = [&](double (&r)[GT], int ta) {
      const int nrow = t1 - ta < GT ? t1 - ta : GT;
      const int bytes = nrow > 0 ? (int)(((int64_t)(nrow - 1) * ld + valid) * 8) : 0;
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc((void*)(x + (int64_t)(nrow > 0 ? ta : 0) * ld + p0), (short)0, bytes, 0x00020000);
#pragma unroll
      for (int i = 0; i < GT; ++i)
        r[i] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, off + (unsigned)(i * ld * 8), 0, 0));
    };
#pragma unroll
    for (int d = 0; d < D; ++d)
      if (t0 + d * GT < t1) ld_tile(v[d], t0 + d * GT);
    for (int ta = t0; ta < t1;) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        if (ta < t1) {
#pragma unroll
          for (int i = 0; i < GT; ++i) s += v[d][i];
          if (ta + D * GT < t1) ld_tile(v[d], ta + D * GT);
          ta += GT;
        }
      }
    }
  }
  if (s == 1234.5) sink[0] = s;
}

int main(int argc, char** argv) {
  const int T = 200;
  const int64_t N = argc > 1 ? atoll(argv[1]) : 100000, ld = N;
  const int iters = 20;
  const int64_t n = T * ld;
  double *a[2], *sink;
  for (int s = 0; s < 2; ++s) {
    CK(hipMalloc(&a[s], n * 8));
    CK(hipMemset(a[s], 0, n * 8));
  }
  CK(hipMalloc(&sink, 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timed = [&](auto launch) -> double {
    for (int w = 0; w < 4; ++w) launch(w & 1);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int it = 0; it < iters; ++it) launch(it & 1);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / iters;
  };
  const double bytes = (double)n * 8;
  printf("{\"MB\": %.0f", bytes / 1e6);
  for (int grid : {1024, 2048}) {
    double ms = timed([&](int s) { linear_k<<<grid, 256>>>((const d2*)a[s], n / 2, sink); });
    printf(", \"linear_g%d\": [%.4f, %.3f]", grid, ms, bytes / (ms * 1e-3) / 1e12);
  }
#define RUN(GT, D)                                                                                             \
  for (int waves : {1024, 1228, 2048, 4096})                                                                   \
    for (int nseg : {1, 2, 4})                                                                                 \
      for (int order : {0, 1}) {                                                                               \
        if (nseg == 1 && order == 1) continue;                                                                 \
        double ms = timed([&](int s) { tile_k<GT, D><<<waves / 4, 256>>>(a[s], ld, T, N, nseg, order, sink); }); \
        printf(", \"tile%d_d%d_w%d_s%d_o%d\": [%.4f, %.3f]", GT, D, waves, nseg, order, ms,                    \
               bytes / (ms * 1e-3) / 1e12);                                                                    \
      }
  RUN(16, 2)
  RUN(8, 4)
  RUN(16, 3)
  RUN(8, 2)
  printf("}\n");
  return 0;
}
