// Mixed read+write HBM ceiling probe (tooling, not product).  The C2 step reads x (162 MB) and writes y
// (165 MB) in one launch; this measures what the chip sustains for that mix:
//   copy   : every wave reads 16 B/lane and writes it elsewhere (grid-stride, unrolled)
//   split  : blocks [0, R) only read (sum) one buffer, blocks [R, grid) only write another -- the fused
//            step's shape (gram role | rollout role) without compute
//   read / write : one direction alone (calibration)
// Buffers of `mb` MB each (default 2048: far past the 256 MB Infinity Cache), two sets alternated per
// launch.  Prints one JSON object: TB/s of algorithmic bytes per pattern.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__);                  \
      return 1;                                                                \
    }                                                                          \
  } while (0)

typedef double d2 __attribute__((ext_vector_type(2)));

template <int U>
__global__ void __launch_bounds__(256) copy_k(const d2* __restrict__ a, d2* __restrict__ b, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    d2 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = a[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) b[i + u * stride] = v[u];
  }
  for (; i < n; i += stride) b[i] = a[i];
}

template <int U>
__device__ void read_part(const d2* __restrict__ a, int64_t n, int64_t tid, int64_t stride, double* sink) {
  d2 s = {0.0, 0.0};
  int64_t i = tid;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    d2 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = a[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) s += v[u];
  }
  for (; i < n; i += stride) s += a[i];
  if (s.x == 1234.5) sink[0] = s.y;
}

template <int U>
__device__ void write_part(d2* __restrict__ b, int64_t n, int64_t tid, int64_t stride) {
  const d2 v = {1.0, 2.0};
  int64_t i = tid;
  for (; i + (U - 1) * stride < n; i += U * stride) {
#pragma unroll
    for (int u = 0; u < U; ++u) b[i + u * stride] = v;
  }
  for (; i < n; i += stride) b[i] = v;
}

template <int U>
__global__ void __launch_bounds__(256) split_k(const d2* __restrict__ a, d2* __restrict__ b, int64_t n, int rblocks,
                                               double* sink) {
  if ((int)blockIdx.x < rblocks) {
    read_part<U>(a, n, (int64_t)blockIdx.x * blockDim.x + threadIdx.x, (int64_t)rblocks * blockDim.x, sink);
  } else {
    const int wb = (int)gridDim.x - rblocks;
    write_part<U>(b, n, (int64_t)((int)blockIdx.x - rblocks) * blockDim.x + threadIdx.x, (int64_t)wb * blockDim.x);
  }
}

template <int U>
__global__ void __launch_bounds__(256) read_k(const d2* __restrict__ a, int64_t n, double* sink) {
  read_part<U>(a, n, (int64_t)blockIdx.x * blockDim.x + threadIdx.x, (int64_t)gridDim.x * blockDim.x, sink);
}

template <int U>
__global__ void __launch_bounds__(256) write_k(d2* __restrict__ b, int64_t n) {
  write_part<U>(b, n, (int64_t)blockIdx.x * blockDim.x + threadIdx.x, (int64_t)gridDim.x * blockDim.x);
}

int main(int argc, char** argv) {
  const int64_t mb = argc > 1 ? atoll(argv[1]) : 2048;
  const int iters = 10;
  const int64_t n = mb * 1000000 / 16;  // d2 elements per buffer
  d2 *a[2], *b[2];
  double* sink;
  for (int s = 0; s < 2; ++s) {
    CK(hipMalloc(&a[s], n * 16));
    CK(hipMalloc(&b[s], n * 16));
    CK(hipMemset(a[s], 0, n * 16));
    CK(hipMemset(b[s], 0, n * 16));
  }
  CK(hipMalloc(&sink, 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timed = [&](auto launch) -> double {
    for (int w = 0; w < 2; ++w) launch(w & 1);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, 0));
    for (int it = 0; it < iters; ++it) launch(it & 1);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / iters;
  };
  printf("{\"buffer_MB\": %lld", (long long)mb);
  for (int grid : {1024, 2048, 4096}) {
    double ms = timed([&](int s) { copy_k<4><<<grid, 256>>>(a[s], b[s], n); });
    printf(", \"copy_g%d_TBps\": %.3f", grid, 2.0 * n * 16 / (ms * 1e-3) / 1e12);
  }
  {
    double ms = timed([&](int s) { read_k<4><<<2048, 256>>>(a[s], n, sink); });
    printf(", \"read_TBps\": %.3f", n * 16 / (ms * 1e-3) / 1e12);
    ms = timed([&](int s) { write_k<4><<<2048, 256>>>(b[s], n); });
    printf(", \"write_TBps\": %.3f", n * 16 / (ms * 1e-3) / 1e12);
  }
  for (int rb : {256, 307, 341, 384}) {
    double ms = timed([&](int s) { split_k<4><<<512, 256>>>(a[s], b[s], n, rb, sink); });
    printf(", \"split512_r%d_TBps\": %.3f", rb, 2.0 * n * 16 / (ms * 1e-3) / 1e12);
  }
  for (int rb : {512, 1024}) {
    double ms = timed([&](int s) { split_k<4><<<2048, 256>>>(a[s], b[s], n, rb, sink); });
    printf(", \"split2048_r%d_TBps\": %.3f", rb, 2.0 * n * 16 / (ms * 1e-3) / 1e12);
  }
  printf("}\n");
  return 0;
}
