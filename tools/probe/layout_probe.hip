// HBM access-pattern probe (tooling, not product): one wave streams 64 patients x T steps either
// time-major (512-B chunks, row stride N*8 B) or 64-patient tiled (its own contiguous 64*T*8 B).
// Read (sum) and write variants; T steps, N patients; prints GB/s per pattern.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int MODE, int PF>  // MODE 0: time-major, 1: tiled
__global__ void __launch_bounds__(256) rd(const double* __restrict__ x, int64_t N, int T, double* out) {
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t p0 = w * 64;
  if (p0 >= N) return;
  const double* base = MODE == 0 ? x + p0 + lane : x + p0 * T + lane;
  const int64_t rs = MODE == 0 ? N : 64;
  double s = 0.0, v[PF];
  for (int k = 0; k < T; k += PF) {
#pragma unroll
    for (int i = 0; i < PF; ++i) v[i] = __builtin_nontemporal_load(base + (int64_t)(k + i < T ? k + i : T - 1) * rs);
#pragma unroll
    for (int i = 0; i < PF; ++i) s += v[i];
  }
  if (s == 1234.5) out[0] = s;
}

template <int MODE>
__global__ void __launch_bounds__(256) wr(double* __restrict__ y, int64_t N, int T) {
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t p0 = w * 64;
  if (p0 >= N) return;
  double* base = MODE == 0 ? y + p0 + lane : y + p0 * T + lane;
  const int64_t rs = MODE == 0 ? N : 64;
  double v = (double)lane;
  for (int k = 0; k < T; ++k) {
    v = v * 1.0000001 + 1.0;
    base[(int64_t)k * rs] = v;
  }
}

int main(int argc, char** argv) {
  int64_t N = argc > 1 ? atoll(argv[1]) : 100000;
  int T = argc > 2 ? atoi(argv[2]) : 200;
  N = (N + 63) / 64 * 64;
  double *x, *y, *o, *fl;
  size_t bytes = (size_t)N * T * 8;
  CK(hipMalloc(&x, bytes)); CK(hipMalloc(&y, bytes)); CK(hipMalloc(&o, 64)); CK(hipMalloc(&fl, (size_t)512 << 20));
  CK(hipMemset(x, 0, bytes));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  const int grid = (int)((N / 64 + 3) / 4);
  auto run = [&](const char* name, auto fn) {
    float tot = 0; int it = 20;
    if (hipDeviceSynchronize() != hipSuccess) { printf("sync failed before %s\n", name); exit(1); }
    for (int i = 0; i < it + 2; ++i) {
      hipMemsetAsync(fl, i, (size_t)512 << 20);  // evict
      hipMemsetAsync(o, 0, 8);
      hipEventRecord(a); fn(); hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b); if (i >= 2) tot += ms;
    }
    printf("%-28s N=%ld T=%d  %.2f us  %.0f GB/s\n", name, (long)N, T, tot / it * 1e3, bytes / (tot / it * 1e-3) / 1e9);
  };
  run("read time-major PF16", [&] { rd<0, 16><<<grid, 256>>>(x, N, T, o); });
  run("read tiled PF16", [&] { rd<1, 16><<<grid, 256>>>(x, N, T, o); });
  run("read time-major PF8", [&] { rd<0, 8><<<grid, 256>>>(x, N, T, o); });
  run("read tiled PF8", [&] { rd<1, 8><<<grid, 256>>>(x, N, T, o); });
  run("write time-major", [&] { wr<0><<<grid, 256>>>(y, N, T); });
  run("write tiled", [&] { wr<1><<<grid, 256>>>(y, N, T); });
  CK(hipDeviceSynchronize());
  CK(hipGetLastError());
  return 0;
}
