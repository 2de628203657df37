// FETCH_SIZE / WRITE_SIZE calibration for C5's access shape (tooling, not product): lane = one patient-major row
// of n_p doubles (row stride ld, n_p ~ U{20..60} like the C5 grids), read as rollout_rk45_flat_kernel's window
// refills do -- 8 consecutive 8-B loads per lane per refill (one 64-B run of the lane's own row, lanes of a wave on
// 64 different rows), clamped at the row's end -- and written as its staged output sectors do (64-B runs as
// 4 x 16-B stores, the row's last partial sector element by element).  Known byte counts printed; run under
//   rocprofv3 --pmc FETCH_SIZE -- tools/probe/bin/window_probe      (and a separate pass for WRITE_SIZE)
// and divide the counter by the printed bytes: the factor for this shape (the streaming-read factor is 1/2).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void __launch_bounds__(256) win_read(const double* __restrict__ t, int64_t ld, const int* __restrict__ n,
                                                int64_t N, double* out) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= N) return;
  const int np = n[p];
  const double* row = t + p * ld;
  double s = 0.0;
  for (int r0 = 0; r0 < np; r0 += 8) {
    double v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = row[r0 + j < np ? r0 + j : np - 1];
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[j];
  }
  if (s == -1234.5) out[0] = s;
}

__global__ void __launch_bounds__(256) sector_write(double* __restrict__ y, int64_t ld, const int* __restrict__ n,
                                                    int64_t N) {
  typedef double d2 __attribute__((ext_vector_type(2)));
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (p >= N) return;
  const int np = n[p];
  double* row = y + p * ld;
  int r = 0;
  for (; r + 8 <= np; r += 8) {
#pragma unroll
    for (int j = 0; j < 8; j += 2) *reinterpret_cast<d2*>(row + r + j) = d2{(double)(r + j), (double)(r + j + 1)};
  }
  for (; r < np; ++r) row[r] = (double)r;
}

int main(int argc, char** argv) {
  const int64_t N = argc > 1 ? atoll(argv[1]) : 1000000;
  const int64_t ld = 64;  // 512-B rows (the C5 cohort's ld is T_max rounded up)
  std::vector<int> hn(N);
  uint32_t s = 12345u;
  int64_t elems = 0;
  for (int64_t i = 0; i < N; ++i) {
    s = s * 1664525u + 1013904223u;
    hn[i] = 20 + (int)((s >> 8) % 41);
    elems += hn[i];
  }
  double *t, *y, *o;
  int* n;
  CK(hipMalloc(&t, (size_t)N * ld * 8));
  CK(hipMalloc(&y, (size_t)N * ld * 8));
  CK(hipMalloc(&o, 64));
  CK(hipMalloc(&n, (size_t)N * 4));
  CK(hipMemset(t, 0, (size_t)N * ld * 8));
  CK(hipMemcpy(n, hn.data(), (size_t)N * 4, hipMemcpyHostToDevice));
  const int grid = (int)((N + 255) / 256);
  for (int it = 0; it < 3; ++it) {
    win_read<<<grid, 256>>>(t, ld, n, N, o);
    sector_write<<<grid, 256>>>(y, ld, n, N);
  }
  CK(hipDeviceSynchronize());
  CK(hipGetLastError());
  printf("rows %ld  elements %ld  row-data bytes %ld (read by win_read, written by sector_write, per dispatch)\n",
         (long)N, (long)elems, (long)(elems * 8));
  return 0;
}
