// Throughput of the two f64 MFMA shapes on gfx950 (one wave per SIMD, 4 independent accumulators):
// cycles per instruction from clock64 around 4096 back-to-back MFMAs.  Build:
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/mfma_rate tools/probe/mfma_f64_rate_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double dbl4 __attribute__((ext_vector_type(4)));

__global__ void k16(double* out, double a, double b, long long* cyc) {
  dbl4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  double x = a + threadIdx.x, y = b - threadIdx.x;
  __syncthreads();
  const long long t0 = clock64();
  for (int i = 0; i < 1024; ++i) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(y, x, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(y, y, c3, 0, 0, 0);
  }
  const long long t1 = clock64();
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

__global__ void k4(double* out, double a, double b, long long* cyc) {
  double c0 = 0, c1 = 0, c2 = 0, c3 = 0;
  double x = a + threadIdx.x, y = b - threadIdx.x;
  __syncthreads();
  const long long t0 = clock64();
  for (int i = 0; i < 1024; ++i) {
    c0 = __builtin_amdgcn_mfma_f64_4x4x4f64(x, y, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_4x4x4f64(y, x, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_4x4x4f64(x, x, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_4x4x4f64(y, y, c3, 0, 0, 0);
  }
  const long long t1 = clock64();
  out[blockIdx.x * blockDim.x + threadIdx.x] = c0 + c1 + c2 + c3;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  double* out;
  long long* cyc;
  hipMalloc(&out, 64 * 8 * sizeof(double));
  hipMalloc(&cyc, 8 * sizeof(long long));
  long long h[8];
  for (int rep = 0; rep < 2; ++rep) {
    k16<<<1, 64>>>(out, 1.0, 2.0, cyc);
    hipMemcpy(h, cyc, 8, hipMemcpyDeviceToHost);
    if (rep) printf("16x16x4f64: %.2f cycles/MFMA (clock64 units)\n", h[0] / 4096.0);
    k4<<<1, 64>>>(out, 1.0, 2.0, cyc);
    hipMemcpy(h, cyc, 8, hipMemcpyDeviceToHost);
    if (rep) printf("4x4x4f64:   %.2f cycles/MFMA (clock64 units)\n", h[0] / 4096.0);
  }
  // 4 waves on one CU (one per SIMD) to see per-SIMD independence
  k16<<<1, 256>>>(out, 1.0, 2.0, cyc);
  hipMemcpy(h, cyc, 8, hipMemcpyDeviceToHost);
  printf("16x16x4f64 (4 waves/block): %.2f\n", h[0] / 4096.0);
  return 0;
}
