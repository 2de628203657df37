// Does f64 MFMA work overlap with VALU work on gfx950?  Cycles (clock64) for loops of
//   A: 8 independent v_mfma_f64_4x4x4f64 per iteration
//   B: 16 independent v_fma_f64 per iteration          (f64 VALU)
//   C: 16 independent v_fma_f32 per iteration          (f32 VALU)
//   D: 16 v_cvt_f64_f32 per iteration
//   and A interleaved with B / C / D inside one wave, and A-only waves beside B-only waves on one SIMD
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/ovl tools/probe/mfma_valu_overlap_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int kIter = 2048;

template <int MODE>
__device__ __forceinline__ void body(double (&c)[8], double (&d)[16], float (&f)[16], double x, double y,
                                     float fx) {
  if (MODE & 1) {
#pragma unroll
    for (int q = 0; q < 8; ++q) c[q] = __builtin_amdgcn_mfma_f64_4x4x4f64(x, y, c[q], 0, 0, 0);
  }
  if (MODE & 2) {
#pragma unroll
    for (int q = 0; q < 16; ++q) d[q] = __builtin_fma(d[q], x, y);
  }
  if (MODE & 4) {
#pragma unroll
    for (int q = 0; q < 16; ++q) f[q] = __builtin_fmaf(f[q], fx, fx);
  }
  if (MODE & 8) {
#pragma unroll
    for (int q = 0; q < 16; ++q) d[q] += (double)f[q];
  }
}

// role per wave: waves with (wave >= split) run MODE_B, others MODE_A
template <int MODE_A, int MODE_B>
__global__ void probe(double* out, double a, double b, long long* cyc, int split) {
  double c[8], d[16];
  float f[16];
  const int w = threadIdx.x / 64;
#pragma unroll
  for (int q = 0; q < 8; ++q) c[q] = q;
#pragma unroll
  for (int q = 0; q < 16; ++q) { d[q] = q * 0.5; f[q] = q * 0.25f; }
  double x = a + threadIdx.x * 1e-9, y = b - threadIdx.x * 1e-9;
  float fx = (float)x;
  __syncthreads();
  const long long t0 = clock64();
  if (w < split) {
    for (int i = 0; i < kIter; ++i) body<MODE_A>(c, d, f, x, y, fx);
  } else {
    for (int i = 0; i < kIter; ++i) body<MODE_B>(c, d, f, x, y, fx);
  }
  const long long t1 = clock64();
  double s = 0;
#pragma unroll
  for (int q = 0; q < 8; ++q) s += c[q];
#pragma unroll
  for (int q = 0; q < 16; ++q) s += d[q] + f[q];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 16 + w] = t1 - t0;
}

template <int A, int B>
void run(const char* name, int threads, int split, double* out, long long* cyc) {
  long long h[16];
  for (int rep = 0; rep < 2; ++rep) {
    probe<A, B><<<1, threads>>>(out, 1.0, 2.0, cyc, split);
    hipMemcpy(h, cyc, 16 * sizeof(long long), hipMemcpyDeviceToHost);
  }
  printf("%-44s", name);
  for (int w = 0; w < threads / 64; ++w) printf(" %7.1f", h[w] / (double)kIter);
  printf("   cycles/iter per wave\n");
}

int main() {
  double* out;
  long long* cyc;
  hipMalloc(&out, 1024 * sizeof(double));
  hipMalloc(&cyc, 16 * sizeof(long long));
  // one wave per SIMD (4 waves)
  run<1, 1>("8 mfma4x4 f64 (1 wave/SIMD)", 256, 4, out, cyc);
  run<2, 2>("16 fma f64", 256, 4, out, cyc);
  run<4, 4>("16 fma f32", 256, 4, out, cyc);
  run<8, 8>("16 cvt f32->f64 + add f64", 256, 4, out, cyc);
  run<3, 3>("8 mfma + 16 fma f64 (same wave)", 256, 4, out, cyc);
  run<5, 5>("8 mfma + 16 fma f32 (same wave)", 256, 4, out, cyc);
  run<9, 9>("8 mfma + 16 cvt+add (same wave)", 256, 4, out, cyc);
  // two waves per SIMD (8 waves): waves 0-3 and 4-7 share SIMDs
  run<1, 1>("2 waves/SIMD: mfma | mfma", 512, 4, out, cyc);
  run<2, 2>("2 waves/SIMD: fma64 | fma64", 512, 4, out, cyc);
  run<1, 2>("2 waves/SIMD: mfma | fma64", 512, 4, out, cyc);
  run<1, 4>("2 waves/SIMD: mfma | fma32", 512, 4, out, cyc);
  run<1, 8>("2 waves/SIMD: mfma | cvt+add64", 512, 4, out, cyc);
  run<3, 3>("2 waves/SIMD: mfma+fma64 | mfma+fma64", 512, 4, out, cyc);
  return 0;
}
