// Operand/result lane layout of v_mfma_f64_4x4x4f64 on gfx950 (tools/probe; not product code).
// For every (lane_a, lane_b) pair: A = e_{lane_a}, B = e_{lane_b}; print the result lanes that become 1.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void probe(double* out) {
  const int la = blockIdx.x >> 6, lb = blockIdx.x & 63, lane = threadIdx.x;
  const double a = lane == la ? 1.0 : 0.0, b = lane == lb ? 1.0 : 0.0;
  double c = 0.0;
  c = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
  out[blockIdx.x * 64 + lane] = c;
}

int main() {
  double* d;
  if (hipMalloc(&d, 4096 * 64 * sizeof(double)) != hipSuccess) return 1;
  probe<<<4096, 64>>>(d);
  std::vector<double> h(4096 * 64);
  if (hipMemcpy(h.data(), d, h.size() * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) return 1;
  for (int la = 0; la < 64; ++la)
    for (int lb = 0; lb < 64; ++lb)
      for (int l = 0; l < 64; ++l) {
        const double v = h[(la * 64 + lb) * 64 + l];
        if (v != 0.0) printf("a%d b%d -> d%d (%g)\n", la, lb, l, v);
      }
  hipFree(d);
  return 0;
}
