// insite_rng.hip — counter-based random bits for the on-device cohort generator.
//
// The reference draws every PK/PD cohort with jax.random (PRNGKey(seed) per subset,
// libs_m/ct/src/data/pkpd/dataset.py:52-54; split / uniform / normal / permutation in
// pkpd_simulation.py:117-197, 233-236, 290-291).  jax's default PRNG is Threefry-2x32-20 (Salmon et al.,
// SC'11) applied to a flat counter array: jax.prng.threefry_2x32(key, iota(n)) pads the counts to an even
// length m, hashes the pairs (c[j], c[j + m/2]) and concatenates the two output halves.  This kernel
// produces exactly those n words on the device -- one thread per pair, two 32-bit stores -- so the
// product's generator (insite_amd/threefry.py, insite_amd/pkpd.py) reproduces the reference's cohorts
// without a host round trip.  Integer work: bound by the store bandwidth (4 B per word), a few hundred
// integer VALU ops per pair.  Pinned by the Random123 known-answer vectors (tests/test_gpu_threefry.py).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "insite_hip.h"
#include "insite_common.h"

namespace {

__device__ __forceinline__ uint32_t rotl32(uint32_t v, int r) { return (v << r) | (v >> (32 - r)); }

__device__ __forceinline__ void threefry2x32_20(uint32_t k0, uint32_t k1, uint32_t& a, uint32_t& b) {
  const uint32_t ks[3] = {k0, k1, k0 ^ k1 ^ 0x1BD11BDAu};
  constexpr int R[2][4] = {{13, 15, 26, 6}, {17, 29, 16, 24}};
  a += ks[0];
  b += ks[1];
#pragma unroll
  for (int g = 0; g < 5; ++g) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      a += b;
      b = rotl32(b, R[g & 1][i]) ^ a;
    }
    a += ks[(g + 1) % 3];
    b += ks[(g + 2) % 3] + (uint32_t)(g + 1);
  }
}

// out[i], i < n: word i of threefry_2x32(key, iota(n)); thread j hashes (j, j + h) with h = ceil(n / 2)
// (the padded count m / 2; the pad count is 0)
__global__ void __launch_bounds__(kBlock)
threefry_iota_kernel(uint32_t k0, uint32_t k1, int64_t n, uint32_t* __restrict__ out) {
  const int64_t h = (n + 1) / 2;
  const int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (j >= h) return;
  uint32_t a = (uint32_t)j;
  uint32_t b = j + h < n ? (uint32_t)(j + h) : 0u;
  threefry2x32_20(k0, k1, a, b);
  out[j] = a;
  if (j + h < n) out[j + h] = b;
}

}  // namespace

extern "C" int32_t insite_threefry2x32_iota_u32(uint32_t key0, uint32_t key1, int64_t n_words, uint32_t* out,
                                                void* stream) {
  if (n_words < 0 || n_words >= 0xFFFFFFFFll) return INSITE_E_INVALID_ARG;
  if (n_words == 0) return INSITE_OK;
  if (!out) return INSITE_E_INVALID_ARG;
  const int64_t h = (n_words + 1) / 2;
  threefry_iota_kernel<<<(unsigned)((h + kBlock - 1) / kBlock), kBlock, 0, reinterpret_cast<hipStream_t>(stream)>>>(
      key0, key1, n_words, out);
  return launch_status();
}
