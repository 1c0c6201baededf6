#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
template <int MODE>
__device__ __forceinline__ void philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1, uint32_t o[4])
{
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0, lo0, hi1, lo1;
    if (MODE == 0) {
      hi0 = __umulhi(0xD2511F53u, c0); lo0 = 0xD2511F53u * c0;
      hi1 = __umulhi(0xCD9E8D57u, c2); lo1 = 0xCD9E8D57u * c2;
    } else {
      uint64_t p0 = (uint64_t)c0 * 0xD2511F53u, p1 = (uint64_t)c2 * 0xCD9E8D57u;
      hi0 = (uint32_t)(p0 >> 32); lo0 = (uint32_t)p0; hi1 = (uint32_t)(p1 >> 32); lo1 = (uint32_t)p1;
    }
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  o[0] = c0; o[1] = c1; o[2] = c2; o[3] = c3;
}
template <int MODE>
__global__ __launch_bounds__(256) void k(uint32_t* out, uint32_t a, uint32_t b, int iters) {
  uint32_t acc = 0, x = threadIdx.x + blockIdx.x * 256;
  for (int i = 0; i < iters; ++i) {
    uint32_t o[4]; philox<MODE>(x, (uint32_t)i, a, acc, a, b, o);
    acc ^= o[0] + o[1] + o[2] + o[3];
  }
  out[threadIdx.x + blockIdx.x * 256] = acc;
}
int main() {
  uint32_t* d; int n = 256 * 4096; hipMalloc(&d, n * 4);
  uint32_t *h0 = (uint32_t*)malloc(n*4), *h1 = (uint32_t*)malloc(n*4);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int rep = 0; rep < 3; ++rep) {
    for (int m = 0; m < 2; ++m) {
      hipEventRecord(e0);
      if (m == 0) k<0><<<4096, 256>>>(d, 7, 9, 2000); else k<1><<<4096, 256>>>(d, 7, 9, 2000);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      hipMemcpy(m ? h1 : h0, d, n * 4, hipMemcpyDeviceToHost);
      double draws = (double)n * 2000;
      printf("mode %d: %.3f ms, %.1f Gdraws/s\n", m, ms, draws / ms / 1e6);
    }
  }
  int same = 1; for (int i = 0; i < n; ++i) same &= h0[i] == h1[i];
  printf("identical %d\n", same);
  return 0;
}
