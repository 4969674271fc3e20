// Exhaustive check of the kernels' quick_gelu (csrc/common.h) against the IEEE-division form over all
// 2^32 float32 inputs (tools/ check, not product code): prints the number of inputs whose results differ
// bitwise and the first few of them. Build: hipcc --offload-arch=gfx950 -O2 tools/qgelu_exhaustive.hip
// -o tools/_bin/qgelu_exhaustive (tools/gpu_qgelu.sh)
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <cstdint>
#include <cstdio>
#include <vector>

#include "../multimodal-image-transformer_amd/csrc/common.h"

// quick_gelu (one value) and quick_gelu_n<4> (four consecutive inputs, so groups mixing the fast and the
// division path are covered) against quick_gelu_ieee
__global__ void check(uint32_t base, uint32_t per_thread, unsigned long long* cnt, uint32_t* first) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long bad = 0;
  uint32_t f = 0xFFFFFFFFu;
  for (uint32_t k = 0; k < per_thread; k += 4) {
    float v[4], x[4];
    for (int i = 0; i < 4; ++i) v[i] = x[i] = __uint_as_float(base + t * per_thread + k + i);
    quick_gelu_n<4>(v);
    for (int i = 0; i < 4; ++i) {
      const float a = quick_gelu_ieee(x[i]), b = v[i], c = quick_gelu(x[i]);
      const bool same_b = __float_as_uint(a) == __float_as_uint(b) || (a != a && b != b);
      const bool same_c = __float_as_uint(a) == __float_as_uint(c) || (a != a && c != c);
      if (!same_b || !same_c) {
        ++bad;
        if (f == 0xFFFFFFFFu) f = base + t * per_thread + k + i;
      }
    }
  }
  cnt[t] = bad;
  first[t] = f;
}

int main() {
  const int threads = 256, blocks = 16384;
  const uint32_t n = threads * blocks, per = 64;  // 2^22 threads x 64 = 2^28 inputs per launch, 16 launches
  unsigned long long* d_cnt;
  uint32_t* d_first;
  hipMalloc(&d_cnt, n * sizeof(unsigned long long));
  hipMalloc(&d_first, n * sizeof(uint32_t));
  std::vector<unsigned long long> cnt(n);
  std::vector<uint32_t> first(n);
  unsigned long long total = 0;
  int shown = 0;
  for (uint32_t l = 0; l < 16; ++l) {
    hipLaunchKernelGGL(check, dim3(blocks), dim3(threads), 0, 0, l << 28, per, d_cnt, d_first);
    if (hipDeviceSynchronize() != hipSuccess) {
      printf("kernel failed\n");
      return 1;
    }
    hipMemcpy(cnt.data(), d_cnt, n * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    hipMemcpy(first.data(), d_first, n * sizeof(uint32_t), hipMemcpyDeviceToHost);
    for (uint32_t i = 0; i < n; ++i) {
      total += cnt[i];
      if (cnt[i] && shown < 8) {
        float x;
        memcpy(&x, &first[i], 4);
        printf("mismatch at x = %.9g (0x%08x)\n", x, first[i]);
        ++shown;
      }
    }
  }
  printf("inputs differing bitwise: %llu of 2^32\n", total);
  return total ? 2 : 0;
}
