// Store-pattern microbenchmark for the 256x256 bf16 GEMM epilogue: one 512-thread
// workgroup per output tile writes its 128 KiB with 16 store instructions per wave (dwordx4 per lane),
// in one of several lane -> address patterns; per workgroup the shader-clock time from the first
// store to the last store's completion. Build: hipcc -O3 --offload-arch=gfx950 tools/store_bench.hip
// -o tools/store_bench ; run: tools/store_bench  (prints one line per pattern x matrix x grid).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

template <int PAT>
__global__ __launch_bounds__(512) void store_kernel(unsigned short* C, long ldc, int tiles_n, unsigned long long* cyc) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, wr = wid >> 2, wc = wid & 3, g = lane >> 4;
  const long m0 = (long)(blockIdx.x / tiles_n) * 256, n0 = (long)(blockIdx.x % tiles_n) * 256;
  u32x4 v = {(unsigned)tid, (unsigned)lane * 3u, 7u, (unsigned)blockIdx.x};
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    long r, c;
    if (PAT == 0) {  // the register epilogue: 16 rows x 64 B (4 lanes per row), wave quadrant 128 x 64
      const int i = q >> 1, jp = q & 1;
      r = wr * 128 + i * 16 + (lane & 15);
      c = wc * 64 + (g & 1) * 16 + (g >> 1) * 8 + jp * 32;
    } else if (PAT == 1) {  // 8 rows x 128 B, wave quadrant
      r = wr * 128 + q * 8 + (lane >> 3);
      c = wc * 64 + (lane & 7) * 8;
    } else if (PAT == 2) {  // 2 rows x 512 B, 32 rows per wave
      r = wid * 32 + q * 2 + (lane >> 5);
      c = (lane & 31) * 8;
    } else if (PAT == 3) {  // 4 rows x 256 B, 32 rows per wave
      r = wid * 32 + (q >> 1) * 4 + (lane >> 4);
      c = (q & 1) * 128 + (lane & 15) * 8;
    } else if (PAT == 4) {  // 2 rows x 512 B, rows interleaved over the waves
      r = (q * 8 + wid) * 2 + (lane >> 5);
      c = (lane & 31) * 8;
    } else {  // PAT 5: 1 row x 1 KiB (two tiles' columns: a 512-column band), 16 rows per wave (n0 even only)
      const long odd = (long)((blockIdx.x % tiles_n) & 1);  // signed: c may step back one tile
      r = wid * 16 + q + odd * 128;
      c = (long)lane * 8 - odd * 256;
    }
    *(u32x4*)(C + (m0 + r) * ldc + n0 + c) = v;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) cyc[blockIdx.x * 8 + wid] = t1 - t0;
}

template <int PAT>
float run(unsigned short* C, long M, long N, int blocks, unsigned long long* d_cyc, double* med_cyc) {
  const int tiles_n = (int)(N / 256);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(store_kernel<PAT>, dim3(blocks), dim3(512), 0, 0, C, N, tiles_n, d_cyc);
  hipEventRecord(e0, 0);
  const int it = 20;
  for (int w = 0; w < it; ++w) hipLaunchKernelGGL(store_kernel<PAT>, dim3(blocks), dim3(512), 0, 0, C, N, tiles_n, d_cyc);
  hipEventRecord(e1, 0);
  if (hipEventSynchronize(e1) != hipSuccess || hipGetLastError() != hipSuccess) {
    fprintf(stderr, "store_kernel<%d> failed: stopping\n", PAT);
    exit(1);
  }
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> h(blocks * 8);
  hipMemcpy(h.data(), d_cyc, h.size() * 8, hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  *med_cyc = (double)h[h.size() / 2];
  (void)M;
  return ms * 1000.f / it;
}

int main() {
  const long M = 4096, Ns[3] = {256, 2048, 2304};
  unsigned short* C;
  unsigned long long* cyc;
  hipMalloc(&C, M * 4096 * 2 + (1 << 20));
  hipMalloc(&cyc, 8 * 4096 * 8);
  const char* names[6] = {"16 rows x 64 B (register epilogue)", "8 rows x 128 B", "2 rows x 512 B, wave rows",
                          "4 rows x 256 B, wave rows", "2 rows x 512 B, interleaved waves", "1 row x 1 KiB"};
  for (long N : Ns) {
    const int tiles = (int)((M / 256) * (N / 256));
    for (int blocks : {8, 64, tiles}) {
      if (blocks > tiles) continue;
      for (int pat = 0; pat < 6; ++pat) {
        if (pat == 5 && (N / 256) % 2) continue;
        double med = 0;
        float us = 0;
        switch (pat) {
          case 0: us = run<0>(C, M, N, blocks, cyc, &med); break;
          case 1: us = run<1>(C, M, N, blocks, cyc, &med); break;
          case 2: us = run<2>(C, M, N, blocks, cyc, &med); break;
          case 3: us = run<3>(C, M, N, blocks, cyc, &med); break;
          case 4: us = run<4>(C, M, N, blocks, cyc, &med); break;
          default: us = run<5>(C, M, N, blocks, cyc, &med); break;
        }
        printf("N=%5ld blocks=%4d  %-36s launch %7.2f us  per-wave store phase %8.0f cycles\n", N, blocks, names[pat],
               us, med);
      }
    }
  }
  hipFree(C);
  hipFree(cyc);
  return 0;
}
