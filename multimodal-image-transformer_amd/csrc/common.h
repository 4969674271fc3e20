// Shared device helpers for the gfx950 (CDNA4 / MI355X) kernels of the captioning train step.
// Wave64 everywhere; bf16 activations with fp32 accumulation, or fp32 end to end (parity mode).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mit_hip.h"

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(bf16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f(float x);
template <> __device__ __forceinline__ float from_f<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f<bf16>(float x) { return (bf16)x; }

// ---------------------------------------------------------------------------------------------
// Counter-based dropout RNG: keep(i) = mix(seed ^ site, i) >= p * 2^32. Stateless, so the
// backward regenerates the forward's mask from (seed, site, element index) without storing it.
// The seed lives in device memory so a captured hipGraph replays with a fresh seed per step.
// ---------------------------------------------------------------------------------------------
// 32-bit "lowbias32" permutation (2 multiplies): the backward regenerates every mask element of
// the attention / FFN / residual dropouts, so the hash is VALU work on the critical kernels (a
// 64-bit splitmix finaliser cost ~3x the instructions: ~9 32-bit multiplies per element)
__device__ __forceinline__ uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
// one lowbias32 round over the element index keyed by (seed, site): the key's two halves fold into one
// wave-uniform word (scalar work), the index's high half (0 below 2^32 elements) is added before the
// round. Was two rounds (the second mixing the high halves): the decoder's dropout sites hash every
// element they touch, forward and backward, so the round is VALU on the critical kernels.
// The index's high half enters by a rotate-add, not a multiply: v_mul_lo_u32 is a quarter-rate VALU op and
// every index below 2^32 (all of the train step's) has a zero high half, so the masks are the ones the
// multiply form gave, bit for bit, at one multiply less per element (the attention backward hashes every
// score it touches).
__device__ __forceinline__ uint32_t mix_u32(uint64_t key, uint64_t idx) {
  const uint32_t k = (uint32_t)key ^ ((uint32_t)(key >> 32) * 0x9E3779B9u);
  const uint32_t hi = (uint32_t)(idx >> 32);
  return lowbias32(((uint32_t)idx ^ k) + ((hi << 16) | (hi >> 16)));
}
// mix_u32 for an index below 2^32, with the key folded once per thread (key_fold): the same value
__device__ __forceinline__ uint32_t key_fold(uint64_t key) { return (uint32_t)key ^ ((uint32_t)(key >> 32) * 0x9E3779B9u); }
__device__ __forceinline__ float drop_mul32(uint32_t kf, uint32_t idx, uint32_t thresh, float scale) {
  return lowbias32(idx ^ kf) >= thresh ? scale : 0.0f;
}
__device__ __forceinline__ uint64_t site_key(const uint64_t* seed, uint32_t site) {
  return (seed ? *seed : 0ull) ^ (0xD6E8FEB86659FD93ull * (uint64_t)(site + 1));
}
// returns the dropout multiplier (0 or 1/(1-p)) for element idx
__device__ __forceinline__ float drop_mul(uint64_t key, uint64_t idx, uint32_t thresh, float scale) {
  return mix_u32(key, idx) >= thresh ? scale : 0.0f;
}
static inline uint32_t drop_threshold(float p) {
  double t = (double)p * 4294967296.0;
  if (t >= 4294967295.0) t = 4294967295.0;
  return (uint32_t)t;
}

// ---------------------------------------------------------------------------------------------
// Wave64 reductions
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// block reduction (blockDim multiple of 64, <= 1024); scratch >= 16 floats
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, nw = blockDim.x >> 6;
  __syncthreads();
  if (l == 0) scratch[w] = v;
  __syncthreads();
  float r = (l < nw) ? scratch[l] : 0.0f;
  r = wave_sum(r);
  return r;
}
__device__ __forceinline__ float block_max(float v, float* scratch) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, nw = blockDim.x >> 6;
  __syncthreads();
  if (l == 0) scratch[w] = v;
  __syncthreads();
  float r = (l < nw) ? scratch[l] : -INFINITY;
  r = wave_max(r);
  return r;
}

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.0f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float quick_gelu(float x) { return x / (1.0f + __expf(-1.702f * x)); }
// GELU (erf form) without ocml's branchy erff, for bf16 epilogues: Phi(x) = 1 - 0.5*erfc(x/sqrt2)
// with erfc(a) = t*P(t)*exp(-a^2), t = 1/(1 + 0.3275911 a) (Abramowitz-Stegun 7.1.26, |error| of
// erf <= 1.5e-7), evaluated on |x| so the negative tail keeps its relative accuracy (no 1 - 1).
// ~12 VALU ops incl. one v_rcp and one v_exp; fp32 parity mode keeps gelu_erf.
__device__ __forceinline__ float gelu_fast(float x) {
  const float a = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, a, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float h = 0.5f * p * t * __expf(-a * a);  // 0.5 * erfc(|x|/sqrt2) = Phi(-|x|)
  return x * (x >= 0.0f ? 1.0f - h : h);
}

// gelu_fast on two values with packed FP32 math (v_pk_fma_f32 / v_pk_mul_f32: two lanes' worth of
// the polynomial per instruction); the rcp / exp stay scalar. The A&S 7.1.26 evaluation with the
// constants folded: t = 1 / (1 + (0.3275911/sqrt2)|x|), h = Phi(-|x|) = t * (P(t)/2) * 2^(-x^2 log2(e)/2)
// (the 0.5 in the coefficients, the exp's log2(e)/2 in one multiply of x^2), y = x >= 0 ? x - x h : x h
// (enc fc1+GELU 85.3-88.1 vs 88.9-90.3 us with the unfolded form, step +0.25 %).
typedef __attribute__((ext_vector_type(2))) float f32x2;
__device__ __forceinline__ f32x2 gelu_fast2(f32x2 x) {
  const f32x2 ax = __builtin_elementwise_abs(x);
  const f32x2 d = __builtin_elementwise_fma(f32x2{0.23164189f, 0.23164189f}, ax, f32x2{1.0f, 1.0f});
  const f32x2 t = {__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
  f32x2 p = __builtin_elementwise_fma(f32x2{0.5307027145f, 0.5307027145f}, t, f32x2{-0.7265760135f, -0.7265760135f});
  p = __builtin_elementwise_fma(p, t, f32x2{0.7107068705f, 0.7107068705f});
  p = __builtin_elementwise_fma(p, t, f32x2{-0.142248368f, -0.142248368f});
  p = __builtin_elementwise_fma(p, t, f32x2{0.127414796f, 0.127414796f});
  const f32x2 z = (x * x) * -0.72134752044448170f;  // -x^2/2 in log2 units
  const f32x2 e = {__builtin_amdgcn_exp2f(z[0]), __builtin_amdgcn_exp2f(z[1])};
  const f32x2 xh = x * (p * t * e);
  const f32x2 xm = x - xh;
  return f32x2{x[0] >= 0.0f ? xm[0] : xh[0], x[1] >= 0.0f ? xm[1] : xh[1]};
}

// Kernel extent asserts (sanitizers): compiled in only by the diagnostic build
// (`make -C multimodal-image-transformer_amd/csrc asserts` -> lib/variants/libmit_hip_asserts.so, loaded with
// MIT_LIB=...; tests/test_asserts_gpu.py runs GEMMs and attentions under it). A failing assert traps the
// kernel with the file:line of the violated extent instead of reading or writing out of range. The
// shipped library compiles none of it.
#ifndef MIT_DEVICE_ASSERTS
#define MIT_DEVICE_ASSERTS 0
#endif
#if MIT_DEVICE_ASSERTS
#include <cassert>
#define MIT_DASSERT(cond) assert(cond)
#else
#define MIT_DASSERT(cond) \
  do {                    \
  } while (0)
#endif

// error plumbing shared by every C-ABI entry point (capi.cpp)
int mit_set_error(const char* fmt, ...);

// launch-plan recording (capi.cpp, mit_plan_*): while a plan records, every launching entry point
// appends a replay closure (arguments copied by value) and then runs normally, so the recorded step
// is a real step and argument errors surface at record time.
#include <functional>
bool mit_plan_recording();
void mit_plan_push(std::function<int()> op);
#define MIT_RECORD(...)                                \
  do {                                                 \
    if (mit_plan_recording()) mit_plan_push(__VA_ARGS__); \
  } while (0)
#define MIT_CHECK_ARG(cond, ...)          \
  do {                                    \
    if (!(cond)) {                        \
      mit_set_error(__VA_ARGS__);         \
      return MIT_ERR_INVALID;             \
    }                                     \
  } while (0)
#define MIT_LAUNCH_CHECK(name)                                              \
  do {                                                                      \
    hipError_t e_ = hipGetLastError();                                      \
    if (e_ != hipSuccess) {                                                 \
      mit_set_error("%s: launch failed: %s", name, hipGetErrorString(e_));  \
      return MIT_ERR_HIP;                                                   \
    }                                                                       \
  } while (0)
