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
// quick_gelu(x) = x / (1 + e^(-1.702 x)), the form the kernels computed through round 5 (the compiler's
// IEEE division expansion: v_div_scale / v_div_fmas / v_div_fixup around a denormal-mode switch)
__device__ __forceinline__ float quick_gelu_ieee(float x) { return x / (1.0f + __expf(-1.702f * x)); }
// the same quotient for |x| <= 51 without the expansion: v_rcp_f32 of d in [1, 2^126), then one
// FMA-corrected quotient (Markstein), the sign of x restored for x = -0 (a Newton step on the reciprocal
// first is not needed: 0 of 2^32 inputs differ without it)
__device__ __forceinline__ float quick_gelu_core(float x) {
  const float d = 1.0f + __expf(-1.702f * x);
  const float y = __builtin_amdgcn_rcpf(d);
  const float q = x * y;
  return copysignf(fmaf(fmaf(-d, q, x), y, q), x);
}
// N values: the core form for all of them, and ONE branch (no lane of a real activation takes it) back to
// the division when any |x| > 51 or is not finite (d near or past the float range). Bitwise identical to
// quick_gelu_ieee over all 2^32 inputs (tools/qgelu_exhaustive.hip); per-value branches cost more than the
// expansion they save (CLIP fc1 374 vs 343 us)
template <int N>
__device__ __forceinline__ void quick_gelu_n(float* v) {
  float x[N];
  bool slow = false;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    x[k] = v[k];
    slow |= !(fabsf(x[k]) <= 51.0f);
    v[k] = quick_gelu_core(x[k]);
  }
  if (__builtin_expect(slow, 0)) {
#pragma unroll
    for (int k = 0; k < N; ++k) v[k] = quick_gelu_ieee(x[k]);
  }
}
__device__ __forceinline__ float quick_gelu(float x) {
  quick_gelu_n<1>(&x);
  return x;
}
// quick_gelu for the bf16 vector epilogues (the CLIP towers' fc1): x * rcp(d), v_rcp_f32 without the
// FMA-corrected quotient -- within ~1 ulp of the division (1/65536 of a bf16 ulp), 4 VALU fewer per value than
// quick_gelu_n and no branch. Large negative x: d = inf, rcp 0, -0 (the division gives -0 too); +inf -> +inf;
// -inf and NaN -> NaN (x * sigmoid(1.702 x) in torch: -inf * 0 = NaN). configs[2] 2028 -> 2048 pairs/s
// (interleaved, one box); its parity side: profiles/r06_grad_metric_report.json (the trimmed worst-tensor
// gradient metric moves 0.2-0.9 %). The scalar / fp32-parity path keeps the exact division (quick_gelu).
// In pairs: the multiplies and the add as packed FP32 (v_pk_mul_f32 / v_pk_add_f32), the same roundings as
// the scalar form (__expf(y) = v_exp_f32(y * log2(e))): bitwise identical, 4 packed VALU + 4 transcendentals
// per two values instead of 8 + 4. (One multiply by the merged constant -1.702 log2(e) would save another,
// but moves the exponent by an ulp on 29 % of inputs, and the fixtures' 64-pin worst-gradient metric with it.)
typedef __attribute__((ext_vector_type(2))) float f32x2;
template <int N>
__device__ __forceinline__ void quick_gelu_fast_n(float* v) {
  static_assert(N % 2 == 0, "quick_gelu_fast_n: pairs of values");
  constexpr float c = -1.702f, l2e = 1.44269504088896341f;
#pragma unroll
  for (int k = 0; k < N; k += 2) {
    const f32x2 x = {v[k], v[k + 1]};
    const f32x2 z = (x * f32x2{c, c}) * f32x2{l2e, l2e};
    const f32x2 d = f32x2{__builtin_amdgcn_exp2f(z[0]), __builtin_amdgcn_exp2f(z[1])} + f32x2{1.0f, 1.0f};
    const f32x2 r = x * f32x2{__builtin_amdgcn_rcpf(d[0]), __builtin_amdgcn_rcpf(d[1])};
    v[k] = r[0];
    v[k + 1] = r[1];
  }
}
// GELU (erf form) for bf16 epilogues with ONE transcendental and no select: x Phi(x) = max(x, 0) - a h,
// a = min(|x|, 6), h = Phi(-a) = 2^q(a), q a degree-7 fit of log2 Phi(-a) on [0, 6] (tools/gelu_fit.py):
// relative error <= 6.6e-6 for |x| <= 6 (1/300 of a bf16 half-ulp; the negative tail keeps its relative
// accuracy, no 1 - 1). Past |x| = 6 the correction term is the constant 6 Phi(-6) = 5.9e-9, so the error
// stays <= 5.9e-9 absolute for every x (a = |x| there would grow it with |x|, and turn x = +inf into
// inf - inf); x = +-inf gives +inf / -5.9e-9. a is the NaN-propagating minimum (v_minimum3_f32, one op like
// v_min_f32), so a NaN input stays NaN. 10 VALU + one v_exp_f32, against the A&S 7.1.26 form's rcp + exp +
// compare / select; fp32 parity mode keeps gelu_erf.
#define MIT_GELU_Q(F) F(-1.834813247e-06f), F(6.159832992e-05f), F(-9.305251297e-04f), F(8.507891558e-03f), \
                      F(-5.396007001e-02f), F(-4.584643841e-01f), F(-1.151251078e+00f), F(-9.999952912e-01f)
#define MIT_GELU_S(c) c
__device__ __forceinline__ float gelu_fast(float x) {
  constexpr float q[8] = {MIT_GELU_Q(MIT_GELU_S)};
  const float a = __builtin_elementwise_minimum(fabsf(x), 6.0f);
  float p = fmaf(q[0], a, q[1]);
#pragma unroll
  for (int k = 2; k < 8; ++k) p = fmaf(p, a, q[k]);
  return fmaf(-a, __builtin_amdgcn_exp2f(p), fmaxf(x, 0.0f));
}

// gelu_fast on two values: the polynomial and the final FMA in packed FP32 (v_pk_fma_f32, two values per
// instruction); min / exp2 / max scalar
__device__ __forceinline__ f32x2 gelu_fast2(f32x2 x) {
  constexpr float q[8] = {MIT_GELU_Q(MIT_GELU_S)};
  const f32x2 a = {__builtin_elementwise_minimum(fabsf(x[0]), 6.0f), __builtin_elementwise_minimum(fabsf(x[1]), 6.0f)};
  f32x2 p = __builtin_elementwise_fma(f32x2{q[0], q[0]}, a, f32x2{q[1], q[1]});
#pragma unroll
  for (int k = 2; k < 8; ++k) p = __builtin_elementwise_fma(p, a, f32x2{q[k], q[k]});
  const f32x2 h = {__builtin_amdgcn_exp2f(p[0]), __builtin_amdgcn_exp2f(p[1])};
  return __builtin_elementwise_fma(-a, h, f32x2{fmaxf(x[0], 0.0f), fmaxf(x[1], 0.0f)});
}
#undef MIT_GELU_S
#undef MIT_GELU_Q

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
