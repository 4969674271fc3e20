// Batched greedy decoding with a KV cache (BASELINE config 5): the per-token
// step of ImageToTextModel.generate (model.py:171-242) for a whole batch of images, every position
// index read from DEVICE memory so the step captures into one hipGraph and replays per token.
//
//   mit_embed_decode    x[b] = Emb[ids[b, pos]] * scale + pe[pos]                 (decoder.py:168-171)
//   mit_kv_store        cache[b, pos, :] = src[b, :]   (this token's K|V row of the self-attn in_proj)
//   mit_attention_decode one query per (batch, head) against Lk cached keys: Lk = *pos + 1 for the
//                       causal self-attention (keys whose token is PAD masked, as the reference's
//                       key-padding mask does), or a fixed S for cross-attention over the image
//   mit_greedy_pick     ids[b, pos+1] = argmax_v logits[b, v] (first maximal index, torch.argmax),
//                       finished[b] once END is produced (model.py:236-240)
//
// The decode attention is HBM-bound (each (b, h) streams its K/V rows once): one 256-thread block
// per (b, h); 8 lanes per key row (16-B loads, a 128-B row per lane group), 8 keys per wave-
// iteration, 4 waves over disjoint key ranges; online softmax in registers, groups and waves
// merged at the end (shuffles, then LDS).
#include "common.h"

namespace {

template <typename T>
__device__ __forceinline__ void load8(const T* p, float* f);
template <>
__device__ __forceinline__ void load8<bf16>(const bf16* p, float* f) {
  const bf16x8 v = *(const bf16x8*)p;
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = (float)v[i];
}
template <>
__device__ __forceinline__ void load8<float>(const float* p, float* f) {
  const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
  f[0] = a[0]; f[1] = a[1]; f[2] = a[2]; f[3] = a[3]; f[4] = b[0]; f[5] = b[1]; f[6] = b[2]; f[7] = b[3];
}
template <typename T>
__device__ __forceinline__ void store8(T* p, const float* f);
template <>
__device__ __forceinline__ void store8<bf16>(bf16* p, const float* f) {
  bf16x8 v;
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (bf16)f[i];
  *(bf16x8*)p = v;
}
template <>
__device__ __forceinline__ void store8<float>(float* p, const float* f) {
  *(f32x4*)p = f32x4{f[0], f[1], f[2], f[3]};
  *(f32x4*)(p + 4) = f32x4{f[4], f[5], f[6], f[7]};
}

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kNegBig = -1e30f;  // running-max sentinel: keeps exp2(m_old - m_new) finite

// merge (m2, l2, acc2) into (m, l, acc)
__device__ __forceinline__ void merge(float& m, float& l, float* acc, float m2, float l2, const float* acc2) {
  const float mn = fmaxf(m, m2);
  const float c1 = exp2f(m - mn), c2 = exp2f(m2 - mn);
  l = l * c1 + l2 * c2;
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = acc[i] * c1 + acc2[i] * c2;
  m = mn;
}

// head_dim DH in {16, 32, 64, 128}: LPR = DH / 8 lanes per key row (8 elements each), KPW = 64 / LPR
// keys per wave iteration
template <typename T, int DH>
__global__ __launch_bounds__(256) void attn_decode_kernel(long H, const T* __restrict__ q, long q_batch,
                                                          const T* __restrict__ k, long k_row, long k_batch,
                                                          const T* __restrict__ v, long v_row, long v_batch,
                                                          T* __restrict__ o, long o_batch, long lk_fixed,
                                                          const int64_t* __restrict__ pos,
                                                          const int64_t* __restrict__ key_tokens, long tok_batch,
                                                          int pad_idx, float scale) {
  constexpr int LPR = DH / 8, KPW = 64 / LPR;
  __shared__ float red[4][2 + DH];
  const int bh = blockIdx.x;
  const long b = bh / H, h = bh % H;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, g = lane / LPR, c = lane % LPR;
  const long Lk = pos ? (*pos + 1) : lk_fixed;

  float qv[8];
  load8<T>(q + b * q_batch + h * DH + c * 8, qv);
#pragma unroll
  for (int i = 0; i < 8; ++i) qv[i] *= scale * kLog2e;

  const T* kb = k + b * k_batch + h * DH + c * 8;
  const T* vb = v + b * v_batch + h * DH + c * 8;
  const int64_t* tb = key_tokens ? key_tokens + b * tok_batch : nullptr;
  float m = kNegBig, l = 0.f, acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  // key j = (it * 4 + w) * KPW + g: the four waves sweep interleaved KPW-key slabs
  for (long j = (long)w * KPW + g; j - g < Lk; j += 4 * KPW) {
    const bool ok = j < Lk && (!tb || tb[j] != pad_idx);
    float kf[8], vf[8];
    if (j < Lk) {
      load8<T>(kb + j * k_row, kf);
      load8<T>(vb + j * v_row, vf);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) kf[i] = vf[i] = 0.f;
    }
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) s = fmaf(qv[i], kf[i], s);
#pragma unroll
    for (int x = 1; x < LPR; x <<= 1) s += __shfl_xor(s, x, 64);
    if (!ok) s = -INFINITY;
    const float mn = fmaxf(m, s);
    const float corr = exp2f(m - mn), p = exp2f(s - mn);
    l = l * corr + p;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = fmaf(p, vf[i], acc[i] * corr);
    m = mn;
  }
  // merge the KPW key groups of the wave (lanes with equal c)
#pragma unroll
  for (int x = LPR; x < 64; x <<= 1) {
    float a2[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) a2[i] = __shfl_xor(acc[i], x, 64);
    merge(m, l, acc, __shfl_xor(m, x, 64), __shfl_xor(l, x, 64), a2);
  }
  if (g == 0) {
    if (c == 0) {
      red[w][0] = m;
      red[w][1] = l;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) red[w][2 + c * 8 + i] = acc[i];
  }
  __syncthreads();
  if (w == 0 && g == 0) {
    for (int w2 = 1; w2 < 4; ++w2) merge(m, l, acc, red[w2][0], red[w2][1], &red[w2][2 + c * 8]);
    float out[8];
    const float inv = 1.0f / l;  // all keys masked -> 0/0 = NaN, as the reference's softmax
#pragma unroll
    for (int i = 0; i < 8; ++i) out[i] = acc[i] * inv;
    store8<T>(o + b * o_batch + h * DH + c * 8, out);
  }
}

template <typename T>
__global__ void kv_store_kernel(long B, long n, const T* __restrict__ src, long s_batch, T* __restrict__ cache,
                                long c_row, long c_batch, const int64_t* __restrict__ pos) {
  const long p = *pos;
  const long total = B * n;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long b = i / n, e = i % n;
    cache[b * c_batch + p * c_row + e] = src[b * s_batch + e];
  }
}

template <typename T>
__global__ void embed_decode_kernel(long B, long d, const int64_t* __restrict__ ids, long ld_ids,
                                    const int64_t* __restrict__ pos, const T* __restrict__ table, float scale,
                                    const float* __restrict__ pe, T* __restrict__ out) {
  const long p = *pos;
  const long total = B * d;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long b = i / d, e = i % d;
    const int64_t id = ids[b * ld_ids + p];
    out[i] = from_f<T>(to_f(table[id * d + e]) * scale + pe[p * d + e]);
  }
}

// one block per row: first index of the maximum (torch.argmax), NaN counts as maximal
__global__ __launch_bounds__(256) void greedy_pick_kernel(long V, const float* __restrict__ logits, long ld,
                                                          int64_t* __restrict__ ids, long ld_ids,
                                                          const int64_t* __restrict__ pos, int64_t end_id,
                                                          int64_t pad_id, int* __restrict__ finished,
                                                          int* __restrict__ n_finished) {
  __shared__ float sv[4];
  __shared__ long si[4];
  const long b = blockIdx.x;
  const float* row = logits + b * ld;
  // (value desc, index asc), NaN largest
  auto better = [](float a, long ia, float bv, long ib) {
    const bool an = a != a, bn = bv != bv;
    if (an != bn) return an;
    if (a != bv && !an) return a > bv;
    return ia < ib;
  };
  float best = -INFINITY;
  long bi = V;  // V = none yet (loses every tie on index)
  for (long j = threadIdx.x; j < V; j += blockDim.x) {
    const float x = row[j];
    if (better(x, j, best, bi)) {
      best = x;
      bi = j;
    }
  }
#pragma unroll
  for (int x = 32; x > 0; x >>= 1) {
    const float ov = __shfl_xor(best, x, 64);
    const long oi = __shfl_xor(bi, x, 64);
    if (better(ov, oi, best, bi)) {
      best = ov;
      bi = oi;
    }
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sv[w] = best;
    si[w] = bi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < (int)(blockDim.x >> 6); ++k)
      if (better(sv[k], si[k], best, bi)) {
        best = sv[k];
        bi = si[k];
      }
    const long p = *pos;
    if (finished[b]) {
      ids[b * ld_ids + p + 1] = pad_id;
    } else {
      ids[b * ld_ids + p + 1] = bi;
      if (bi == end_id) {
        finished[b] = 1;
        atomicAdd(n_finished, 1);
      }
    }
  }
}

inline unsigned grid_for(long n, int block = 256, long cap = 8192) {
  long g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

}  // namespace

#define DISPATCH_DT(dtype, ...)       \
  do {                                \
    if ((dtype) == MIT_BF16) {        \
      typedef bf16 T;                 \
      __VA_ARGS__;                    \
    } else {                          \
      typedef float T;                \
      __VA_ARGS__;                    \
    }                                 \
  } while (0)

extern "C" int mit_attention_decode(int dtype, long B, long H, long Dh, const void* q, long q_batch, const void* k,
                                    long k_row, long k_batch, const void* v, long v_row, long v_batch, void* o,
                                    long o_batch, long Lk, const int64_t* pos, const int64_t* key_tokens,
                                    long tok_batch, int pad_idx, float scale, void* stream) {
  MIT_RECORD([=]() { return mit_attention_decode(dtype, B, H, Dh, q, q_batch, k, k_row, k_batch, v, v_row, v_batch, o, o_batch, Lk, pos, key_tokens, tok_batch, pad_idx, scale, stream); });
  MIT_CHECK_ARG(q && k && v && o, "mit_attention_decode: null pointer");
  MIT_CHECK_ARG(Dh == 16 || Dh == 32 || Dh == 64 || Dh == 128, "mit_attention_decode: head_dim %ld unsupported", Dh);
  MIT_CHECK_ARG(dtype == MIT_BF16 || dtype == MIT_F32, "mit_attention_decode: bad dtype");
  MIT_CHECK_ARG(pos || Lk > 0, "mit_attention_decode: need a device position or Lk > 0");
  const long esz = dtype == MIT_BF16 ? 2 : 4;
  MIT_CHECK_ARG(((uintptr_t)q | (uintptr_t)k | (uintptr_t)v | (uintptr_t)o) % 16 == 0 &&
                    (q_batch * esz) % 16 == 0 && (k_row * esz) % 16 == 0 && (k_batch * esz) % 16 == 0 &&
                    (v_row * esz) % 16 == 0 && (v_batch * esz) % 16 == 0 && (o_batch * esz) % 16 == 0,
                "mit_attention_decode: rows must be 16-B aligned");
  if (B <= 0 || H <= 0) return MIT_OK;
#define MIT_DECODE_LAUNCH(DH_)                                                                                       \
  DISPATCH_DT(dtype, hipLaunchKernelGGL((attn_decode_kernel<T, DH_>), dim3((unsigned)(B * H)), dim3(256), 0,          \
                                        (hipStream_t)stream, H, (const T*)q, q_batch, (const T*)k, k_row, k_batch,    \
                                        (const T*)v, v_row, v_batch, (T*)o, o_batch, Lk, pos, key_tokens, tok_batch, \
                                        pad_idx, scale))
  switch (Dh) {
    case 16: MIT_DECODE_LAUNCH(16); break;
    case 32: MIT_DECODE_LAUNCH(32); break;
    case 64: MIT_DECODE_LAUNCH(64); break;
    default: MIT_DECODE_LAUNCH(128); break;
  }
#undef MIT_DECODE_LAUNCH
  MIT_LAUNCH_CHECK("mit_attention_decode");
  return MIT_OK;
}

extern "C" int mit_kv_store(int dtype, long B, long n, const void* src, long s_batch, void* cache, long c_row,
                            long c_batch, const int64_t* pos, void* stream) {
  MIT_RECORD([=]() { return mit_kv_store(dtype, B, n, src, s_batch, cache, c_row, c_batch, pos, stream); });
  MIT_CHECK_ARG(src && cache && pos, "mit_kv_store: null pointer");
  if (B <= 0 || n <= 0) return MIT_OK;
  DISPATCH_DT(dtype, hipLaunchKernelGGL(kv_store_kernel<T>, dim3(grid_for(B * n)), dim3(256), 0, (hipStream_t)stream,
                                        B, n, (const T*)src, s_batch, (T*)cache, c_row, c_batch, pos));
  MIT_LAUNCH_CHECK("mit_kv_store");
  return MIT_OK;
}

extern "C" int mit_embed_decode(int dtype, long B, long d, const int64_t* ids, long ld_ids, const int64_t* pos,
                                const void* table, float scale, const float* pe, void* out, void* stream) {
  MIT_RECORD([=]() { return mit_embed_decode(dtype, B, d, ids, ld_ids, pos, table, scale, pe, out, stream); });
  MIT_CHECK_ARG(ids && pos && table && pe && out, "mit_embed_decode: null pointer");
  if (B <= 0) return MIT_OK;
  DISPATCH_DT(dtype, hipLaunchKernelGGL(embed_decode_kernel<T>, dim3(grid_for(B * d)), dim3(256), 0,
                                        (hipStream_t)stream, B, d, ids, ld_ids, pos, (const T*)table, scale, pe,
                                        (T*)out));
  MIT_LAUNCH_CHECK("mit_embed_decode");
  return MIT_OK;
}

extern "C" int mit_greedy_pick(long B, long V, const float* logits, long ld, int64_t* ids, long ld_ids,
                               const int64_t* pos, int64_t end_id, int64_t pad_id, int* finished, int* n_finished,
                               void* stream) {
  MIT_RECORD([=]() { return mit_greedy_pick(B, V, logits, ld, ids, ld_ids, pos, end_id, pad_id, finished, n_finished, stream); });
  MIT_CHECK_ARG(logits && ids && pos && finished && n_finished && ld >= V && V > 0, "mit_greedy_pick: bad arguments");
  if (B <= 0) return MIT_OK;
  hipLaunchKernelGGL(greedy_pick_kernel, dim3((unsigned)B), dim3(256), 0, (hipStream_t)stream, V, logits, ld, ids,
                     ld_ids, pos, end_id, pad_id, finished, n_finished);
  MIT_LAUNCH_CHECK("mit_greedy_pick");
  return MIT_OK;
}
