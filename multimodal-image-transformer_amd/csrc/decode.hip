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

// The same decode attention for d_model = H * DH = 512 with one 8-wave block per IMAGE: a wave
// instruction reads one whole 1-KiB key (or value) row -- lane l holds dims 8l .. 8l+7, i.e. head
// 8l / DH, and a head's score is reduced over its DH / 8 lanes -- so a block streams its image's K/V
// rows contiguously (the (b, h)-block kernel reads 128-B pieces of every row, 8 times per DRAM page)
// with U rows per wave in flight before the first use. Wave w takes keys w*U .. w*U+U-1 (+8U per
// iteration); the 8 waves' softmax states merge once in LDS.
// sum over the LPH (2 / 4 / 8 / 16) consecutive lanes of a head by DPP: quad_perm [1,0,3,2] and
// [2,3,0,1], then row_half_mirror (lane i <-> 7 - i: the other quad's sum) and row_mirror (i <-> 15 - i)
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, false));
}
template <int LPH>
__device__ __forceinline__ float head_sum(float v) {
  if constexpr (LPH >= 2) v += dpp_f<0xB1>(v);
  if constexpr (LPH >= 4) v += dpp_f<0x4E>(v);
  if constexpr (LPH >= 8) v += dpp_f<0x141>(v);
  if constexpr (LPH >= 16) v += dpp_f<0x140>(v);
  return v;
}

template <int DH, int U, bool NT>
__global__ __launch_bounds__(512) void attn_decode_rows_kernel(const bf16* __restrict__ q, long q_batch,
                                                               const bf16* __restrict__ k, long k_row, long k_batch,
                                                               const bf16* __restrict__ v, long v_row, long v_batch,
                                                               bf16* __restrict__ o, long o_batch, long lk_fixed,
                                                               const int64_t* __restrict__ pos,
                                                               const int64_t* __restrict__ key_tokens, long tok_batch,
                                                               int pad_idx, float scale) {
  constexpr int LPH = DH / 8;
  __shared__ float red[8][64][10];
  const long b = blockIdx.x;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const long Lk = pos ? (*pos + 1) : lk_fixed;
  float qv[8];
  load8<bf16>(q + b * q_batch + lane * 8, qv);
#pragma unroll
  for (int i = 0; i < 8; ++i) qv[i] *= scale * kLog2e;
  const bf16* kb = k + b * k_batch + lane * 8;
  const bf16* vb = v + b * v_batch + lane * 8;
  const int64_t* tb = key_tokens ? key_tokens + b * tok_batch : nullptr;
  float m = kNegBig, l = 0.f, acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  // the U keys of an iteration as ONE online-softmax block: the U scores are independent (dot products
  // and head reductions pipeline), one max / one rescale per block and one exp2 per key (was a dependent
  // max -> 2 exp2 -> rescale chain per key); head reductions over the LPH lanes by DPP within the row.
  // The next block's K / V rows are loaded before this block's math (two register buffers): one memory
  // round trip per wave instead of one per block (the cross-attention's 197 keys: 4 blocks per wave).
  // the key-padding tokens of a block are loaded with its K / V rows (vmcnt counts in order: a token
  // load issued after the next block's prefetch would wait for that prefetch too)
  auto load_blk = [&](long j0, bf16x8 (&kr)[U], bf16x8 (&vr)[U], int64_t (&tk)[U]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long j = j0 + u;
      if (j < Lk) {
        if constexpr (NT) {  // once-read stream: non-temporal, so it does not evict the weights from L2 / MALL
          kr[u] = __builtin_nontemporal_load((const bf16x8*)(kb + j * k_row));
          vr[u] = __builtin_nontemporal_load((const bf16x8*)(vb + j * v_row));
        } else {
          kr[u] = *(const bf16x8*)(kb + j * k_row);
          vr[u] = *(const bf16x8*)(vb + j * v_row);
        }
        tk[u] = tb ? tb[j] : 0;
      } else {
        kr[u] = vr[u] = bf16x8{};
        tk[u] = pad_idx;
      }
    }
  };
  auto math_blk = [&](long j0, const bf16x8 (&kr)[U], const bf16x8 (&vr)[U], const int64_t (&tk)[U]) {
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) ok[u] = j0 + u < Lk && (!tb || tk[u] != pad_idx);
    float s[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float t = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) t = fmaf(qv[i], (float)kr[u][i], t);
      s[u] = t;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) s[u] = head_sum<LPH>(s[u]);
    float bm = -INFINITY;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!ok[u]) s[u] = -INFINITY;
      bm = fmaxf(bm, s[u]);
    }
    const float mn = fmaxf(m, bm);
    const float corr = exp2f(m - mn);
    l *= corr;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] *= corr;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float p = exp2f(s[u] - mn);
      l += p;
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = fmaf(p, (float)vr[u][i], acc[i]);
    }
    m = mn;
  };
  bf16x8 ka[U], va[U], kb2[U], vb2[U];
  int64_t ta[U], tb2[U];
  long j0 = (long)w * U;
  if (j0 < Lk) load_blk(j0, ka, va, ta);
  while (j0 < Lk) {
    const long j1 = j0 + 8 * U;
    if (j1 < Lk) load_blk(j1, kb2, vb2, tb2);
    math_blk(j0, ka, va, ta);
    if (j1 >= Lk) break;
    const long j2 = j1 + 8 * U;
    if (j2 < Lk) load_blk(j2, ka, va, ta);
    math_blk(j1, kb2, vb2, tb2);
    j0 = j2;
  }
  float* mine = red[w][lane];
  mine[0] = m;
  mine[1] = l;
#pragma unroll
  for (int i = 0; i < 8; ++i) mine[2 + i] = acc[i];
  __syncthreads();
  if (w == 0) {
    for (int w2 = 1; w2 < 8; ++w2) merge(m, l, acc, red[w2][lane][0], red[w2][lane][1], &red[w2][lane][2]);
    float out[8];
    const float inv = 1.0f / l;  // all keys masked -> 0/0 = NaN, as the reference's softmax
#pragma unroll
    for (int i = 0; i < 8; ++i) out[i] = acc[i] * inv;
    store8<bf16>(o + b * o_batch + lane * 8, out);
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
                                                          const int64_t* pos, int64_t end_id,
                                                          int64_t pad_id, int* __restrict__ finished,
                                                          int* __restrict__ n_finished, int* __restrict__ ticket,
                                                          int64_t* pos_adv) {  // may alias pos: no __restrict__
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
  if ((V & 3) == 0 && (ld & 3) == 0 && ((uintptr_t)logits & 15) == 0) {
    // 16-B loads, 4 per thread in flight before the first compare (the scalar loop was one dependent
    // load round trip per 256 logits: 18 us for a 256 x 10000 step)
    const long nv = V >> 2;
    const f32x4* r4 = (const f32x4*)row;
    for (long i0 = threadIdx.x; i0 < nv; i0 += 4L * blockDim.x) {
      f32x4 x[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const long i = i0 + (long)u * blockDim.x;
        x[u] = i < nv ? r4[i] : f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const long j = 4 * (i0 + (long)u * blockDim.x) + t;
          if (j < V && better(x[u][t], j, best, bi)) {
            best = x[u][t];
            bi = j;
          }
        }
    }
  } else {
    for (long j = threadIdx.x; j < V; j += blockDim.x) {
      const float x = row[j];
      if (better(x, j, best, bi)) {
        best = x;
        bi = j;
      }
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
    // position advance folded in (was its own launch): every block has READ the old *pos before it
    // takes a ticket -- the vmcnt(0) below retires this block's load of *pos (and its ids store)
    // before the atomic issues, so the last ticket holder's write of the new position cannot
    // overtake any block's read of the old one
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (ticket && atomicAdd(ticket, 1) == (int)gridDim.x - 1) {
      *pos_adv = p + 1;
      *ticket = 0;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Decode-step GEMM with the post-LN residual blocks folded in (bf16 step only). The per-token step
// of the 6-layer decoder was 76 launches, 24 of them tiny (LayerNorm, kv_store, step_inc: 4-5 us
// each for ~0.5 MB of traffic). Here a LayerNorm is never its own launch:
//  * the PRODUCER of a pre-LN sum z = A W^T + b + residual writes z in f32 plus, per 64-column tile,
//    each row's (mean, M2) over those columns (Chan's parallel form: merged exactly, in a fixed order,
//    by the consumer -- no atomics, deterministic);
//  * a CONSUMER whose operand is LN(z) merges the row statistics and normalises z while staging its
//    64 A rows into LDS (a_stats != NULL), and a residual LN(z) is applied element-wise in the
//    epilogue (r_mode 2);
//  * the self-attention in_proj writes its K|V columns straight into the cache row at *pos.
// 64x64 output tile per 4-wave block; B fragments streamed from global one K-step ahead (as in
// gemm_rs_kernel), waves split K, partial tiles summed once in LDS.
// ------------------------------------------------------------------------------------------------
constexpr int DG_BK = 64;
constexpr int DG_RLD = 68;                          // fp32 row stride of a partial tile in LDS
constexpr uint32_t DG_OOB = 0x80000000u;

__device__ __forceinline__ int dg_xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, rr = nwg % 8, x = bid % 8, y = bid / 8;
  return (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + y;
}

// merge the per-64-column (mean, M2) partials of one row of width W -> (mean, rstd); all partial loads
// issued before the first use (W <= 64 * DG_PMAX)
constexpr int DG_PMAX = 16;
__device__ __forceinline__ void dg_row_stats(const float* __restrict__ st, long W, float eps, float& mean, float& rstd) {
  const int P = (int)((W + 63) / 64);
  f32x2 part[DG_PMAX];
#pragma unroll
  for (int p = 0; p < DG_PMAX; ++p) part[p] = p < P ? *(const f32x2*)(st + 2 * p) : f32x2{0.f, 0.f};
  float s = 0.f;
#pragma unroll
  for (int p = 0; p < DG_PMAX; ++p) s += part[p][0] * (float)max(0L, min(64L, W - 64L * p));
  mean = s / (float)W;
  float m2 = 0.f;
#pragma unroll
  for (int p = 0; p < DG_PMAX; ++p) {
    const float dm = part[p][0] - mean;
    m2 += part[p][1] + dm * dm * (float)max(0L, min(64L, W - 64L * p));
  }
  rstd = rsqrtf(m2 / (float)W + eps);
}

// NW waves split K; BMR x 64 output tile (BMR = 64, or 32 with 8 waves: half the fragment and
// accumulator registers, so two buffers of operands still fit 2 waves per SIMD)
template <int AMODE, int ACT, int RMODE, bool CF32, int NW, int BMR>
__global__ __launch_bounds__(NW * 64) void decode_gemm_kernel(mit_decode_gemm_args g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int FR = BMR / 16;                          // 16-row fragments per wave
  constexpr int TPR = 256 / BMR, CPT = 64 / TPR;        // epilogue (threads 0-255): threads per row, columns each
  const long M = g.M, N = g.N, K = g.K;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nbn = (int)((N + 63) / 64), nbm = (int)((M + BMR - 1) / BMR);
  // an XCD's blocks: every row block of consecutive column blocks, so each weight column block is
  // fetched by one XCD (the weights, not the B <= 256 activation rows, are the operand that matters;
  // row-major blocks had every XCD fetch every weight: 80 MB for the 10 MB head)
  const int bid = dg_xcd_remap(blockIdx.x, nbm * nbn);
  const int bm = bid % nbm, bn = bid / nbm;
  const long m0 = (long)bm * BMR, n0 = (long)bn * 64;
  const bool epi = tid < 256;
  const int b_bytes = (int)(2 * ((N - 1) * g.ldb + K));
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)g.B, (short)0, b_bytes, 0x00020000);
  const long brow = n0 + (lane & 15);
  const int kl = 8 * (lane >> 4);
  auto ldb8 = [&](long row, long k) -> bf16x8 {
    const uint32_t off = (row < N && k < K) ? (uint32_t)((row * g.ldb + k) * 2) : DG_OOB;
    return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rb, (int)off, 0, 0));
  };
  auto loadb = [&](int s, bf16x8 (&b)[4][2]) {
    const long k0 = (long)s * DG_BK + kl;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i) b[i][kk] = ldb8(brow + i * 16, k0 + kk * 32);
  };
  const int ns = (int)((K + DG_BK - 1) / DG_BK);
  bf16x8 b0[4][2], b1[4][2];
  int s = w;
  if (s < ns) loadb(s, b0);

  // epilogue operands first: none of them depends on the product, so their round trips overlap the
  // K loop instead of following it
  const int r = (tid & 255) / TPR, cq = (tid % TPR) * CPT;
  const long gr = m0 + r;
  const bool rok = epi && gr < M;
  float bias[CPT], res[CPT];
#pragma unroll
  for (int c = 0; c < CPT; ++c) bias[c] = res[c] = 0.f;
  if (g.bias && epi) {
#pragma unroll
    for (int c = 0; c < CPT; ++c) bias[c] = n0 + cq + c < N ? g.bias[n0 + cq + c] : 0.f;
  }
  if constexpr (RMODE == 1) {
    if (rok) {
#pragma unroll
      for (int h = 0; h < CPT; h += 8)
        if (n0 + cq + h < N) {
          const bf16x8 x = *(const bf16x8*)((const bf16*)g.r + gr * g.ldr + n0 + cq + h);
#pragma unroll
          for (int i = 0; i < 8; ++i) res[h + i] = (float)x[i];
        }
    }
  } else if constexpr (RMODE == 2) {
    if (rok) {
      const float* zr = (const float*)g.r + gr * g.ldr;
      f32x4 z[CPT / 4], ga[CPT / 4], be[CPT / 4];
#pragma unroll
      for (int c = 0; c < CPT; c += 4) {
        const long gc = n0 + cq + c;
        const bool ok = gc < N;
        z[c / 4] = ok ? *(const f32x4*)(zr + gc) : f32x4{};
        ga[c / 4] = ok ? *(const f32x4*)(g.r_gamma + gc) : f32x4{};
        be[c / 4] = ok ? *(const f32x4*)(g.r_beta + gc) : f32x4{};
      }
      float mu, rs;
      dg_row_stats(g.r_stats + gr * 2 * ((N + 63) / 64), N, g.eps, mu, rs);
#pragma unroll
      for (int c = 0; c < CPT; c += 4)
#pragma unroll
        for (int i = 0; i < 4; ++i) res[c + i] = (z[c / 4][i] - mu) * rs * ga[c / 4][i] + be[c / 4][i];
    }
  }
  const long p = g.cache ? *g.pos : 0;

  // A operand: bf16 rows straight from global (AMODE 0), or LN(z) rows staged in LDS (AMODE 1)
  const long alda = AMODE ? (K * 2 + 16) : 0;  // LDS row stride (bytes): 16-B pad -> conflict-free reads
  __amdgpu_buffer_rsrc_t ra;
  if constexpr (AMODE == 0) {
    const int a_bytes = (int)(2 * ((M - 1) * g.lda + K));
    ra = __builtin_amdgcn_make_buffer_rsrc((void*)g.A, (short)0, a_bytes, 0x00020000);
  } else {
    // wave w normalises rows RPW*w .. RPW*w+RPW-1 (RPW = BMR / NW: 16 with 4 waves x 64 rows, 4 with
    // 8 waves x 32 rows); lane l owns columns 8l .. 8l+7 (+512 per pass). The first pass's z loads go
    // out before the row statistics are merged (lanes 0 .. RPW-1 of the wave, one row each, shared by
    // shuffles): one round trip, not two
    constexpr int RPW = BMR / NW;
    static_assert(RPW * NW == BMR && RPW <= 16, "LN-operand staging: BMR / NW rows per wave");
    float mu_l = 0.f, rs_l = 0.f;
    if (lane < RPW && m0 + w * RPW + lane < M)
      dg_row_stats(g.a_stats + (m0 + w * RPW + lane) * 2 * ((K + 63) / 64), K, g.eps, mu_l, rs_l);
    for (long k = 8L * lane; k - 8L * lane < K; k += 512) {
      const bool kok = k < K;
      f32x4 z[RPW][2];
#pragma unroll
      for (int i = 0; i < RPW; ++i) {
        const int rr = w * RPW + i;
        if (kok && m0 + rr < M) {
          const float* zr = (const float*)g.A + (m0 + rr) * g.lda + k;
          z[i][0] = *(const f32x4*)zr;
          z[i][1] = *(const f32x4*)(zr + 4);
        } else {
          z[i][0] = z[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
      const f32x4 g0 = kok ? *(const f32x4*)(g.a_gamma + k) : f32x4{}, g1 = kok ? *(const f32x4*)(g.a_gamma + k + 4) : f32x4{};
      const f32x4 e0 = kok ? *(const f32x4*)(g.a_beta + k) : f32x4{}, e1 = kok ? *(const f32x4*)(g.a_beta + k + 4) : f32x4{};
#pragma unroll
      for (int i = 0; i < RPW; ++i) {
        const int rr = w * RPW + i;
        const float mu = __shfl(mu_l, i, 64), rs = __shfl(rs_l, i, 64);
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          o[j] = (bf16)((z[i][0][j] - mu) * rs * g0[j] + e0[j]);
          o[j + 4] = (bf16)((z[i][1][j] - mu) * rs * g1[j] + e1[j]);
        }
        if (kok) *(bf16x8*)(smem + rr * alda + k * 2) = o;
      }
    }
    __syncthreads();
  }
  auto loada = [&](int s, bf16x8 (&a)[FR][2]) {
    const long k0 = (long)s * DG_BK + kl;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < FR; ++i) {
        const long k = k0 + kk * 32;
        if constexpr (AMODE == 0) {
          const long row = m0 + i * 16 + (lane & 15);
          const uint32_t off = (row < M && k < K) ? (uint32_t)((row * g.lda + k) * 2) : DG_OOB;
          a[i][kk] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(ra, (int)off, 0, 0));
        } else {
          const int row = i * 16 + (lane & 15);
          a[i][kk] = k < K ? *(const bf16x8*)(smem + row * alda + k * 2) : bf16x8{};
        }
      }
  };

  f32x4 acc[FR][4];
#pragma unroll
  for (int i = 0; i < FR; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](bf16x8 (&a)[FR][2], bf16x8 (&b)[4][2]) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < FR; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][kk], b[j][kk], acc[i][j], 0, 0, 0);
  };
  {  // both operands one K-step ahead of the MFMAs (wave w: K-steps w, w+NW, ...)
    bf16x8 a0[FR][2], a1[FR][2];
    if (s < ns) loada(s, a0);
    for (; s < ns; s += 2 * NW) {
      if (s + NW < ns) {
        loada(s + NW, a1);
        loadb(s + NW, b1);
      }
      mma(a0, b0);
      if (s + NW >= ns) break;
      if (s + 2 * NW < ns) {
        loada(s + 2 * NW, a0);
        loadb(s + 2 * NW, b0);
      }
      mma(a1, b1);
    }
  }
  if constexpr (AMODE == 1) __syncthreads();  // the reduction below reuses the staged A's LDS

  float* red = (float*)smem;
  {
    float* mine = red + w * BMR * DG_RLD;
    const int gq = lane >> 4;
#pragma unroll
    for (int i = 0; i < FR; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t) mine[(i * 16 + gq * 4 + t) * DG_RLD + j * 16 + (lane & 15)] = acc[i][j][t];
  }
  __syncthreads();
  if (!epi) return;
  float v[CPT];
#pragma unroll
  for (int c = 0; c < CPT; c += 4) {
    f32x4 a = *(const f32x4*)(red + r * DG_RLD + cq + c);
#pragma unroll
    for (int q = 1; q < NW; ++q) a += *(const f32x4*)(red + (q * BMR + r) * DG_RLD + cq + c);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float x = a[i] + bias[c + i];
      if (ACT == MIT_ACT_RELU) x = fmaxf(x, 0.f);
      v[c + i] = x + res[c + i];
    }
  }
  if constexpr (RMODE == 3) {  // greedy pick folded in: the row's (value, first column) maximum of this tile
    uint64_t best = 0;
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const long gc = n0 + cq + c;
      const uint32_t u = __float_as_uint(v[c]);
      const uint32_t o = v[c] != v[c] ? 0xFFFFFFFFu : ((u & 0x80000000u) ? ~u : (u | 0x80000000u));
      const uint64_t k = ((uint64_t)o << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)gc);
      if (gc < N && k > best) best = k;
    }
#pragma unroll
    for (int x = 1; x < TPR; x <<= 1) {
      const uint64_t o = ((uint64_t)(uint32_t)__shfl_xor((int)(best >> 32), x, 64) << 32) |
                         (uint32_t)__shfl_xor((int)(uint32_t)best, x, 64);
      best = o > best ? o : best;
    }
    if (rok && (tid % TPR) == 0) atomicMax(g.argmax_keys + (bn % MIT_ARGMAX_SLOTS) * M + gr, (unsigned long long)best);
    return;
  }
  if (g.stats_out) {  // this tile's (mean, M2) per row over its valid columns; TPR lanes per row
    const int nv = (int)min(64L, N - n0);
    float sm = 0.f;
#pragma unroll
    for (int c = 0; c < CPT; ++c) sm += (cq + c < nv) ? v[c] : 0.f;
#pragma unroll
    for (int x = 1; x < TPR; x <<= 1) sm += __shfl_xor(sm, x, 64);
    const float mp = sm / (float)nv;
    float q2 = 0.f;
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
      const float dv = v[c] - mp;
      q2 += (cq + c < nv) ? dv * dv : 0.f;
    }
#pragma unroll
    for (int x = 1; x < TPR; x <<= 1) q2 += __shfl_xor(q2, x, 64);
    if (rok && (tid % TPR) == 0) {
      float* so = g.stats_out + (gr * nbn + bn) * 2;
      so[0] = mp;
      so[1] = q2;
    }
  }
  if (!rok) return;
#pragma unroll
  for (int h = 0; h < CPT; h += 8) {
    const long gc = n0 + cq + h;
    if (gc >= N) continue;
    const float* vv = v + h;
    if (g.C) {
      if constexpr (CF32) {
        float* o = (float*)g.C + gr * g.ldc + gc;
        *(f32x4*)o = f32x4{vv[0], vv[1], vv[2], vv[3]};
        *(f32x4*)(o + 4) = f32x4{vv[4], vv[5], vv[6], vv[7]};
      } else {
        bf16x8 o;
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] = (bf16)vv[i];
        *(bf16x8*)((bf16*)g.C + gr * g.ldc + gc) = o;
      }
    }
    if (g.z_out) {
      float* o = g.z_out + gr * g.ldz + gc;
      *(f32x4*)o = f32x4{vv[0], vv[1], vv[2], vv[3]};
      *(f32x4*)(o + 4) = f32x4{vv[4], vv[5], vv[6], vv[7]};
    }
    if (g.cache && gc >= g.kv_col0) {
      bf16x8 o;
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = (bf16)vv[i];
      *(bf16x8*)((bf16*)g.cache + gr * g.c_batch + p * g.c_row + (gc - g.kv_col0)) = o;
    }
  }
}

// out[m, :] = LN(z[m, :]) in bf16 from the producer's row statistics: the vocabulary head's operand
// (a 10000-column head re-staging LN rows per 64-column block cost 45 us; this + the 128 GEMM ~13)
__global__ __launch_bounds__(256) void decode_ln_kernel(long M, long W, const float* __restrict__ z, long ldz,
                                                        const float* __restrict__ stats, const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, float eps, bf16* __restrict__ out,
                                                        long ldo) {
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= M) return;
  float mu, rs;
  dg_row_stats(stats + r * 2 * ((W + 63) / 64), W, eps, mu, rs);
  for (long k = 8L * lane; k < W; k += 512) {
    const float* zr = z + r * ldz + k;
    const f32x4 z0 = *(const f32x4*)zr, z1 = *(const f32x4*)(zr + 4);
    const f32x4 g0 = *(const f32x4*)(gamma + k), g1 = *(const f32x4*)(gamma + k + 4);
    const f32x4 e0 = *(const f32x4*)(beta + k), e1 = *(const f32x4*)(beta + k + 4);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o[j] = (bf16)((z0[j] - mu) * rs * g0[j] + e0[j]);
      o[j + 4] = (bf16)((z1[j] - mu) * rs * g1[j] + e1[j]);
    }
    *(bf16x8*)(out + r * ldo + k) = o;
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
  if (dtype == MIT_BF16 && H * Dh == 512 && B < (1L << 31)) {
    // the cross-attention's fixed memory K/V (no position: 620 MB per cfg1 token step, far past the 256 MB
    // Infinity Cache) streams non-temporally, so the layers' weights and self-attention caches stay
    // cached between token steps: 371.8-372.6 k -> 383.3-383.8 k tokens/s (configs[4], one box)
    const bool nt = pos == nullptr;
#define MIT_ROWS_LAUNCH(DH_)                                                                                          \
  if (nt)                                                                                                             \
    hipLaunchKernelGGL((attn_decode_rows_kernel<DH_, 8, true>), dim3((unsigned)B), dim3(512), 0, (hipStream_t)stream, \
                       (const bf16*)q, q_batch, (const bf16*)k, k_row, k_batch, (const bf16*)v, v_row, v_batch,       \
                       (bf16*)o, o_batch, Lk, pos, key_tokens, tok_batch, pad_idx, scale);                            \
  else                                                                                                                \
    hipLaunchKernelGGL((attn_decode_rows_kernel<DH_, 8, false>), dim3((unsigned)B), dim3(512), 0,                     \
                       (hipStream_t)stream, (const bf16*)q, q_batch, (const bf16*)k, k_row, k_batch, (const bf16*)v,  \
                       v_row, v_batch, (bf16*)o, o_batch, Lk, pos, key_tokens, tok_batch, pad_idx, scale)
    switch (Dh) {
      case 16: MIT_ROWS_LAUNCH(16); break;
      case 32: MIT_ROWS_LAUNCH(32); break;
      case 64: MIT_ROWS_LAUNCH(64); break;
      default: MIT_ROWS_LAUNCH(128); break;
    }
#undef MIT_ROWS_LAUNCH
    MIT_LAUNCH_CHECK("mit_attention_decode");
    return MIT_OK;
  }
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
                     ld_ids, pos, end_id, pad_id, finished, n_finished, (int*)nullptr, (int64_t*)nullptr);
  MIT_LAUNCH_CHECK("mit_greedy_pick");
  return MIT_OK;
}

// one block: row b's pick from the largest of its head argmax slot keys, the keys reset, then *pos += 1 once
// every row has read the old position (the __syncthreads orders the block's reads before thread 0's write)
__global__ __launch_bounds__(1024) void greedy_pick_keys_kernel(long B, unsigned long long* __restrict__ keys,
                                                                int64_t* __restrict__ ids, long ld_ids, int64_t* pos,
                                                                int64_t end_id, int64_t pad_id, int* __restrict__ finished,
                                                                int* __restrict__ n_finished) {
  const long p = *pos;
  for (long b = threadIdx.x; b < B; b += blockDim.x) {
    unsigned long long k = 0ull;
#pragma unroll
    for (int sl = 0; sl < MIT_ARGMAX_SLOTS; ++sl) {
      const unsigned long long ks = keys[sl * B + b];
      k = ks > k ? ks : k;
    }
#pragma unroll
    for (int sl = 0; sl < MIT_ARGMAX_SLOTS; ++sl) keys[sl * B + b] = 0ull;
    const int64_t bi = (int64_t)(0xFFFFFFFFu - (uint32_t)k);
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
  __syncthreads();
  if (threadIdx.x == 0) *pos = p + 1;
}

extern "C" int mit_greedy_pick_keys(long B, unsigned long long* keys, int64_t* ids, long ld_ids, int64_t* pos,
                                    int64_t end_id, int64_t pad_id, int* finished, int* n_finished, void* stream) {
  MIT_RECORD([=]() { return mit_greedy_pick_keys(B, keys, ids, ld_ids, pos, end_id, pad_id, finished, n_finished, stream); });
  MIT_CHECK_ARG(keys && ids && pos && finished && n_finished, "mit_greedy_pick_keys: null pointer");
  MIT_CHECK_ARG(B > 0 && B < (1L << 30), "mit_greedy_pick_keys: B = %ld", B);
  hipLaunchKernelGGL(greedy_pick_keys_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, B, keys, ids, ld_ids, pos,
                     end_id, pad_id, finished, n_finished);
  MIT_LAUNCH_CHECK("mit_greedy_pick_keys");
  return MIT_OK;
}

extern "C" int mit_greedy_pick_advance(long B, long V, const float* logits, long ld, int64_t* ids, long ld_ids,
                                       int64_t* pos, int64_t end_id, int64_t pad_id, int* finished, int* n_finished,
                                       int* ticket, void* stream) {
  MIT_RECORD([=]() { return mit_greedy_pick_advance(B, V, logits, ld, ids, ld_ids, pos, end_id, pad_id, finished, n_finished, ticket, stream); });
  MIT_CHECK_ARG(logits && ids && pos && finished && n_finished && ticket && ld >= V && V > 0,
                "mit_greedy_pick_advance: bad arguments");
  MIT_CHECK_ARG(B > 0 && B < (1L << 30), "mit_greedy_pick_advance: B = %ld", B);
  hipLaunchKernelGGL(greedy_pick_kernel, dim3((unsigned)B), dim3(256), 0, (hipStream_t)stream, V, logits, ld, ids,
                     ld_ids, pos, end_id, pad_id, finished, n_finished, ticket, pos);
  MIT_LAUNCH_CHECK("mit_greedy_pick_advance");
  return MIT_OK;
}

namespace {
template <int AMODE, int ACT, int RMODE, bool CF32, int NW, int BMR>
int launch_decode_gemm_nw(const mit_decode_gemm_args* g, hipStream_t s) {
  const long nblk = ((g->M + BMR - 1) / BMR) * ((g->N + 63) / 64);
  const int red = NW * BMR * DG_RLD * 4;
  const int lds = AMODE ? (int)max((long)BMR * (g->K * 2 + 16), (long)red) : red;
  static int attr = 0;
  if (attr < lds) {
    (void)hipFuncSetAttribute((const void*)decode_gemm_kernel<AMODE, ACT, RMODE, CF32, NW, BMR>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr = lds;
  }
  hipLaunchKernelGGL((decode_gemm_kernel<AMODE, ACT, RMODE, CF32, NW, BMR>), dim3((unsigned)nblk), dim3(NW * 64), lds, s, *g);
  MIT_LAUNCH_CHECK("mit_decode_gemm");
  return MIT_OK;
}
// bf16 operand with K >= 512 (linear2 at K = d_ff, and since round 3 the K = 512 residual-LN GEMMs
// self-out / cross-out): 8 waves split K over 32 x 64 tiles (twice the blocks, a quarter of the K
// steps per wave: the K loop is one L2 round trip per step). Threshold K >= 512 vs 1024: 782 vs 824 us
// per token step at B = 256, interleaved on one box. The LN-operand GEMMs (in_proj, cross-q, linear1,
// head) on 8 waves x 32 rows as well (4 rows staged per wave): 782 -> 730 us per token step.
template <int AMODE, int ACT, int RMODE, bool CF32>
int launch_decode_gemm(const mit_decode_gemm_args* g, hipStream_t s) {
  // the vocabulary head (argmax epilogue, N = 10000): 4 waves x 64 rows, half the blocks of the 8-wave
  // form and each weight block read by 4 instead of 8 row blocks (with the column-major block order:
  // 700 -> 690 us per token step at B = 256)
  if (RMODE == 3) return launch_decode_gemm_nw<AMODE, ACT, RMODE, CF32, 4, 64>(g, s);
  if (AMODE != 0 || g->K >= 512) return launch_decode_gemm_nw<AMODE, ACT, RMODE, CF32, 8, 32>(g, s);
  return launch_decode_gemm_nw<AMODE, ACT, RMODE, CF32, 4, 64>(g, s);
}
}  // namespace

extern "C" int mit_decode_gemm(const mit_decode_gemm_args* g, void* stream) {
  MIT_CHECK_ARG(g != nullptr, "mit_decode_gemm: null args");
  MIT_RECORD([c = *g, stream]() { return mit_decode_gemm(&c, stream); });
  MIT_CHECK_ARG(g->M >= 0 && g->N > 0 && g->K > 0, "mit_decode_gemm: bad extents M=%ld N=%ld K=%ld", g->M, g->N, g->K);
  MIT_CHECK_ARG(g->A && g->B, "mit_decode_gemm: null operand");
  MIT_CHECK_ARG(g->C || g->z_out || g->argmax_keys, "mit_decode_gemm: no output");
  // N % 8: the 8-column output vectors; the argmax head writes no C (any vocabulary, columns >= N masked)
  MIT_CHECK_ARG(g->K % 8 == 0 && (g->N % 8 == 0 || g->argmax_keys) && g->ldb % 8 == 0 && g->lda >= g->K &&
                    g->ldb >= g->K,
                "mit_decode_gemm: K, N (unless argmax_keys), ldb must be multiples of 8 and lda/ldb >= K");
  MIT_CHECK_ARG(g->act == MIT_ACT_NONE || g->act == MIT_ACT_RELU, "mit_decode_gemm: act %d unsupported", g->act);
  MIT_CHECK_ARG(g->r_mode >= 0 && g->r_mode <= 2, "mit_decode_gemm: bad r_mode %d", g->r_mode);
  const bool lna = g->a_stats != nullptr;
  MIT_CHECK_ARG(!lna || (g->a_gamma && g->a_beta && g->K <= 64 * DG_PMAX && g->lda % 4 == 0),
                "mit_decode_gemm: LN operand needs gamma/beta, K <= 1024, lda % 4 == 0");
  MIT_CHECK_ARG(lna || g->lda % 8 == 0, "mit_decode_gemm: bf16 A needs lda % 8 == 0");
  MIT_CHECK_ARG(g->r_mode == 0 || (g->r && g->ldr >= g->N && g->ldr % 8 == 0), "mit_decode_gemm: bad residual");
  MIT_CHECK_ARG(g->r_mode != 2 || (g->r_stats && g->r_gamma && g->r_beta && g->N <= 64 * DG_PMAX),
                "mit_decode_gemm: LN residual needs stats and N <= 1024");
  MIT_CHECK_ARG(!g->C || (g->ldc >= g->N && g->ldc % 8 == 0), "mit_decode_gemm: bad ldc");
  MIT_CHECK_ARG(!g->z_out || (g->ldz >= g->N && g->ldz % 8 == 0), "mit_decode_gemm: bad ldz");
  MIT_CHECK_ARG(!g->cache || (g->pos && g->kv_col0 % 8 == 0 && g->c_row % 8 == 0 && g->c_batch % 8 == 0),
                "mit_decode_gemm: cache needs pos and 8-element aligned strides");
  MIT_CHECK_ARG(!g->stats_out || g->z_out, "mit_decode_gemm: stats_out needs z_out");
  MIT_CHECK_ARG(2 * ((g->N - 1) * g->ldb + g->K) < (1L << 31) && (lna || 2 * ((g->M - 1) * g->lda + g->K) < (1L << 31)),
                "mit_decode_gemm: operand spans >= 2 GiB");
  const uintptr_t al = (uintptr_t)g->A | (uintptr_t)g->B | (uintptr_t)g->C | (uintptr_t)g->z_out | (uintptr_t)g->r |
                       (uintptr_t)g->cache | (uintptr_t)g->a_gamma | (uintptr_t)g->a_beta | (uintptr_t)g->r_gamma |
                       (uintptr_t)g->r_beta;
  MIT_CHECK_ARG(al % 16 == 0, "mit_decode_gemm: pointers must be 16-B aligned");
  MIT_CHECK_ARG(!g->argmax_keys || (!lna && g->act == MIT_ACT_NONE && g->r_mode == 0 && !g->C && !g->z_out &&
                                     !g->cache && ((uintptr_t)g->argmax_keys % 8) == 0 && g->N < (1L << 32)),
                "mit_decode_gemm: argmax_keys needs bf16 A rows, no activation / residual / other output");
  if (g->M == 0) return MIT_OK;
  hipStream_t s = (hipStream_t)stream;
  if (g->argmax_keys) return launch_decode_gemm<0, MIT_ACT_NONE, 3, false>(g, s);
  const bool relu = g->act == MIT_ACT_RELU;
  if (g->c_f32) {
    MIT_CHECK_ARG(lna && !relu && g->r_mode == 0, "mit_decode_gemm: f32 C only for the LN-operand head GEMM");
    return launch_decode_gemm<1, MIT_ACT_NONE, 0, true>(g, s);
  }
  if (lna) {
    MIT_CHECK_ARG(g->r_mode == 0, "mit_decode_gemm: LN operand with a residual unsupported");
    return relu ? launch_decode_gemm<1, MIT_ACT_RELU, 0, false>(g, s) : launch_decode_gemm<1, MIT_ACT_NONE, 0, false>(g, s);
  }
  MIT_CHECK_ARG(!relu || g->r_mode == 0, "mit_decode_gemm: ReLU with a residual unsupported");
  if (relu) return launch_decode_gemm<0, MIT_ACT_RELU, 0, false>(g, s);
  switch (g->r_mode) {
    case 1: return launch_decode_gemm<0, MIT_ACT_NONE, 1, false>(g, s);
    case 2: return launch_decode_gemm<0, MIT_ACT_NONE, 2, false>(g, s);
    default: return launch_decode_gemm<0, MIT_ACT_NONE, 0, false>(g, s);
  }
}

extern "C" int mit_decode_layernorm(long M, long W, const float* z, long ldz, const float* stats, const float* gamma,
                                    const float* beta, float eps, void* out, long ldo, void* stream) {
  MIT_RECORD([=]() { return mit_decode_layernorm(M, W, z, ldz, stats, gamma, beta, eps, out, ldo, stream); });
  MIT_CHECK_ARG(z && stats && gamma && beta && out, "mit_decode_layernorm: null pointer");
  MIT_CHECK_ARG(W > 0 && W % 8 == 0 && W <= 64 * DG_PMAX && ldz >= W && ldo >= W && ldz % 4 == 0 && ldo % 8 == 0,
                "mit_decode_layernorm: bad extents W=%ld ldz=%ld ldo=%ld", W, ldz, ldo);
  MIT_CHECK_ARG((((uintptr_t)z | (uintptr_t)gamma | (uintptr_t)beta | (uintptr_t)out) % 16) == 0,
                "mit_decode_layernorm: pointers must be 16-B aligned");
  if (M <= 0) return MIT_OK;
  hipLaunchKernelGGL(decode_ln_kernel, dim3((unsigned)((M + 3) / 4)), dim3(256), 0, (hipStream_t)stream, M, W, z, ldz,
                     stats, gamma, beta, eps, (bf16*)out, ldo);
  MIT_LAUNCH_CHECK("mit_decode_layernorm");
  return MIT_OK;
}
